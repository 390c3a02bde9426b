"""The independent pure-Python restatement of the association (oracle/assoc_py.py, written from
Object.cc / Tracking.cc / LocalMapping.cc / isolation_forest.h, not from assoc_ref.cpp) run over
the WHOLE fr3 streams the GPU parity fixtures cover:

    python tools/make_assoc_py_golden.py [demo|full|configc]  ->  tests/golden/replay_fr3_demo_eao_py.npz
                                                                  tests/golden/replay_fr3_full_py.npz
                                                                  tests/golden/replay_config_c_200_py.npz

Same record as tools/make_fr3_golden.py (every detection's row, final object records, point-set
CRCs, input digest). tests/test_oracle_assoc_py.py then requires these to equal the C++ oracle's
fixtures that the engine is tested against -- two independent restatements agreeing over all
405 EAO frames and all 2582 Full frames. Pure Python: minutes for the demo stream, tens of
minutes for the Full one, hence fixtures."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
import assoc_py as ap  # noqa: E402
from make_fr3_golden import point_crcs, stream_digest  # noqa: E402
from tools import synth  # noqa: E402

STREAMS = {"demo": ("replay_fr3_demo_eao_py.npz", None, None, "EAO"),
           "full": ("replay_fr3_full_py.npz", 0, 2582, "Full"),
           # BASELINE configs[3] at its scale (64 objects x 2000 points): the 200 frames of
           # tools/make_config_c_golden.py -- NP subsampling at n > 3m (Object.cc:780-789) and
           # forests over clouds of >= 1500 points (Object.cc:1202-1309)
           "configc": ("replay_config_c_200_py.npz", None, None, "EAO")}


def stream(key):
    if key == "configc":
        return synth.assoc_stream_config_c(1000)[:200]
    _, start, n, _ = STREAMS[key]
    return synth.assoc_stream_fr3_real(start, n)


def main():
    which = sys.argv[1:] or list(STREAMS)
    for key in which:
        name, _, _, flag = STREAMS[key]
        fr = stream(key)
        t0 = time.time()
        p = ap.Replay(flag)
        outs = []
        for t, f in enumerate(fr):
            outs.append(p.step(t + 1, f))
            if (t + 1) % 100 == 0:
                print("%s: frame %d, %.0f s" % (key, t + 1, time.time() - t0), flush=True)
        ints, fl, pts = p.objects()
        out = os.path.join(ROOT, "tests", "golden", name)
        np.savez_compressed(out, det_out=np.concatenate(outs), obj_ints=ints, obj_floats=fl,
                            obj_pts_crc=point_crcs(pts), obj_pts_len=np.array([len(q) for q in pts], np.int32),
                            digest=stream_digest(fr), n_frames=np.int32(len(fr)), flag=np.bytes_(flag))
        print("%s: %d frames, %d objects, %.0f s -> %s" % (key, len(fr), len(ints), time.time() - t0, out), flush=True)


if __name__ == "__main__":
    main()
