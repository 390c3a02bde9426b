"""Oracle outputs of the association replay on the reference's fr3_long_office inputs.

    python tools/make_fr3_golden.py   ->  tests/golden/replay_fr3_demo_eao.npz
                                          tests/golden/replay_fr3_full.npz

The streams come from tools/synth.assoc_stream_fr3_real over tests/golden/fr3_inputs.npz
(the real YOLO boxes and GT poses, see tools/make_fr3_inputs.py):
  * demo: rgb_seq_pose.txt's 405 frames, flag EAO (BASELINE configs[1]);
  * full: rgb_full_demo.txt's 2582 frames, flag Full (BASELINE configs[2]).
The oracle (oracle/, CPU restatement) replays each one frame by frame with LocalMapping's
object maintenance at the stream's keyframes.  Stored: every detection's
(method, object id, class, points) row, the final object records (ints, floats) and a
CRC32 of each object's sorted map-point id set, plus a digest of the generated inputs so a
test can tell a generator change from an engine mismatch.  The full stream takes about a
minute of oracle time, too long for the GPU test to recompute -- hence the fixture.
"""
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
STREAMS = {"replay_fr3_demo_eao.npz": (None, None, "EAO"), "replay_fr3_full.npz": (0, 2582, "Full")}


def stream_digest(frames):
    h = 0
    for f in frames:
        for k in ("T", "boxes", "ids", "pos", "uv", "bad", "lines"):
            if k in f:  # (streams without line sets: Config C)
                h = zlib.crc32(np.ascontiguousarray(f[k]).tobytes(), h)
        h = zlib.crc32(bytes([1 if f["kf"] else 0]), h)
    return np.uint32(h)


def point_crcs(pts):
    return np.array([zlib.crc32(np.sort(p).astype(np.int32).tobytes()) for p in pts], np.uint32)


def replay_oracle(frames, flag):
    r = orc.Replay(flag)
    outs = []
    for t, f in enumerate(frames):
        outs.append(r.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            r.local_mapping()
    ints, fl, pts = r.objects()
    return np.concatenate(outs), ints, fl, pts


def main():
    for name, (start, n, flag) in STREAMS.items():
        fr = synth.assoc_stream_fr3_real(start, n)
        t0 = time.time()
        det, ints, fl, pts = replay_oracle(fr, flag)
        np.savez_compressed(os.path.join(OUT, name), det_out=det, obj_ints=ints, obj_floats=fl,
                            obj_pts_crc=point_crcs(pts), obj_pts_len=np.array([len(p) for p in pts], np.int32),
                            digest=stream_digest(fr), n_frames=np.int32(len(fr)), flag=np.bytes_(flag))
        print("%s: %d frames, %d detections, %d objects, oracle %.1f s" % (name, len(fr), len(det), len(ints),
                                                                           time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
