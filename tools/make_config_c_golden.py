"""Oracle outputs of the association replay on BASELINE configs[3]'s stream at the config's
scale: the first 200 frames of the 1000-frame Config C stream (tools/synth.assoc_stream_config_c:
64 objects x 2000 map points, 16 classes, 8 detections per frame), flag EAO.

    python tools/make_config_c_golden.py   ->  tests/golden/replay_config_c_200.npz

Stored as tools/make_fr3_golden.py stores the fr3 streams: every detection's row, the final
object records, the CRC of each object's sorted map-point ids, the input digest; and the largest
cloud an isolation forest ran on (the replay's clouds reach the config's ~2000 points)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
from tools import synth  # noqa: E402
from make_fr3_golden import point_crcs, replay_oracle, stream_digest  # noqa: E402

N_STREAM, N_FRAMES = 1000, 200


def main():
    fr = synth.assoc_stream_config_c(N_STREAM)[:N_FRAMES]
    t0 = time.time()
    det, ints, fl, pts = replay_oracle(fr, "EAO")
    out = os.path.join(ROOT, "tests", "golden", "replay_config_c_200.npz")
    np.savez_compressed(out, det_out=det, obj_ints=ints, obj_floats=fl, obj_pts_crc=point_crcs(pts),
                        obj_pts_len=np.array([len(p) for p in pts], np.int32), digest=stream_digest(fr),
                        n_frames=np.int32(len(fr)), n_stream=np.int32(N_STREAM), flag=np.bytes_("EAO"))
    print("%s: %d frames, %d detections, %d objects, largest cloud %d points, oracle %.1f s"
          % (out, len(fr), len(det), len(ints), ints[:, 4].max(), time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
