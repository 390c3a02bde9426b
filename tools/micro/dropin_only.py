"""The bench's per-frame drop-in leg alone (bench.dropin_leg: both passes, every frame checked
against the oracle) on the bench's own inputs -- development aid for the single-frame paths.
  python tools/micro/dropin_only.py [frames]   (EAO_ACCEL_LIB selects a library build)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "eao-slam_amd", "python")]
import torch  # noqa: E402,F401  (HIP runtime first, as the bench)
import bench  # noqa: E402
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 405
torch.cuda.is_available()
frames = synth.assoc_stream_fr3_real()[:F]
rendered, rposes = synth.frame_stream(F, seed=0xEA0, structure=True)
W, H = bench.W, bench.H
yy, xx = np.mgrid[0:H, 0:W]
tb = np.rint(14 * np.sin(xx.astype(np.float32) / 37.0)).astype(np.int16)
tr = np.rint(11 * np.cos(yy.astype(np.float32) / 29.0 + xx.astype(np.float32) / 83.0)).astype(np.int16)
color = np.stack([np.stack([np.clip(r.astype(np.int16) + tb, 0, 255), r.astype(np.int16),
                            np.clip(r.astype(np.int16) - tr, 0, 255)], -1).astype(np.uint8) for r in rendered])
gray = np.stack([orc.color_to_gray(c, rgb=True) for c in color])
res = bench.dropin_leg(ea, 0, frames, color, gray, rposes.astype(np.float32), "EAO", check=True)
print(json.dumps(res, default=float), flush=True)
