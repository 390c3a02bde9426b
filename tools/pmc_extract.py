"""Extraction-only workload for rocprofv3 counter passes: the batched ORB
extraction of bench.py's 405-frame stream, run --reps times (no association,
no matching), so per-dispatch PMC values of the ORB kernels are isolated.

  rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d OUT -o run -- python3 tools/pmc_extract.py
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import torch  # noqa: E402
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=None)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--config", choices=["eao", "b"], default="eao",
                help="eao: 640x480, 1000 features (configs[1]); b: 1920x1080, 4000 features (configs[4])")
a = ap.parse_args()
W, H, NF = (640, 480, 1000) if a.config == "eao" else (1920, 1080, 4000)
a.frames = a.frames or (405 if a.config == "eao" else 256)
frames, _ = synth.frame_stream(a.frames, W, H)
dev = torch.device("cuda", 0)
d_frames = torch.from_numpy(np.stack(frames)).to(dev)
orb = ea.Orb(NF, 1.2, 8, 20, 7, W, H, max_batch=a.frames)
cap = orb.cap
kps = torch.zeros((a.frames, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.zeros((a.frames, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros(a.frames, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
for _ in range(a.reps):
    orb.extract_batch_device(d_frames.data_ptr(), a.frames, W, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(),
                             cap, s.cuda_stream)
torch.cuda.synchronize()
print("keypoints/frame %.1f" % cnt.float().mean().item())
