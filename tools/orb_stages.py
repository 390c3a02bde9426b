"""Per-stage extraction times (HIP events on the extraction stream) of the batched ORB
extraction, for A/B work on the extraction kernels: Config A (640x480, 1000 features,
405 frames) and Config B (1920x1080, 4000 features, 256 frames)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import torch  # noqa: E402
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
out = {}
for name, (W, H, NF, F) in {"a": (640, 480, 1000, 405), "b": (1920, 1080, 4000, 256)}.items():
    frames, _ = synth.frame_stream(F, W, H)
    d_frames = torch.from_numpy(np.stack(frames)).to(dev)
    orb = ea.Orb(NF, 1.2, 8, 20, 7, W, H, max_batch=F)
    cap = orb.cap
    kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    orb.set_timing(True)
    st = []
    for r in range(a.reps + 2):
        orb.extract_batch_device(d_frames.data_ptr(), F, W, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap,
                                 s.cuda_stream)
        s.synchronize()
        if r >= 2:
            st.append(orb.stage_ms())
    m = np.median(np.stack(st), 0)
    out[name] = dict(stages_ms=[round(float(x), 4) for x in m], total_ms=round(float(m.sum()), 4),
                     keypoints_per_frame=round(float(cnt.float().mean().item()), 1))
    print(name, json.dumps(out[name]), flush=True)
print(json.dumps(out))
