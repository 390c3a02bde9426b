"""k_fast stage time for the bench workload (405 frames), development aid:
prints the five extraction stage times (ms) of the batched path."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 405
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (640, 480)
NF = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
fr, _ = synth.frame_stream(F, w=W, h=H)
dev = torch.device("cuda", 0)
orb = ea.Orb(NF, 1.2, 8, 20, 7, W, H, max_batch=F)
cap = orb.cap
d_fr = torch.from_numpy(np.stack(fr)).to(dev)
kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros(F, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
orb.set_timing(True)
acc = []
for it in range(6):
    orb.extract_batch_device(d_fr.data_ptr(), F, W, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap, s.cuda_stream)
    torch.cuda.synchronize()
    if it:
        acc.append(orb.stage_ms())
m = np.mean(np.array(acc), 0)
print("ablate=%s stages(ms) pyramid %.3f fast %.3f distribute %.3f blur %.3f describe %.3f | kps/frame %.1f" %
      ((os.environ.get("EAO_FAST_ABLATE", "0"),) + tuple(m) + (cnt.float().mean().item(),)), flush=True)
