"""Per-stage extraction time of the bench workload (405 frames 640x480, or a Config B
batch with args F W H NF), development aid: eao_orb_stage_ms averaged over 10 launches."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 405
W, H, NF = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (640, 480, 1000)
# the EAO bench's frames have office-like straight structure (bench.py); STRUCT=0: the plain
# procedural texture of Config B and the PMC extract
fr, _ = synth.frame_stream(min(F, 64) if W > 640 else F, w=W, h=H, structure=os.environ.get("STRUCT", "1") != "0")
fr = np.stack([fr[i % len(fr)] for i in range(F)])
dev = torch.device("cuda", 0)
orb = ea.Orb(NF, 1.2, 8, 20, 7, W, H, max_batch=F)
cap = orb.cap
d_fr = torch.from_numpy(fr).to(dev)
kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros(F, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
orb.set_timing(True)
st = []
for it in range(12):
    orb.extract_batch_device(d_fr.data_ptr(), F, W, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap, s.cuda_stream)
    s.synchronize()
    if it >= 2:
        st.append(orb.stage_ms())
m = np.mean(np.stack(st), 0)
print("frames %d %dx%d: " % (F, W, H) + " ".join("%s %.3f" % (k, v) for k, v in
      zip(["pyramid", "fast", "distribute", "describe"], m)) + " | total %.3f ms" % m.sum(), flush=True)
