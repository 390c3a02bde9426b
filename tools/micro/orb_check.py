"""Batched GPU extraction vs the oracle over a whole synthetic stream
(development aid): prints the frames whose keypoints/descriptors differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python"), os.path.join(ROOT, "oracle")]
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 405
W, H, NF = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (640, 480, 1000)
fr, _ = synth.frame_stream(F, w=W, h=H)
dev = torch.device("cuda", 0)
orb = ea.Orb(NF, 1.2, 8, 20, 7, W, H, max_batch=F)
cap = orb.cap
d_fr = torch.from_numpy(np.stack(fr)).to(dev)
kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.zeros(F, dtype=torch.int32, device=dev)
orb.extract_batch_device(d_fr.data_ptr(), F, W, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap, None)
torch.cuda.synchronize()
n = cnt.cpu().numpy()
hk = kps.cpu().numpy().view(ea.KP_DTYPE).reshape(F, cap)
hd = desc.cpu().numpy()
bad = []
for t in range(F):
    ok, od = orc.extract(fr[t], NF, 1.2, 8)
    if not (n[t] == len(ok) and np.array_equal(hk[t, :n[t]], ok) and np.array_equal(hd[t, :n[t]], od)):
        g = hk[t, :n[t]]
        lv = [(l, int((g["octave"] == l).sum()), int((ok["octave"] == l).sum())) for l in range(8)]
        lv = [x for x in lv if x[1] != x[2] or not np.array_equal(g[g["octave"] == x[0]], ok[ok["octave"] == x[0]])]
        bad.append((t, int(n[t]), len(ok), lv))
print("frames %d mismatching %d %s" % (F, len(bad), bad[:10]), flush=True)
