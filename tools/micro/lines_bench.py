"""Line stage of the bench workload (405 colour frames 640x480, as bench.py builds them): mean ms
per eao_lines_detect_color_batch_device over 10 launches, and the lines of every frame hashed so
two builds (EAO_ACCEL_LIB) can be compared; with --check the first frames against the oracle.
Development aid."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

F, W, H, LCAP = 405, 640, 480, 512
dev = torch.device("cuda", 0)
rendered, _ = synth.frame_stream(F, seed=0xEA0, structure=True)
d_render = torch.from_numpy(rendered).to(dev)
yy, xx = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
tb = (14 * torch.sin(xx.float() / 37.0)).round().to(torch.int16)
tr = (11 * torch.cos(yy.float() / 29.0 + xx.float() / 83.0)).round().to(torch.int16)
g16 = d_render.to(torch.int16)
d_color = torch.stack([(g16 + tb).clamp(0, 255), g16, (g16 - tr).clamp(0, 255)], -1).to(torch.uint8).contiguous()
lines = ea.Lines(W, H, max_batch=F)
d_lines = torch.zeros((F, LCAP, 6), dtype=torch.float32, device=dev)
d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ms = []
for it in range(12):
    e0.record(s)
    lines.detect_color_batch_device(d_color.data_ptr(), F, 3 * W, 3, 50.0, d_lines.data_ptr(), d_cnt.data_ptr(), LCAP,
                                    s.cuda_stream)
    e1.record(s)
    s.synchronize()
    if it >= 2:
        ms.append(e0.elapsed_time(e1))
cnt = d_cnt.cpu().numpy()
out = d_lines.cpu().numpy()
h = hashlib.sha256()
for f in range(F):
    h.update(out[f, :max(cnt[f], 0)].tobytes())
h.update(cnt.tobytes())
print("lib %s: line stage %.3f ms per %d frames (min %.3f), mean lines %.2f, digest %s" % (
    os.path.basename(os.path.dirname(ea.LIB_PATH)), float(np.mean(ms)), F, float(np.min(ms)), float(cnt.mean()),
    h.hexdigest()[:16]), flush=True)
if "--check" in sys.argv:
    from oracle import pyoracle as orc  # the checker (development aid only)
    col = d_color[:8].cpu().numpy()
    bad = [f for f in range(8) if not np.array_equal(out[f, :cnt[f]], orc.edlines_color(col[f]))]
    print("oracle check of 8 frames: mismatches", bad, flush=True)
