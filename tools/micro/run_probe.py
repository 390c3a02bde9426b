"""Association replay timing from Python (development aid): eao_replay_run
over the bench stream, optionally with torch's HIP runtime brought up first."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
if "torch" in sys.argv:
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda")
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

packed = ea.Replay.pack(synth.assoc_stream_fr3(405))
a = ea.Assoc()
for rep in range(4):
    rp = ea.Replay(a, "EAO")
    t0 = time.perf_counter()
    rp.run(packed)
    dt = time.perf_counter() - t0
    print("%s rep %d: %.1f ms" % ("torch" if "torch" in sys.argv else "plain", rep, dt * 1e3), flush=True)
    rp.close()
