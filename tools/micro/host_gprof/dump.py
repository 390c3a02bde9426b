"""Dump the packed fr3 association stream (EAO, or Full with `full`) as raw arrays for main.cpp."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

full = "full" in sys.argv
frames = synth.assoc_stream_fr3_real(0, 2582) if full else synth.assoc_stream_fr3_real()
pk = ea.Replay.pack(frames)
out = sys.argv[-1]
with open(out, "wb") as f:
    np.array([pk["n"], int(pk["nb"].sum()), int(pk["npt"].sum()), 1 if full else 0], np.int32).tofile(f)
    for k in ("ids", "T", "nb", "boxes", "npt", "mp", "pos", "uv", "bad", "kf"):
        np.ascontiguousarray(pk[k]).tofile(f)
    nl = np.array([len(l) for l in pk["lines"]], np.int32)
    nl.tofile(f)
    np.ascontiguousarray(np.concatenate([np.asarray(l, np.float32).reshape(-1, 4) for l in pk["lines"]])).tofile(f)
print("frames", pk["n"], "boxes", int(pk["nb"].sum()), "points", int(pk["npt"].sum()), "lines", int(nl.sum()))
