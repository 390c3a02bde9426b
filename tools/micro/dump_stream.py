"""Dump the bench's association stream (fr3 shape) for tools/micro/replay_driver."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools import synth  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stream.bin"
kind = sys.argv[2] if len(sys.argv) > 2 else "fr3"
nfr = int(sys.argv[3]) if len(sys.argv) > 3 else (405 if kind == "fr3" else 1000)
fr = synth.assoc_stream_fr3(nfr) if kind == "fr3" else synth.assoc_stream_config_c(nfr)
with open(out, "wb") as f:
    np.array([len(fr)], np.int32).tofile(f)
    for t in fr:
        np.array([len(t["boxes"]), len(t["ids"]), int(t["kf"])], np.int32).tofile(f)
        for k, dt in (("T", np.float32), ("boxes", np.int32), ("ids", np.int32), ("pos", np.float32),
                      ("uv", np.float32), ("bad", np.uint8)):
            np.ascontiguousarray(t[k], dt).tofile(f)
