import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "eao-slam_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    # torch (device buffers for the batched-path tests) must bring up its HIP
    # runtime before the engine library's: initialise it first when GPU tests run
    if "not gpu" not in (config.getoption("markexpr", "") or ""):
        try:
            import torch
            torch.cuda.is_available()
        except Exception:
            pass


@pytest.fixture(scope="session")
def frames():
    from tools import synth
    fr, poses = synth.frame_stream(4)
    return fr, poses
