"""The association kernels' embedded code object and its argument table (eao-slam_amd/gen_co.py,
csrc/hsa_lane.cpp): the kernels the HSA launch lanes dispatch are present with the explicit
arguments the host passes, and the COV5 hidden arguments lie past them. CPU-only (the table is
generated at build time from the code object's AMDGPU metadata)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "eao-slam_amd", "lib", "gen")
LIB = os.path.join(ROOT, "eao-slam_amd", "lib", "libeao_accel.so")

# kernel (demangled prefix, as hsa_kernel_id looks it up) -> explicit argument count
LANE_KERNELS = {
    "eao::k_rects_np(": 22,
    "eao::k_np_pairs(": 12,
    "eao::k_stage(": 3,
    "eao::k_iforest_sum(": 14,  # + the packed outlier masks' outputs (sharded replays)
    "eao::k_publish(": 4,
    "void eao::k_iforest_tree<64>(": 16,
    "void eao::k_iforest_tree<1024>(": 16,
}


def _rows():
    path = os.path.join(GEN, "assoc_co_meta.inc")
    if not os.path.exists(path):
        pytest.skip("engine not built (make -C eao-slam_amd)")
    rows = []
    for line in open(path):
        m = re.match(r'\s*\{"(.*?)", "(.*?)", (\d+), (\d+), (\d+), (\d+), \{(.*?)\}, \{(.*?)\}, \{(.*?)\}\},', line)
        if m:
            rows.append(dict(name=m.group(1), sym=m.group(2), karg=int(m.group(3)), nargs=int(m.group(6)),
                             off=[int(x) for x in m.group(7).split(",")], size=[int(x) for x in m.group(8).split(",")],
                             hidden=[int(x) for x in m.group(9).split(",")]))
    return rows


def test_lane_kernels_in_table():
    rows = _rows()
    for prefix, nargs in LANE_KERNELS.items():
        hit = [r for r in rows if r["name"].startswith(prefix)]
        assert len(hit) == 1, prefix
        r = hit[0]
        assert r["nargs"] == nargs and r["sym"].endswith(".kd"), (prefix, r)
        end = max(o + s for o, s in zip(r["off"], r["size"]))
        assert end <= r["karg"] <= 512, (prefix, end, r["karg"])
        hid = [h for h in r["hidden"] if h >= 0]
        assert all(h >= end for h in hid), (prefix, r["hidden"])  # hidden arguments follow the explicit ones
        assert r["hidden"][3] >= 0, prefix  # group size x: every lane kernel reads blockDim


def test_code_object_embedded():
    if not os.path.exists(LIB):
        pytest.skip("engine not built")
    syms = subprocess.check_output(["nm", "-D", LIB], text=True)
    assert re.search(r"\beao_assoc_co\b", syms) and re.search(r"\beao_assoc_co_end\b", syms)
    co = os.path.join(GEN, "assoc.co")
    with open(co, "rb") as f:
        assert f.read(4) == b"\x7fELF"
