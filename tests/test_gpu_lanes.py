"""The association's HSA launch lanes (eao-slam_amd/csrc/hsa_lane.cpp) on the GPU.

eao_lane_selftest drives three lanes with barrier packets gated by host signals:
  * a completion marker held across four full reuses of its signal slot (4 x 64 later records of
    its lane) reads complete and makes a wait on it a no-op (round-5 review: a held marker used to
    alias the slot's later launch);
  * a barrier written for a use that completes while the barrier is still held has its dependency
    cleared when the slot is reused; a committed one delays the reuse until it has retired (counted
    on its lane's retire signal: under rocprofv3 the queue's read index counts forwarded packets);
  * 6000 runs of 1..7 held packets + a record, so runs meet the ring end at many alignments (each
    run that would wrap is committed in two parts: the host SIGSEGV of round 5 under rocprofv3).
The replay tests (test_gpu_replay.py, test_gpu_fr3.py) run the same lanes on the association."""
import pytest

import eao_accel as ea

pytestmark = pytest.mark.gpu


def test_lane_selftest():
    n = ea.lane_selftest(0)
    assert n > 6000 * 2, n


def test_lane_selftest_repeats_on_fresh_lanes():
    # lanes opened and closed within one process, as pooled replays on several engines do
    for _ in range(3):
        ea.lane_selftest(0)
