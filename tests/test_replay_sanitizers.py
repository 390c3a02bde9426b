"""Sanitizer builds of the engine's host orchestration (replay.cpp through the host harness of
tests/native): AddressSanitizer + UndefinedBehaviorSanitizer over the fr3 / point-record /
stream / flag scenarios, ThreadSanitizer over the two-thread (Tracking + LocalMapping) handle
test. The scenarios are tests/test_replay_host.py's own, each also checked against the oracle.

The sanitizer runtime is preloaded into a child Python (tests/native/san_driver.py) that starts
no further process. Skipped when LD_PRELOAD is already set (a preload of the environment's own is
left alone)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def san_builds():
    if os.environ.get("LD_PRELOAD"):
        pytest.skip("LD_PRELOAD is set by the environment")
    subprocess.check_call(["make", "-s", "-C", os.path.join(os.path.dirname(HERE), "oracle")])
    subprocess.check_call(["make", "-s", "-C", NATIVE, "all", "san"])
    return os.path.join(NATIVE, "_build")


def _drive(so, runtime, env_opts, scenarios, timeout):
    rt = _runtime(runtime)
    if rt is None:
        pytest.skip(runtime + " not found")
    env = dict(os.environ, LD_PRELOAD=rt, **env_opts)
    p = subprocess.run([sys.executable, os.path.join(NATIVE, "san_driver.py"), so] + scenarios, env=env,
                       capture_output=True, text=True, timeout=timeout)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "SAN DRIVER OK" in p.stdout, out[-4000:]
    for s in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer"):
        assert s not in out, out[-4000:]


def test_asan_ubsan_host_orchestration(san_builds):
    _drive(os.path.join(san_builds, "libreplay_host_asan.so"), "libasan.so",
           dict(ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"),
           ["fr3", "updates", "run_updates", "stream", "flags", "threads"], 900)


def test_tsan_two_threads_one_handle(san_builds):
    _drive(os.path.join(san_builds, "libreplay_host_tsan.so"), "libtsan.so",
           dict(TSAN_OPTIONS="halt_on_error=1"), ["threads", "run_updates"], 900)
