"""Runs tests/test_replay_host.py's scenarios on a sanitizer build of the host harness, in a
process started by tests/test_replay_sanitizers.py with the sanitizer runtime preloaded (no
subprocess is started from here: a preloaded runtime would follow it into make / g++).
usage: san_driver.py <harness .so> <scenario>...   Prints "SAN DRIVER OK" at the end."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "eao-slam_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pyoracle as orc  # noqa: E402
import test_replay_host as T  # noqa: E402


def main():
    so, scen = sys.argv[1], sys.argv[2:]
    orc.lib()
    H = ctypes.CDLL(so)
    H.harness_assoc_create.restype = ctypes.c_void_p
    runs = {
        "fr3": lambda: T.test_host_fr3_real_stream_matches_oracle(H, "Full"),
        "updates": lambda: T.test_host_point_updates_match_oracle(H, "EAO"),
        "run_updates": lambda: T.test_host_run_updates_matches_oracle(H),
        "stream": lambda: T.test_host_run_stream_matches_oracle(H),
        "flags": lambda: [T.test_host_orchestration_matches_oracle(H, f, l)
                          for f, l in [("NP", False), ("IoU", False), ("EAO", True)]],
        "threads": lambda: T.test_host_two_threads_share_one_handle(H),
    }
    for s in scen:
        runs[s]()
        print("scenario", s, "ok", flush=True)
    print("SAN DRIVER OK", flush=True)


if __name__ == "__main__":
    main()
