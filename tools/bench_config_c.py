"""Config C (SURVEY.md §8d input 4, §8e): the object-sharded association.

Kept as a shortcut: it is `bench.py --config c` (see bench.run_config_c).

  python tools/bench_config_c.py [--frames 1000] [--gpus N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if __name__ == "__main__":
    sys.exit(__import__("subprocess").call([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c"] +
                                           sys.argv[1:]))
