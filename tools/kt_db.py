"""Per-kernel summary of a rocprofv3 results.db (the SQLite output of --kernel-trace): calls, mean /
median duration in us, grid and LDS, for development comparisons.
  python tools/kt_db.py gpurun_out/<dir>/run_results.db [name-filter]"""
import sqlite3
import sys

import numpy as np

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select name, duration, grid_x, grid_y, lds_size from kernels").fetchall()
by = {}
for n, d, gx, gy, lds in rows:
    if flt and flt not in n:
        continue
    k = (n.split("(")[0][:48], gx, gy, lds)
    by.setdefault(k, []).append(d / 1e3)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print("%-48s grid %6d x %-4d lds %6d  n=%5d mean %8.1f us  median %8.1f us" % (k[0], k[1], k[2], k[3], len(v),
                                                                             np.mean(v), np.median(v)))
