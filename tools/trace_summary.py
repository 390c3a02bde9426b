"""Per-kernel duration summary of a rocprofv3 --kernel-trace SQLite output (development aid).

python tools/trace_summary.py <run_results.db> [--gaps]"""
import collections
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, stream_id, grid_y from kernels order by start").fetchall()
d = collections.defaultdict(list)
for n, s, e, st, gy in rows:
    d[n.split('(')[0] + ("@%d" % st if "--by-stream" in sys.argv else "")].append(e - s)
print("%d dispatches, span %.1f ms" % (len(rows), (rows[-1][2] - rows[0][1]) / 1e6 if rows else 0))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    print("%-36s n=%5d avg %7.1f us med %7.1f p90 %7.1f max %7.1f tot %8.2f ms"
          % (k[:36], len(v), v.mean() / 1e3, np.median(v) / 1e3, np.percentile(v, 90) / 1e3, v.max() / 1e3,
             v.sum() / 1e6))
if "--gaps" in sys.argv:  # GPU busy fraction: union of kernel intervals over the span
    iv = sorted((s, e) for _, s, e, _, _ in rows)
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print("busy %.1f ms of %.1f ms" % (busy / 1e6, (iv[-1][1] - iv[0][0]) / 1e6))
if "--timeline" in sys.argv:  # a window of dispatches: start offset, duration, gap after the previous end
    k = int(sys.argv[sys.argv.index("--timeline") + 1])
    w = rows[len(rows) // 2:len(rows) // 2 + k]
    t0, pe = w[0][1], w[0][1]
    for n, s, e, st, gy in w:
        print("%9.1f us  dur %7.1f  gap %7.1f  stream %d  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - pe) / 1e3, st,
                                                                n.split('(')[0][:40]))
        pe = max(pe, e)
