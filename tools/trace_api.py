"""Host-API / copy / kernel timeline around the frame-start launches of a rocprofv3
--kernel-trace --hip-trace --memory-copy-trace database (development aid).

python tools/trace_api.py <run_results.db> [--schema]"""
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
if "--schema" in sys.argv:
    for (n,) in c.execute("select name from sqlite_master where type in ('table','view')"):
        cols = [r[1] for r in c.execute("pragma table_info('%s')" % n)]
        print(n, cols)
    sys.exit(0)
k = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
k = [(n.split('(')[0], s, e, st) for n, s, e, st in k]
m = c.execute("select start, end, size from memory_copies order by start").fetchall()
a = c.execute("select name, start, end from regions where category like '%HIP%' order by start").fetchall()
print("kernels %d copies %d api %d" % (len(k), len(m), len(a)))
names = {}
for n, s, e in a:
    names.setdefault(n, []).append(e - s)
for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1]))[:14]:
    v = np.array(v)
    print("  %-34s n=%6d avg %6.1f us tot %7.1f ms" % (n[:34], len(v), v.mean() / 1e3, v.sum() / 1e6))
if m:
    d = np.array([(e - s) for s, e, _ in m])
    print("copies: avg %.1f us med %.1f" % (d.mean() / 1e3, np.median(d) / 1e3))
# frame starts: the k_rects kernel; the hipMemcpyAsync issued last before it on the host
mc = [(s, e) for n, s, e in a if n.startswith("hipMemcpyAsync") or n.startswith("hipLaunchKernel")]
ev = [(s, e) for n, s, e in a if n.startswith("hipEventSynchronize") or n.startswith("hipEventQuery")]
rows = []
import bisect
ms = [s for s, _ in mc]
cs = [s for s, _, _ in m]
for i, (n, s, e, st) in enumerate(k):
    if n != "eao::k_rects":
        continue
    j = bisect.bisect_left(ms, s) - 3  # stage, rects, np: the first of the three launches
    if j < 0:
        continue
    api_s, api_e = mc[j]
    q = bisect.bisect_left(cs, api_s)
    cp = m[q] if q < len(m) else None
    npe = next((e2 for n2, s2, e2, st2 in k[i + 1:] if st2 == st and n2 == "eao::k_np_pairs"), e)
    rows.append(((api_e - api_s) / 1e3, ((cp[0] - api_s) / 1e3) if cp else -1, ((cp[1] - cp[0]) / 1e3) if cp else -1,
                 (s - api_s) / 1e3, (npe - api_s) / 1e3))
r = np.array(rows[len(rows) // 3:])
print("frame starts %d (medians, us from the staging call): api %.1f | copy start %.1f dur %.1f | "
      "rects start %.1f | NP end %.1f" % (len(r), *np.median(r, 0)))
