"""Association dispatches that ran long inside a traced step, and what ran beside them.
  python tools/kt_outliers.py gpurun_out/<dir>/run_kernel_trace.csv [threshold_us]
For each association kernel (k_rects_np, k_np_pairs, k_iforest_*, k_publish): count, median, p99,
max; then every dispatch over the threshold with the other kernels overlapping it (name, overlap us).
Development aid (round-5 review, Weak 5: association dispatches stalled behind the line stage)."""
import csv
import sys

import numpy as np

path = sys.argv[1]
th = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
rows = []
for r in csv.DictReader(open(path)):
    rows.append((r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort(key=lambda x: x[1])
ASSOC = ("k_rects_np", "k_np_pairs", "k_iforest", "k_publish", "k_stage")
by = {}
for n, s, e in rows:
    if any(a in n for a in ASSOC):
        by.setdefault(n, []).append((e - s) / 1e3)
for n, v in sorted(by.items()):
    v = np.array(v)
    print("%-40s n=%5d median %7.1f p99 %7.1f max %8.1f us, over %g us: %d" % (n, len(v), np.median(v), np.percentile(v, 99),
                                                                           v.max(), th, (v > th).sum()))
print("-- dispatches over %g us and the kernels beside them" % th)
for n, s, e in rows:
    if not any(a in n for a in ASSOC) or (e - s) / 1e3 <= th:
        continue
    beside = {}
    for m, s2, e2 in rows:
        if (m, s2, e2) == (n, s, e) or e2 <= s or s2 >= e:
            continue
        beside[m] = beside.get(m, 0) + (min(e, e2) - max(s, s2)) / 1e3
    top = sorted(beside.items(), key=lambda kv: -kv[1])[:4]
    print("%-32s %8.1f us at %.3f ms | %s" % (n, (e - s) / 1e3, (s - rows[0][1]) / 1e6,
                                             ", ".join("%s %.0f" % (k.split("::")[-1], v) for k, v in top)))
