"""Per-dispatch durations of one kernel from a rocprofv3 kernel trace (development aid): grouped by
grid size, median / mean us, in dispatch order of the first occurrence.

python3 tools/kt_levels.py <kernel_trace.csv> <kernel-name-substring>"""
import collections
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if sys.argv[2] in r["Kernel_Name"]]
g = collections.OrderedDict()
for r in sel:
    key = (r["Grid_Size_X"], r["Grid_Size_Y"], r.get("Workgroup_Size_X", ""))
    g.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in g.items():
    v = np.array(v)
    tot += np.median(v)
    print("grid %s x %s (wg %s): %4d dispatches, median %.1f us, mean %.1f us" % (k[0], k[1], k[2], len(v), np.median(v), v.mean()))
print("sum of medians %.1f us" % tot)
