"""Association GPU chain per frame from a rocprofv3 --kernel-trace SQLite database (development aid).

python tools/chain_trace.py <run_results.db>
For every frame start (k_rects_np) it lists the kernels that ran on the association
streams since the previous frame start, and summarises per frame: busy time of the
association kernels, the forest chains (k_stage -> k_iforest_tree -> k_iforest_sum
[-> k_np_pairs]) with their launch gaps, and the frame period."""
import collections
import re
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, stream_id, grid_x, grid_y from kernels order by start").fetchall()
K = [(re.sub(r"<.*$", "", n.split('(')[0].replace("eao::", "").replace("void ", "")), s, e, st, gx, gy) for n, s, e, st, gx, gy in rows]
ASSOC = {"k_stage", "k_iforest_tree", "k_iforest_sum", "k_np_pairs", "k_rects_np", "k_pack_masks", "k_rects"}
A = [k for k in K if k[0] in ASSOC]
fs = [i for i, k in enumerate(A) if k[0] == "k_rects_np"]
print("assoc dispatches %d, frame starts %d" % (len(A), len(fs)))
per = collections.defaultdict(list)
period, busy, nforest, chain = [], [], [], []
for a, b in zip(fs[:-1], fs[1:]):
    seg = A[a:b]
    t0, t1 = A[a][1], A[b][1]
    period.append((t1 - t0) / 1e3)
    iv = sorted((s, e) for _, s, e, *_ in seg)
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    busy.append(tot / 1e3)
    for n, s, e, st, gx, gy in seg:
        per[n].append((e - s) / 1e3)
    trees = [k for k in seg if k[0] == "k_iforest_tree"]
    nforest.append(len(trees))
    # stage start -> last kernel of that stream's chain end, per forest batch
    for j, k in enumerate(seg):
        if k[0] != "k_stage":
            continue
        st = k[3]
        tail = [x for x in seg[j + 1:] if x[3] == st]
        end = k[2]
        for x in tail:
            if x[0] in ("k_stage", "k_rects_np"):
                break
            end = x[2]
        chain.append((end - k[1]) / 1e3)
P = np.array(period[len(period) // 10:])
print("frame period: med %.1f mean %.1f us | assoc GPU busy per frame med %.1f mean %.1f us | forest launches/frame %.2f"
      % (np.median(P), P.mean(), np.median(busy), np.mean(busy), np.mean(nforest)))
print("forest chain (stage start -> chain end): med %.1f mean %.1f p90 %.1f us" %
      (np.median(chain), np.mean(chain), np.percentile(chain, 90)))
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    print("  %-16s n=%5d avg %6.1f med %6.1f p90 %6.1f max %7.1f us" % (n, len(v), v.mean(), np.median(v),
                                                                       np.percentile(v, 90), v.max()))
# launch gaps inside one stream's forest chain
gaps = collections.defaultdict(list)
for x, y in zip(A[:-1], A[1:]):
    pass
bys = collections.defaultdict(list)
for k in A:
    bys[k[3]].append(k)
for st, L in bys.items():
    for x, y in zip(L[:-1], L[1:]):
        if y[1] - x[2] < 200000:  # same burst (< 200 us apart)
            gaps[x[0] + "->" + y[0]].append((y[1] - x[2]) / 1e3)
for kname, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:10]:
    v = np.array(v)
    print("  gap %-34s n=%5d med %6.1f mean %6.1f us" % (kname, len(v), np.median(v), v.mean()))
