"""Host events of the association replay (EAO_REPLAY_TRACE) against the GPU kernel trace of the
same run (rocprofv3 --kernel-trace SQLite), both on the steady clock (development aid).

python tools/replay_timeline.py <trace.bin> [<run_results.db>]
Host events: 1 frame begin, 2 frame-start launch, 3 frame-start done, 4 association loop end,
5 forest batch launch (slot, clouds, max n), 6/7 forest wait begin/end (slot, phase),
8/9 local mapping begin/end. The last replay pass in the file is analysed."""
import collections
import re
import sqlite3
import sys

import numpy as np

ev = np.fromfile(sys.argv[1], dtype=np.dtype([("t", "<i8"), ("ev", "<i4"), ("a", "<i4"), ("b", "<i4"),
                                               ("c", "<i4")]))
# passes: the frame ids restart
fr = np.nonzero(ev["ev"] == 1)[0]
starts = [fr[0]] + [fr[i] for i in range(1, len(fr)) if ev["a"][fr[i]] <= ev["a"][fr[i - 1]]]
ev = ev[starts[-1]:]
t = ev["t"].astype(np.float64) / 1e3  # us
E = ev["ev"]
print("events %d, frames %d, span %.1f ms" % (len(ev), int((E == 1).sum()), (t[-1] - t[0]) / 1e3))
# per-frame host phases
seg = collections.defaultdict(list)
fi = np.nonzero(E == 1)[0]
for a, b in zip(fi[:-1], fi[1:]):
    loc = {}
    for k in range(a, b):
        loc.setdefault(int(E[k]), t[k])
    t0 = t[a]
    order = [(1, "F"), (2, "fs_launch"), (3, "fs_done"), (4, "loop_end"), (8, "lm_begin"), (9, "lm_end")]
    prev = t0
    for e, name in order[1:]:
        if e in loc:
            seg[name].append(loc[e] - prev)
            prev = loc[e]
    seg["to_next_frame"].append(t[b] - prev)
    seg["period"].append(t[b] - t0)
    w = [(t[k2], int(E[k2]), int(ev["b"][k2])) for k2 in range(a, b) if E[k2] in (6, 7)]
    tot = collections.defaultdict(float)
    for (ta, ea, pa), (tb, eb, pb) in zip(w[:-1], w[1:]):
        if ea == 6 and eb == 7:
            tot[pa] += tb - ta
    for ph, v in tot.items():
        seg["forest_wait_phase%d" % ph].append(v)
    seg["launches"].append(sum(1 for k2 in range(a, b) if E[k2] == 5))
print("per frame (us, median / mean over %d frames):" % len(seg["period"]))
for k, v in seg.items():
    v = np.array(v, np.float64)
    n = len(seg["period"])
    print("  %-22s med %7.1f mean %7.1f  (per frame: %7.1f)" % (k, np.median(v), v.mean(), v.sum() / n))
if len(sys.argv) < 3:
    sys.exit(0)
c = sqlite3.connect(sys.argv[2])
rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
K = [(re.sub(r"<.*$", "", n.split('(')[0].replace("eao::", "").replace("void ", "")), s / 1e3, e / 1e3, st) for n, s, e, st in rows]
K = [k for k in K if t[0] - 1000 <= k[1] <= t[-1] + 1000]
rn = [k for k in K if k[0] == "k_rects_np"]
fs = np.nonzero(E == 2)[0]
done = np.nonzero(E == 3)[0]
print("kernels in the window %d, frame-start kernels %d, host frame starts %d" % (len(K), len(rn), len(fs)))
if rn and len(rn) == len(fs):
    d_start = np.array([k[1] - t[i] for k, i in zip(rn, fs)])
    d_dur = np.array([k[2] - k[1] for k in rn])
    d_seen = np.array([t[j] - k[2] for k, j in zip(rn, done)]) if len(done) == len(rn) else None
    print("frame start: kernel start - launch event med %.1f mean %.1f | duration med %.1f | host sees it "
          "done after kernel end: med %.1f us" % (np.median(d_start), d_start.mean(), np.median(d_dur),
                                                   np.median(d_seen) if d_seen is not None else -1))
    # what the frame-start kernel waited for: the last forest kernel ending before it starts
    tree = [k for k in K if k[0] in ("k_iforest_sum", "k_np_pairs", "k_iforest_tree")]
    tree_end = np.array([k[2] for k in tree])
    waited, tail = [], []
    for k, i in zip(rn, fs):
        j = np.searchsorted(tree_end, k[1] + 0.5) - 1
        if j >= 0 and k[1] - tree_end[j] < 15:
            waited.append(k[1] - t[i])
            tail.append(tree_end[j] - t[i])
    print("frame starts queued behind a forest chain: %d of %d; forest chain ends med %.1f us after the launch event"
          % (len(waited), len(rn), np.median(tail) if tail else -1))
st = [k for k in K if k[0] == "k_stage"]
fl = np.nonzero(E == 5)[0]
if len(st) == len(fl):
    tr_ = [k for k in K if k[0] == "k_iforest_tree"]
    a = np.array([k[1] - t[i] for k, i in zip(st, fl)])
    dur = np.array([k[2] - k[1] for k in tr_])
    print("forest batches %d: stage start - launch event med %.1f | tree med %.1f mean %.1f p90 %.1f us"
          % (len(st), np.median(a), np.median(dur), dur.mean(), np.percentile(dur, 90)))
    # the batch's chain on its stream: k_stage -> k_iforest_tree -> k_iforest_sum (+ speculative NP)
    by_stream = collections.defaultdict(list)
    for k in K:
        by_stream[k[3]].append(k)
    parts = []
    for s0 in st:
        q = by_stream[s0[3]]
        i = q.index(s0)
        if i + 2 < len(q) and q[i + 1][0] == "k_iforest_tree" and q[i + 2][0] == "k_iforest_sum":
            t1, t2 = q[i + 1], q[i + 2]
            parts.append((s0[2] - s0[1], t1[1] - s0[2], t1[2] - t1[1], t2[1] - t1[2], t2[2] - t2[1], t2[2] - s0[1]))
    if parts:
        P = np.array(parts)
        print("forest chain (med / mean us): stage %.1f / %.1f | gap %.1f / %.1f | tree %.1f / %.1f | gap %.1f / %.1f"
              " | sum %.1f / %.1f | stage start -> sum end %.1f / %.1f"
              % tuple(v for c in range(6) for v in (np.median(P[:, c]), P[:, c].mean())))
    mx = ev["c"][fl]
    for lo, hi in ((0, 130), (130, 200), (200, 400), (400, 800), (800, 1600), (1600, 99999)):
        m = (mx >= lo) & (mx < hi)
        if m.any():
            print("   max n in [%4d, %5d): %4d batches, tree med %.1f us" % (lo, hi, m.sum(), np.median(dur[m])))
else:
    print("forest launches %d vs k_stage dispatches %d: not matched" % (len(fl), len(st)))
