"""How predictable is the number of generator draws a subtree of IsolationTree::Build takes?
(development aid for a speculative parallel tree build). CPU simulation of Node::Build's draw
sequence (isolation_forest.h:165-224: a Lemire-3 dimension draw, then a canonical-float split
draw when min != max; leaves by count or depth take none) over Gaussian clouds, libstdc++'s
mt19937 through numpy's legacy MT19937 seeding.

  (1) how often a left subtree takes exactly 2 (cl - 1) draws (a full split down to single
      items: the depth limit does not bind), by left size;
  (2) for fixed (items, depth, max depth), how many distinct draw counts occur and how much of
      the mass the 1 / 4 / 8 / 16 most frequent ones hold."""
import collections
import sys

import numpy as np

sys.setrecursionlimit(10000)


class Rng:
    def __init__(self, seed):
        self.bg = np.random.MT19937(0)
        self.bg._legacy_seeding(seed)
        self.buf = []

    def raw(self):
        if not self.buf:
            self.buf = list(self.bg.random_raw(1024).astype(np.uint64)[::-1])
        return int(self.buf.pop())


def draws(rng, X, idx, depth, maxd, stats=None):
    n = len(idx)
    if n <= 1 or depth >= maxd:
        return 0
    while True:  # uniform_int_distribution<uint32_t>(0, 2): Lemire
        prod = rng.raw() * 3
        if (prod & 0xffffffff) >= 3 or (prod & 0xffffffff) >= (2 ** 32 - 3) % 3:
            break
    dim = prod >> 32
    v = X[idx, dim]
    mn, mx = v.min(), v.max()
    if mn == mx:
        return 1
    r = np.float32(rng.raw() * 2.0 ** -32)
    split = np.float32(np.float32(r * np.float32(mx - mn)) + mn)
    L, R = idx[v < split], idx[v >= split]
    if len(L) == 0:
        return 2
    cl = draws(rng, X, L, depth + 1, maxd, stats)
    if stats is not None:
        stats.append((len(L), cl == 2 * (len(L) - 1)))
    return 2 + cl + draws(rng, X, R, depth + 1, maxd, stats)


def main():
    rs = np.random.default_rng(1)
    out = collections.defaultdict(lambda: [0, 0])
    for n in (150, 300, 600, 1200):
        for trial in range(2):
            X = rs.normal(0, 0.1, (n, 3)).astype(np.float32)
            psi = n // 2
            maxd = int(np.ceil(np.log2(psi)))
            for t in range(50):
                st = []
                draws(Rng(1000 * trial + t), X, rs.choice(n, psi, replace=False), 0, maxd, st)
                for cl, ok in st:
                    key = (n, "cl<=8" if cl <= 8 else "cl<=32" if cl <= 32 else "cl<=64" if cl <= 64 else "cl>64")
                    out[key][0] += 1
                    out[key][1] += ok
    print("(1) left subtrees taking exactly 2 (cl - 1) draws")
    for k in sorted(out):
        print("  cloud %5d %-7s nodes %6d  exact %.2f" % (k + (out[k][0], out[k][1] / out[k][0])))
    print("(2) draw counts of one subtree at fixed (items, depth, max depth), 3000 samples")
    for cl, d, maxd in ((12, 5, 9), (24, 5, 9), (24, 3, 9), (48, 4, 9), (48, 6, 10)):
        c = collections.Counter()
        for t in range(3000):
            X = rs.normal(0, 0.1, (cl, 3)).astype(np.float32)
            c[draws(Rng(t), X, np.arange(cl), d, maxd)] += 1
        top = [v for _, v in c.most_common(16)]
        print("  items %2d depth %d max %2d: %2d distinct, top1 %.2f top4 %.2f top8 %.2f top16 %.2f"
              % (cl, d, maxd, len(c), top[0] / 3000, sum(top[:4]) / 3000, sum(top[:8]) / 3000,
                 sum(top[:16]) / 3000))


if __name__ == "__main__":
    main()
