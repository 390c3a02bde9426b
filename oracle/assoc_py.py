"""assoc_py.py -- a second, independent CPU restatement of the EAO object association
(TEST INFRASTRUCTURE ONLY: imported by tests/ alone, never by the product).

Written in Python straight from the reference text, not from oracle/assoc_ref.cpp, so that a
misreading of Object.cc shared by the C++ oracle and the product cannot pass unnoticed
(tests/test_oracle_assoc_py.py runs both on the same streams). Same replay model as the oracle
(SURVEY.md appendix B): one call per frame with Tcw, the YOLO boxes in file order (score 0,
Q1), the tracked map points in keypoint order (id, world position, undistorted keypoint, bad
flag) and the frame's line segments; LocalMapping's object maintenance runs when the caller
says a keyframe was inserted; LocalMapping's map-point changes arrive as point records.

What it restates, with the reference lines each part follows:
  * Tracking object section, src/Tracking.cc:1243-1696 (steps 1-10), AssociateObjAndPoints
    :2434-2468, AssociateObjAndLines :2472-2527, InitObjMap :2531-2598, SampleObjYaw and
    WorldToImg :2600-2862, std::sort(VIC) :64-68,2849;
  * Object_2D, src/Object.cc:63-158 (frame mean / boxplot), ObjectDataAssociation :162-710,
    NoParaDataAssociation :714-930;
  * Object_Map, src/Object.cc:967-1198 (ComputeMeanAndStandard), :1202-1309 (iForest
    erase), :1313-1554 (DataAssociateUpdate), :1558-1603 (ComputeProjectRectFrame),
    :1607-2178 (merges, overlap), :2193-2248 (UpdateObjPose);
  * LocalMapping object maintenance, src/LocalMapping.cc:86-92,772-882;
  * include/isolation_forest.h (whole) with libstdc++ (GCC 11) mt19937, uniform_int /
    uniform_real / generate_canonical and std::shuffle; src/detect_3d_cuboid/
    object_3d_util.cpp:176-208,349-434 and matrix_utils.cpp:201-205 (line merge);
  * src/Converter.cc:28-38,101-107,193-212; g2o SE3Quat (ctor + normalizeRotation, inverse,
    operator*), Eigen Quaternion(Matrix3) and _transformVector.

Number semantics follow the C++ types: float expressions in numpy float32 (one rounding per
operation, no contraction, Q27), double ones in Python floats; float overloads of sin / cos /
atan2 / sqrt are glibc's sinf / cosf / atan2f (ctypes) and sqrtf (= correctly rounded), Q23 /
Q26. The quirks shared with the oracle are the documented SURVEY §8c definitions: Q1, Q4
(int32 wrap), Q6, Q7 (out_point false), Q8 (erase stops after the last outlier), Q10 (frame
merge dead), Q11 (Rect truncation, cvRound in contains), Q12 (3x3 gemm: float accumulate,
then (float)((double)t + c)), Q22 (duplicate test by exact equality), Q24, Q29 (size()-2 of a
one-frame object reads the front). cv::Mat aliasing is kept: the map object's mCenter3D
shares its buffer with its first Object_2D's _Pos (Object.cc:679, Tracking.cc:2566), so
ComputeMeanAndStandard's in-place `mCenter3D = sum / n` rewrites that observation too.
"""
import ctypes
import math
import os

import numpy as np

F = np.float32
F64 = np.float64
INT_MIN = -2147483648
M64 = (1 << 64) - 1

_m = ctypes.CDLL("libm.so.6")
for _n, _a in (("sinf", 1), ("cosf", 1), ("atan2f", 2)):
    getattr(_m, _n).restype = ctypes.c_float
    getattr(_m, _n).argtypes = [ctypes.c_float] * _a


def sinf(x):
    return F(_m.sinf(float(x)))


def cosf(x):
    return F(_m.cosf(float(x)))


def atan2f(y, x):
    return F(_m.atan2f(float(y), float(x)))


def sqrtf(x):
    return np.sqrt(F(x))


def smax(a, b):  # std::max: (a < b) ? b : a
    return b if a < b else a


def smin(a, b):  # std::min: (b < a) ? b : a
    return b if b < a else a


def i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def cdiv(a, b):  # C integer division (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def trunc_i32(f):
    """(int)float: truncation; x86 cvttss2si gives INT_MIN for NaN / out of range (Q11)."""
    f = float(f)
    if not math.isfinite(f) or f >= 2147483648.0 or f <= -2147483649.0:
        return INT_MIN
    return int(f)


def cv_round(f):
    """cvRound(float): round half to even (SSE2 cvtss2si), Q11 / Q25."""
    f = float(f)
    if not math.isfinite(f) or abs(f) >= 2147483648.0:
        return INT_MIN
    return int(np.rint(f))


def u64(v):
    return v & M64


def fdiv(a, b):
    with np.errstate(all="ignore"):
        return F(F(a) / F(b))


# ---------------------------------------------------------------------------
# libstdc++ (GCC 11) random engines and distributions, <random> / <bits/uniform_int_dist.h>
class MT19937:
    """std::mt19937: init_genrand seeding, 624-word twist, tempering."""

    def __init__(self, seed):
        # init_genrand: x[i] = 1812433253 * (x[i-1] ^ (x[i-1] >> 30)) + i. numpy's legacy
        # RandomState seeds an int the same way (its state is used as the 624 words only).
        self.mt = np.random.RandomState(seed & 0xFFFFFFFF).get_state()[1].astype(np.uint64)
        self.buf = []
        self.i = 624
        self.next = self._stream().__next__  # g.next() == g(), without the method call

    def _stream(self):
        while True:
            self._gen()
            yield from self.buf

    def _gen(self):
        old = self.mt
        new = old.copy()
        U, L, A = np.uint64(0x80000000), np.uint64(0x7FFFFFFF), np.uint64(0x9908B0DF)

        def step(k0, k1, src):
            y = (new[k0:k1] & U) | (old[k0 + 1:k1 + 1] & L)
            new[k0:k1] = src ^ (y >> np.uint64(1)) ^ np.where(y & np.uint64(1), A, np.uint64(0))

        step(0, 227, old[397:624])          # mt[k + 397] not yet updated
        step(227, 454, new[0:227])          # mt[k - 227] updated above
        step(454, 623, new[227:396])
        y = (new[623] & U) | (new[0] & L)
        new[623] = new[396] ^ (y >> np.uint64(1)) ^ (A if int(y) & 1 else np.uint64(0))
        self.mt = new
        y = new.copy()
        y ^= y >> np.uint64(11)
        y ^= (y << np.uint64(7)) & np.uint64(0x9D2C5680)
        y ^= (y << np.uint64(15)) & np.uint64(0xEFC60000)
        y ^= y >> np.uint64(18)
        self.buf = (y & np.uint64(0xFFFFFFFF)).tolist()
        self.i = 0

    def __call__(self):
        if self.i >= 624:
            self._gen()
        v = self.buf[self.i]
        self.i += 1
        return v


def uniform_u32(g, n):
    """uniform_int_distribution<...>{0, n - 1}(g) for a 32-bit engine and n <= 2^32 - 1
    values: Lemire's nearly-divisionless _S_nd with 64-bit products (GCC 11)."""
    prod = g() * n
    low = prod & 0xFFFFFFFF
    if low < n:
        thr = ((1 << 32) - n) % n
        while low < thr:
            prod = g() * n
            low = prod & 0xFFFFFFFF
    return prod >> 32


def shuffle(a, g):
    """std::shuffle (GCC 11 <bits/stl_algo.h>): two swap positions per draw while
    (2^32 - 1) / n >= n, else one uniform_int draw per position."""
    n = len(a)
    if n == 0:
        return
    if (0xFFFFFFFF // n) >= n:
        i = 1
        if n % 2 == 0:
            j = uniform_u32(g, 2)
            a[i], a[j] = a[j], a[i]
            i += 1
        while i != n:
            r = i + 1
            x = uniform_u32(g, r * (r + 1))
            p1, p2 = x // (r + 1), x % (r + 1)
            a[i], a[p1] = a[p1], a[i]
            a[i + 1], a[p2] = a[p2], a[i + 1]
            i += 2
        return
    for i in range(1, n):
        j = uniform_u32(g, i + 1)
        a[i], a[j] = a[j], a[i]


_TWO32 = F(4294967296.0)
_ONE_MINUS = np.nextafter(F(1), F(0))


def uniform_float(g, a, b):
    """uniform_real_distribution<float>(a, b)(g) = generate_canonical<float, 24> * (b - a) + a."""
    r = F(g()) / _TWO32
    if r >= F(1):
        r = _ONE_MINUS
    return F(F(r * F(F(b) - F(a))) + F(a))


# ---------------------------------------------------------------------------
# include/isolation_forest.h
def calc_h(i):
    return math.log(i) + 0.5772156649


def calc_c(n):
    if n > 2:
        return 2.0 * calc_h(n - 1) - (2.0 * (n - 1)) / float(n)
    if n == 2:
        return 1.0
    return 0.0


_C_CACHE = {}


def _c(n):
    v = _C_CACHE.get(n)
    if v is None:
        v = _C_CACHE[n] = calc_c(n)
    return v


def iforest_scores(data, trees=50, seed=12345, sample=None):
    """IsolationForest<float, 3>::Build(trees, seed, data, sample) + GetAnomalyScores; None
    when Build fails. A node's subtree membership depends on values only (items equal in the
    split dimension go the same way), so the std::sort order inside Node::Build is not needed;
    the draws are consumed in the depth-first build order of the reference."""
    data = np.ascontiguousarray(data, np.float32)
    n = len(data)
    psi = n // 2 if sample is None else sample
    if n == 0 or psi == 0 or psi > n:
        return None
    colsl = [data[:, 0].tolist(), data[:, 1].tolist(), data[:, 2].tolist()]
    max_depth = int(math.ceil(math.log2(psi)))
    gen = MT19937(seed)
    total = np.zeros(n)
    rows = np.arange(n)
    for _ in range(trees):
        tg = MT19937(gen()).next  # uniform_int<uint32>(0, 2^32-1): a raw draw (Q21)
        ids = list(range(n))
        shuffle(ids, tg)
        dim, split, left, right, val = [], [], [], [], []
        _build(tg, ids[:psi], 0, max_depth, colsl, dim, split, left, right, val)
        # GetPathLen (isolation_forest.h:240-252) for every item, level by level
        dim_a = np.asarray(dim)
        split_a = np.asarray(split, np.float32)
        left_a, right_a = np.asarray(left), np.asarray(right)
        leaf = left_a < 0
        node = np.zeros(n, np.int64)
        for _ in range(max_depth):
            inner = ~leaf[node]
            if not inner.any():
                break
            v = data[rows, dim_a[node]]
            nxt = np.where(v < split_a[node], left_a[node], right_a[node])
            node = np.where(inner, nxt, node)
        total += np.asarray(val)[node]
    avg = total / float(trees)
    c = calc_c(psi)
    return np.array([math.pow(2.0, -v / c) for v in avg.tolist()])


def _build(g, s, depth, max_depth, colsl, dim, split, left, right, val):
    """Node::Build (isolation_forest.h:165-224) on the sample items s; appends the node in
    pre-order and returns its index. A leaf keeps depth + CalculateC(size) (GetPathLen)."""
    k = len(dim)
    dim.append(0)
    split.append(0.0)
    left.append(-1)
    right.append(-1)
    m = len(s)
    val.append(depth + _c(m))
    if m - 1 < 1 or depth >= max_depth:
        return k
    d = uniform_u32(g, 3)
    vl = colsl[d]
    vals = [vl[i] for i in s]
    lo, hi = min(vals), max(vals)  # Node::Build sorts by dim and reads both ends
    if lo == hi:
        return k
    sp = float(uniform_float(g, lo, hi))
    ls = [i for i in s if vl[i] < sp]
    if not ls:
        return k
    rs = [i for i in s if vl[i] >= sp]
    dim[k] = d
    split[k] = sp
    left[k] = _build(g, ls, depth + 1, max_depth, colsl, dim, split, left, right, val)
    right[k] = _build(g, rs, depth + 1, max_depth, colsl, dim, split, left, right, val)
    return k


# ---------------------------------------------------------------------------
# libstdc++ std::sort (introsort, GCC 11 <bits/stl_algo.h>, <bits/stl_heap.h>): the order of
# equal keys matters for mvAngleTimesAndScore (Tracking.cc:2849), which can exceed 16 rows.
def std_sort(a, less):
    n = len(a)
    if n > 1:
        _introsort(a, 0, n, 2 * (n.bit_length() - 1), less)
        _final_insertion(a, 0, n, less)


def _introsort(a, first, last, depth, less):
    while last - first > 16:
        if depth == 0:
            _heap_sort(a, first, last, less)
            return
        depth -= 1
        mid = first + (last - first) // 2
        _median_to_first(a, first, first + 1, mid, last - 1, less)
        cut = _unguarded_partition(a, first + 1, last, first, less)
        _introsort(a, cut, last, depth, less)
        last = cut


def _median_to_first(a, r, x, y, z, less):
    if less(a[x], a[y]):
        if less(a[y], a[z]):
            a[r], a[y] = a[y], a[r]
        elif less(a[x], a[z]):
            a[r], a[z] = a[z], a[r]
        else:
            a[r], a[x] = a[x], a[r]
    elif less(a[x], a[z]):
        a[r], a[x] = a[x], a[r]
    elif less(a[y], a[z]):
        a[r], a[z] = a[z], a[r]
    else:
        a[r], a[y] = a[y], a[r]


def _unguarded_partition(a, first, last, pivot, less):
    while True:
        while less(a[first], a[pivot]):
            first += 1
        last -= 1
        while less(a[pivot], a[last]):
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _linear_insert(a, last, less):
    val = a[last]
    nxt = last - 1
    while less(val, a[nxt]):
        a[last] = a[nxt]
        last = nxt
        nxt -= 1
    a[last] = val


def _insertion(a, first, last, less):
    if first == last:
        return
    for i in range(first + 1, last):
        if less(a[i], a[first]):
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            _linear_insert(a, i, less)


def _final_insertion(a, first, last, less):
    if last - first > 16:
        _insertion(a, first, first + 16, less)
        for i in range(first + 16, last):
            _linear_insert(a, i, less)
    else:
        _insertion(a, first, last, less)


def _adjust_heap(a, first, hole, ln, val, less):
    top = hole
    child = hole
    while child < (ln - 1) // 2:
        child = 2 * (child + 1)
        if less(a[first + child], a[first + child - 1]):
            child -= 1
        a[first + hole] = a[first + child]
        hole = child
    if (ln & 1) == 0 and child == (ln - 2) // 2:
        child = 2 * (child + 1)
        a[first + hole] = a[first + child - 1]
        hole = child - 1
    parent = (hole - 1) // 2
    while hole > top and less(a[first + parent], val):
        a[first + hole] = a[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[first + hole] = val


def _heap_sort(a, first, last, less):
    ln = last - first
    if ln >= 2:
        parent = (ln - 2) // 2
        while True:
            _adjust_heap(a, first, parent, ln, a[first + parent], less)
            if parent == 0:
                break
            parent -= 1
    while last - first > 1:
        last -= 1
        val = a[last]
        a[last] = a[first]
        _adjust_heap(a, first, 0, last - first, val, less)


# ---------------------------------------------------------------------------
# cv::Rect (OpenCV 3.2) and Converter::bboxOverlapratio*, Converter.cc:193-212
def rect_and(a, b):
    x1, y1 = max(a[0], b[0]), max(a[1], b[1])
    w = min(a[0] + a[2], b[0] + b[2]) - x1
    h = min(a[1] + a[3], b[1] + b[3]) - y1
    if w <= 0 or h <= 0:
        return (0, 0, 0, 0)
    return (x1, y1, w, h)


def area(r):
    return i32(r[2] * r[3])


def iou(a, b):
    ov = area(rect_and(a, b))
    return fdiv(F(ov), F(i32(area(a) + area(b) - ov)))


def former(a, b):
    return fdiv(F(area(rect_and(a, b))), F(area(a)))


def latter(a, b):
    return fdiv(F(area(rect_and(a, b))), F(area(b)))


def contains(r, u, v):
    """Rect_<int>::contains(Point2f -> Point via cvRound), Q11."""
    px, py = cv_round(u), cv_round(v)
    return r[0] <= px < r[0] + r[2] and r[1] <= py < r[1] + r[3]


def rect_f(x, y, w, h):  # cv::Rect(float, float, float, float): truncation (Q11)
    return (trunc_i32(x), trunc_i32(y), trunc_i32(w), trunc_i32(h))


# ---------------------------------------------------------------------------
# cv::Mat products (Q12) and the pinhole projection, Object.cc:1338-1346 / Tracking.cc:2600-2619
def gemm3(R, P, c):
    """R (3x3 float32) * P (n x 3 float32) + c (3 float32): (float)((double)t + c)."""
    out = np.empty(P.shape, np.float32)
    for r in range(3):
        t = (R[r, 0] * P[:, 0] + R[r, 1] * P[:, 1]) + R[r, 2] * P[:, 2]
        out[:, r] = (t.astype(F64) + float(c[r])).astype(np.float32)
    return out


def project(T, P, K):
    """Rcw * P + tcw, then u = fx * xc * invzc + cx with invzc = 1.0 / zc (double)."""
    P = np.asarray(P, np.float32).reshape(-1, 3)
    with np.errstate(all="ignore"):
        c = gemm3(T[:3, :3], P, T[:3, 3])
        inv = (1.0 / c[:, 2].astype(F64)).astype(np.float32)
        u = (K[0] * c[:, 0]) * inv + K[2]
        v = (K[1] * c[:, 1]) * inv + K[3]
    return u, v


def seq_sum(rows):
    """cv::Mat += in a loop: float accumulation in order, starting from zeros."""
    if not len(rows):
        return np.zeros(3, np.float32)
    a = np.concatenate([np.zeros((1, 3), np.float32), np.asarray(rows, np.float32).reshape(-1, 3)])
    return np.add.accumulate(a, axis=0, dtype=np.float32)[-1].copy()


def fsum_seq(vals):
    s = F(0)
    for v in vals:
        s = F(s + v)
    return s


# ---------------------------------------------------------------------------
# Eigen / g2o rigid transforms (double)
def quat_from_R(m):
    """Eigen quaternion_assign_impl<Matrix3, 3, 3>; coeffs as (x, y, z, w)."""
    t = (m[0][0] + m[1][1]) + m[2][2]
    q = [0.0, 0.0, 0.0, 0.0]
    if t > 0.0:
        t = math.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2][1] - m[1][2]) * t
        q[1] = (m[0][2] - m[2][0]) * t
        q[2] = (m[1][0] - m[0][1]) * t
    else:
        i = 0
        if m[1][1] > m[0][0]:
            i = 1
        if m[2][2] > m[i][i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k][j] - m[j][k]) * t
        q[j] = (m[j][i] + m[i][j]) * t
        q[k] = (m[k][i] + m[i][k]) * t
    return q


def se3(R, t):
    """g2o::SE3Quat(R, t): quaternion of R, normalizeRotation (w >= 0, then normalize)."""
    q = quat_from_R(R)
    if q[3] < 0:
        q = [-x for x in q]
    z = (q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3])
    if z > 0.0:
        s = math.sqrt(z)
        q = [x / s for x in q]
    return (q, list(t))


def cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def qrot(q, v):
    """Eigen QuaternionBase::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv."""
    qv = q[:3]
    uv = cross(qv, v)
    uv = [x + x for x in uv]
    c = cross(qv, uv)
    return [(v[i] + q[3] * uv[i]) + c[i] for i in range(3)]


def se3_apply(p, v):
    r = qrot(p[0], v)
    return [r[i] + p[1][i] for i in range(3)]


def se3_inv(p):
    qc = [-p[0][0], -p[0][1], -p[0][2], p[0][3]]
    t = qrot(qc, [x * -1.0 for x in p[1]])
    return (qc, t)


SE3_ID = ([0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0])


# ---------------------------------------------------------------------------
# detect_3d_cuboid/object_3d_util.cpp:176-208,349-434
def merge_break_lines(L, dist_thr=20.0, angle_deg=5.0, length_thr=30.0):
    L = [list(r) for r in L]
    total = len(L)
    counter = 0
    athr = angle_deg / 180.0 * math.pi
    can = True
    while can and counter < 500:
        counter += 1
        can = False
        ang = [math.atan2(L[i][3] - L[i][1], L[i][2] - L[i][0]) for i in range(total)]
        for s1 in range(total - 1):
            for s2 in range(s1 + 1, total):
                diff = abs(ang[s1] - ang[s2])
                if smin(diff, math.pi - diff) < athr:
                    a, b = L[s1], L[s2]
                    d12 = math.sqrt((a[2] - b[0]) * (a[2] - b[0]) + (a[3] - b[1]) * (a[3] - b[1]))
                    d21 = math.sqrt((b[2] - a[0]) * (b[2] - a[0]) + (b[3] - a[1]) * (b[3] - a[1]))
                    if d12 < dist_thr or d21 < dist_thr:
                        st = a[0:2] if a[0] < b[0] else b[0:2]
                        en = a[2:4] if a[2] > b[2] else b[2:4]
                        mang = math.atan2(en[1] - st[1], en[0] - st[0])
                        tmp = abs(ang[s1] - mang)
                        if smin(tmp, math.pi - tmp) < athr:
                            L[s1] = [st[0], st[1], en[0], en[1]]
                            L[s2] = list(L[total - 1])  # fast_RemoveRow, matrix_utils.cpp:201-205
                            total -= 1
                            can = True
                            break
            if can:
                break
    out = []
    for i in range(total):
        dx, dy = L[i][2] - L[i][0], L[i][3] - L[i][1]
        if math.sqrt(dx * dx + dy * dy) > length_thr:
            out.append(L[i])
    return out


# ---------------------------------------------------------------------------
class MapPoint:
    __slots__ = ("id", "pos", "bad", "feat", "oidv")

    def __init__(self, pid):
        self.id = pid
        self.pos = np.zeros(3, np.float32)
        self.bad = False
        self.feat = (F(0), F(0))
        self.oidv = {}  # object_id_vector


class Obj2D:
    __slots__ = ("cls", "box", "k", "pts", "sum", "pos", "feat_rect", "bad", "method", "mnId", "raw_lines",
                 "_lines", "cols", "rows")

    def __init__(self, k, b, raw_lines, cols, rows):
        self.k = k
        self.cls = int(b[0])
        self.box = (int(b[1]), int(b[2]), int(b[3]), int(b[4]))
        self.pts = []
        self.sum = np.zeros(3, np.float32)
        self.pos = None
        self.feat_rect = (0, 0, 0, 0)
        self.bad = False
        self.method = 0
        self.mnId = -1
        self.raw_lines = raw_lines
        self._lines = None
        self.cols, self.rows = cols, rows

    def lines(self):
        """mObjLinesEigen, AssociateObjAndLines (Tracking.cc:2472-2527); evaluated when first
        read (SampleObjYaw), which gives the same rows: it depends on this frame only."""
        if self._lines is None:
            L = []
            for r in (self.raw_lines if self.raw_lines is not None else []):
                x1, y1, x2, y2 = (float(v) for v in r)
                if x2 < x1:  # align_left_right_edges
                    x1, y1, x2, y2 = x2, y2, x1, y1
                L.append((x1, y1, x2, y2))
            bx, by, bw, bh = self.box
            left = smax(0.0, bx - 15.0)
            right = float(smin(self.cols, bx + bw + 15))
            top = smax(0.0, by - 15.0)
            bottom = float(smin(self.rows, by + bh + 15))
            ins = [r for r in L if left <= r[0] <= right and top <= r[1] <= bottom
                   and left <= r[2] <= right and top <= r[3] <= bottom]
            self._lines = merge_break_lines(ins, 20.0, 5.0, 30.0)
        return self._lines


class ObjMap:
    def __init__(self):
        self.mnId = 0
        self.cls = 0
        self.frames = []
        self.pts = []
        self.sum = None
        self.center = None
        self.std = np.zeros(3, np.float32)
        self.cstd = np.zeros(3, np.float32)
        self.cstd_all = F(0)
        self.last = self.lastlast = (0, 0, 0, 0)
        self.last_add = self.lastlast_add = 0
        self.confidence = 0
        self.reobj = {}
        self.sametime = {}
        self.bad = False
        self.proj = (0, 0, 0, 0)
        self.xyz_min = [F(0)] * 3
        self.xyz_max = [F(0)] * 3
        self.cc = [0.0, 0.0, 0.0]  # cuboidCenter (Eigen::Vector3d)
        self.lenth = self.width = self.height = F(0)
        self.rotY = self.rotP = self.rotR = F(0)
        self.rmax = F(0)
        self.err_par = self.err_yaw = F(0)
        self.pose = SE3_ID
        self.pose_wo = SE3_ID
        self.corners_w = [[0.0, 0.0, 0.0] for _ in range(8)]
        self.angles = []  # mvAngleTimesAndScore rows (5 float32)


def _positions(pts):
    return np.array([p.pos for p in pts], np.float32).reshape(-1, 3)


def _pos_key(p):
    x = p.pos
    if not np.all(np.isfinite(x)):
        return None  # a - b of inf or NaN is never 0: never a duplicate (Q22)
    return (float(x[0]), float(x[1]), float(x[2]))


_T_TABLE = None


def t_table():
    """data/t_test.txt (read with ifstream >> float, Object.cc:448-458)."""
    global _T_TABLE
    if _T_TABLE is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                            "t_test.txt")
        with open(path) as fh:
            vals = [F(float(x)) for x in fh.read().split()][:122 * 9]
        _T_TABLE = [vals[9 * r:9 * r + 9] for r in range(122)]
    return _T_TABLE


YAW_CLASSES = (73, 64, 65, 66, 56)


class Replay:
    """One mono_tum process's object association; API of
    oracle/pyoracle.Replay."""

    def __init__(self, flag="iForest", w=640, h=480, K=(535.4, 539.2, 320.1, 247.6)):
        self.flag = flag
        self.cols, self.rows = w, h
        self.K = [F(k) for k in K]
        self.mps = {}
        self.objs = []
        self.ini = False
        self.ini_frame = 0
        self.biforest = True  # Object.cc:31, process global, cleared by "None" for good (Q6)
        self.T = np.eye(4, dtype=np.float32)
        self.fid = 0
        self.stats = dict(forests=0, merges=0, overlap_merges=0, yaw=0)

    def close(self):
        pass

    # ---- Tracking::TrackWithMotionModel object section, Tracking.cc:1243-1696
    def frame(self, fid, T, boxes, ids, pos, uv, bad=None, lines=None):
        with np.errstate(all="ignore"):
            return self._frame(int(fid), T, boxes, ids, pos, uv, bad, lines)

    def _frame(self, fid, T, boxes, ids, pos, uv, bad, lines):
        self.fid = fid
        self.T = np.asarray(T, np.float32).reshape(4, 4)
        boxes = np.asarray(boxes, np.int32).reshape(-1, 5)
        ids = np.asarray(ids, np.int32).reshape(-1)
        pos = np.asarray(pos, np.float32).reshape(-1, 3)
        uv = np.asarray(uv, np.float32).reshape(-1, 2)
        bad = np.zeros(len(ids), np.uint8) if bad is None else np.asarray(bad, np.uint8).reshape(-1)
        raw_lines = None if lines is None else np.asarray(lines, np.float32).reshape(-1, 4)
        # STEP 1 (:1245-1256)
        o2 = [Obj2D(k, b, raw_lines, self.cols, self.rows) for k, b in enumerate(boxes.tolist())]
        tracked = []
        for i, pid in enumerate(ids.tolist()):
            p = self.mps.get(pid)
            if p is None:
                p = self.mps[pid] = MapPoint(pid)
            p.pos = pos[i].copy()
            p.bad = bool(bad[i])
            tracked.append(p)
        # STEP 2 AssociateObjAndPoints (:2434-2468)
        good = np.array([not p.bad for p in tracked], bool)
        pu = np.rint(uv[:, 0].astype(F64)) if len(uv) else np.zeros(0)
        pv = np.rint(uv[:, 1].astype(F64)) if len(uv) else np.zeros(0)
        for f in o2:
            x, y, w, h = f.box
            m = good & (pu >= x) & (pu < x + w) & (pv >= y) & (pv < y + h)
            sel = np.nonzero(m)[0]
            for i in sel.tolist():
                tracked[i].feat = (uv[i, 0], uv[i, 1])
                f.pts.append(tracked[i])
            f.sum = seq_sum(pos[sel])
        # STEP 3 (AssociateObjAndLines): Obj2D.lines(), evaluated where SampleObjYaw reads it
        # STEP 4 (:1288-1300)
        for f in o2:
            self.frame_mean(f)
            if len(f.pts) < 8:
                continue
            self.boxplot(f)
        # STEP 5 (:1318-1368)
        for f in o2:
            n = len(f.pts)
            f.pos[:] = self.mat_div(f.sum, n)
            if n < 4:
                continue
            xs = sorted(float(p.feat[0]) for p in f.pts)
            ys = sorted(float(p.feat[1]) for p in f.pts)
            x_min, x_max, y_min, y_max = F(xs[0]), F(xs[-1]), F(ys[0]), F(ys[-1])
            if x_min < 0:
                x_min = F(0)
            if y_min < 0:
                y_min = F(0)
            if x_max > self.cols:
                x_max = F(self.cols)
            if y_max > self.rows:
                y_max = F(self.rows)
            f.feat_rect = rect_f(x_min, y_min, F(x_max - x_min), F(y_max - y_min))
        # STEP 6 (:1380-1460)
        for a in range(len(o2)):
            num = 0
            for b in range(len(o2)):
                if a == b:
                    continue
                if float(latter(o2[a].box, o2[b].box)) > 0.05:
                    num += 1
            if num > 4:
                o2[a].bad = True
        area_img = F(self.cols * self.rows)
        for a in range(len(o2)):
            f = o2[a]
            if f.bad:
                continue
            if f.cls in (0, 63, 15):
                f.bad = True
            if float(fdiv(F(area(f.box)), area_img)) > 0.5:
                f.bad = True
            x, y, w, h = f.box
            if len(f.pts) < 5:
                f.bad = True
            elif 5 <= len(f.pts) < 10:
                if x < 20 or y < 20 or x + w > self.cols - 20 or y + h > self.rows - 20:
                    f.bad = True
            for b in range(len(o2)):
                g = o2[b]
                if g.bad or a == b:
                    continue
                if float(iou(f.box, g.box)) > 0.3:
                    # mScore is 0 for every box (Q1): "keep the higher score" drops l
                    g.bad = True
                if float(iou(f.box, g.box)) > 0.05:
                    if float(former(f.box, g.box)) > 0.85:
                        f.bad = True
                    if float(latter(f.box, g.box)) > 0.85:
                        g.bad = True
        kept = []
        for f in o2:
            if f.bad:
                f.method = -1
            else:
                kept.append(f)
        # STEP 7/8: mLastFrame.mvObjectFrame is never copied (Q10)
        # STEP 9 InitObjMap (:2531-2598)
        if not self.ini:
            good_id = -1
            for f in kept:
                if len(f.pts) < 10:
                    f.method = 6
                    continue
                good_id += 1
                self.ini = True
                self.ini_frame = fid
                o = self.new_object(f, good_id, fid)
                f.method = 7
                self.mean_std(o)
                self.objs.append(o)
        # STEP 10 (:1541-1672)
        if fid > self.ini_frame and self.ini:
            for o in self.objs:
                if o.bad:
                    continue
                if u64(o.last_add) > u64(fid - 30):
                    self.project_rect(o)
                else:
                    o.proj = (0, 0, 0, 0)
            for f in kept:
                if len(f.pts) < 5:
                    f.method = 6
                    continue
                self.associate(f)
            for i in range(len(self.objs) - 1, -1, -1):
                if self.flag == "NA":
                    continue
                o = self.objs[i]
                if o.bad:
                    continue
                df = len(o.frames)
                if df < 10 and u64(o.last_add) < u64(fid - 30):
                    if df < 5:
                        o.bad = True
                    else:
                        ov = False
                        for j in range(len(self.objs) - 1, -1, -1):
                            if self.objs[j].bad or i == j:
                                continue
                            if self.whether_overlap(o, self.objs[j]):
                                ov = True
                                break
                        if ov:
                            o.bad = True
            for i in range(len(self.objs) - 1, -1, -1):
                if self.objs[i].last_add != fid:
                    continue
                for j in range(len(self.objs) - 1, -1, -1):
                    if i != j and self.objs[j].last_add == fid:
                        m = self.objs[i].sametime
                        k = self.objs[j].mnId
                        m[k] = m.get(k, 0) + 1
            for i in range(len(self.objs) - 1, -1, -1):
                o = self.objs[i]
                if o.bad:
                    continue
                if u64(o.last_add) < u64(fid - 5):
                    continue
                if o.cls in YAW_CLASSES and o.last_add == fid:
                    self.sample_yaw(o)
        out = np.zeros((len(o2), 4), np.int32)
        for f in o2:
            out[f.k] = (f.method, f.mnId, f.cls, len(f.pts))
        return out

    @staticmethod
    def mat_div(s, n):
        """cv::Mat / n: convertTo with alpha = (float)(1.0 / n), beta 0 (Q12)."""
        alpha = F(1.0 / n) if n else F(np.inf)
        return (s * alpha + F(0)).astype(np.float32)

    def frame_mean(self, f):
        """Object_2D::ComputeMeanAndStandardFrame (Object.cc:63-102); _Pos in place."""
        keep = []
        for p in f.pts:
            if p.bad:
                f.sum = (f.sum - p.pos).astype(np.float32)
            else:
                keep.append(p)
        f.pts = keep
        v = self.mat_div(f.sum, len(f.pts))
        if f.pos is None:
            f.pos = v
        else:
            f.pos[:] = v

    def boxplot(self, f):
        """Object_2D::RemoveOutliersByBoxPlot (Object.cc:106-158): sum_pos_3d is left as it is."""
        P = _positions(f.pts)
        z = gemm3(self.T[:3, :3], P, self.T[:3, 3])[:, 2]
        zs = np.sort(z)
        n = len(zs)
        if n // 4 <= 0 or n * 3 // 4 >= n - 1:
            return
        q1, q3 = zs[n // 4], zs[n * 3 // 4]
        iqr = F(q3 - q1)
        max_th = F(float(q3) + 1.5 * float(iqr))
        f.pts = [p for p, zz in zip(f.pts, z.tolist()) if not zz > max_th]
        self.frame_mean(f)

    def new_object(self, f, mnId, fid):
        """InitObjMap (Tracking.cc:2546-2577) / new object (Object.cc:661-701)."""
        o = ObjMap()
        o.frames.append(f)
        o.mnId = mnId
        o.cls = f.cls
        o.confidence = 1
        o.last_add = o.lastlast_add = fid
        o.last = f.box
        o.sum = f.sum      # cv::Mat header copies: shared buffers
        o.center = f.pos
        for p in f.pts:
            p.oidv.setdefault(mnId, 1)
            o.pts.append(p)
        f.mnId = mnId
        return o

    # ---- Object_2D::ObjectDataAssociation, Object.cc:162-710
    def associate(self, f):
        flag = self.flag
        if flag == "None":
            self.biforest = False
        objs = self.objs
        fid = self.fid
        cur = f.box
        iou_max = F(0)
        b_iou, id_iou, iou_max_id = False, -1, -1
        thr = F(0.5)
        # STEP 1
        if flag not in ("NA", "NP"):
            for i, o in enumerate(objs):
                if f.cls != o.cls or o.bad:
                    continue
                if u64(o.last_add) == u64(fid - 1):
                    if u64(o.lastlast_add) == u64(fid - 2):
                        L, LL = o.last, o.lastlast
                        ltx = F(L[0] * 2 - LL[0])
                        if ltx < 0:
                            ltx = F(0)
                        lty = F(L[1] * 2 - LL[1])
                        if lty < 0:
                            lty = F(0)
                        rdx = F((L[0] + L[2]) * 2 - (LL[0] + LL[2]))
                        if ltx > self.cols:
                            rdx = F(self.cols)
                        rdy = F((L[1] + L[3]) * 2 - (LL[1] + LL[3]))
                        if lty > self.rows:
                            rdy = F(self.rows)
                        pred = rect_f(ltx, lty, F(rdx - ltx), F(rdy - lty))
                        thr = F(0.6)
                    else:
                        pred = o.last
                    v = iou(cur, pred)
                    if v > thr and v > iou_max:
                        iou_max = v
                        iou_max_id = i
            if iou_max > 0 and iou_max_id >= 0:
                if self.update(objs[iou_max_id], f, 1):
                    b_iou, id_iou = True, iou_max_id
                    f.method = 1
        # STEP 2
        b_np, id_np = False, -1
        np_ids = []
        if flag not in ("NA", "IoU"):
            for i in range(len(objs) - 1, -1, -1):
                o = objs[i]
                if f.cls != o.cls or o.bad:
                    continue
                r = self.np_test(f, o)
                if r == 0:
                    break
                if r == 2:
                    continue
                np_ids.append(i)
            if np_ids:
                if b_iou:
                    for i in np_ids:
                        if i != id_iou:
                            self.reobj(id_iou, i)
                else:
                    for a, i in enumerate(np_ids):
                        if self.update(objs[i], f, 2):
                            b_np, id_np = True, i
                            f.method = 2
                            if len(np_ids) > a + 1:
                                for j in np_ids[a + 1:]:
                                    self.reobj(i, j)
                                break
        # STEP 3
        b_pro, id_pro = False, -1
        pro_ids = []
        if flag not in ("NA", "IoU", "NP"):
            fmax = F(0)
            pmax_id = -1
            for i in range(len(objs) - 1, -1, -1):
                o = objs[i]
                if f.cls != o.cls or o.bad:
                    continue
                if len(f.pts) >= 10 and len(o.frames) > 8:
                    continue
                v = smax(iou(cur, o.proj), iou(f.feat_rect, o.proj))
                if float(v) >= 0.25 and v > fmax:
                    fmax = v
                    pmax_id = i
                    pro_ids.append(i)
            if float(fmax) >= 0.25:
                pro_ids.sort()
                if b_iou or b_np:
                    re = id_np if b_np else id_iou
                    for j in reversed(pro_ids):
                        if j != re:
                            self.reobj(re, j)
                else:
                    if self.update(objs[pmax_id], f, 4):
                        b_pro, id_pro = True, pmax_id
                        f.method = 4
                    for j in reversed(pro_ids):
                        if j != pmax_id:
                            self.reobj(pmax_id, j)
        # STEP 4 t-test
        b_t = False
        t_ids, t_lower = [], []
        if flag not in ("NA", "IoU", "NP"):
            tt = t_table()
            for i in range(len(objs) - 1, -1, -1):
                o = objs[i]
                if f.cls != o.cls or o.bad:
                    continue
                df = len(o.frames)
                if df <= 8:
                    continue
                v = smax(iou(cur, o.proj), iou(f.feat_rect, o.proj))
                sq = math.sqrt(df)
                t = []
                for a in range(3):
                    dis = abs(F(o.center[a] - f.pos[a]))
                    t.append(F(F64(dis) / (F64(o.cstd[a]) / sq)))
                row = tt[min(df - 1, 121)]
                mean3 = F(F(F(t[0] + t[1]) + t[2]) / F(3))
                if t[0] < row[5] and t[1] < row[5] and t[2] < row[5]:
                    t_ids.append(i)
                elif float(v) > 0.25:
                    if t[0] < row[8] and t[1] < row[8] and t[2] < row[8]:
                        t_ids.append(i)
                    elif float(v) > 0.25 and mean3 < 10:
                        t_ids.append(i)
                    else:
                        t_lower.append(i)
                elif mean3 < 4:
                    self.project_rect(o)
                    vf = smax(iou(cur, o.proj), iou(f.feat_rect, o.proj))
                    if float(vf) > 0.25:
                        t_lower.append(i)
            if b_iou or b_np or b_pro:
                re = id_pro if b_pro else (id_np if b_np else id_iou)
                for j in t_ids:
                    if j != re:
                        self.reobj(re, j)
                for j in t_lower:
                    if j != re:
                        self.reobj(re, j)
            else:
                for a, i in enumerate(t_ids):
                    if self.update(objs[i], f, 3):
                        b_t = True
                        f.method = 3
                        for j in t_ids[a + 1:]:
                            self.reobj(i, j)
                        for j in t_lower:
                            if j != i:
                                self.reobj(i, j)
                        break
        # create a new object (:648-701)
        if b_iou or b_np or b_pro or b_t:
            return
        x, y, w, h = f.box
        if x < 10 or y < 10 or x + w > self.cols - 10 or y + h > self.rows - 10:
            f.bad = True
            return
        o = self.new_object(f, len(objs), fid)
        f.method = 5
        self.iforest(o)
        self.mean_std(o)
        objs.append(o)

    def reobj(self, a, b):
        m = self.objs[a].reobj
        k = self.objs[b].mnId
        m[k] = m.get(k, 0) + 1

    def np_test(self, f, o):
        """Object_2D::NoParaDataAssociation (Object.cc:714-930): Wilcoxon rank-sum in 3 axes."""
        fp = [p for p in f.pts if not p.bad]  # out_point is false (Q7)
        m = len(fp)
        op = [p for p in o.pts if not p.bad]
        n = len(op)
        if m < 20:
            return 0
        if n < 20:
            return 2
        Q = _positions(op)
        if n > 3 * m:
            n = 3 * m
            step = len(o.pts) // n
            S = [np.sort(Q[:, a])[::step] for a in range(3)]  # axes sorted independently (Q3)
        else:
            S = [Q[:, a] for a in range(3)]
        n = len(S[0])
        Pm = _positions(fp)
        half_n = F(cdiv(i32(n * (n + 1)), 2))
        half_m = F(cdiv(i32(m * (m + 1)), 2))
        prod = i32(i32(m * n) * (m + n + 1))  # int arithmetic, wraps (Q4)
        q = cdiv(prod, 12)
        sq = math.sqrt(q) if q >= 0 else float("nan")
        r1 = F(0.5 * m * (m + n + 1) - 1.282 * sq)
        r2 = F(0.5 * m * (m + n + 1) + 1.282 * sq)
        add = 0
        for a in range(3):
            srt = np.sort(S[a])
            x1 = Pm[:, a]
            lo = np.searchsorted(srt, x1, "left")
            hi = np.searchsorted(srt, x1, "right")
            w12 = int(lo.sum())
            w21 = int((n - hi).sum())
            w00 = int((hi - lo).sum())
            assert max(w12, w21, w00) < (1 << 24)  # the float counters stay exact
            wx = F(smin(F(F(w12) + half_m), F(F(w21) + half_n)) + F(F(w00) / F(2)))
            if wx > r1 and wx < r2:
                add += 1
        return 1 if add == 3 else 2

    # ---- Object_Map
    def project_rect(self, o):
        """ComputeProjectRectFrame (Object.cc:1558-1603)."""
        if not o.pts:
            return
        u, v = project(self.T, _positions(o.pts), self.K)
        x_min, x_max = F(u.min()), F(u.max())
        y_min, y_max = F(v.min()), F(v.max())
        if x_min < 0:
            x_min = F(0)
        if y_min < 0:
            y_min = F(0)
        if x_max > self.cols:
            x_max = F(self.cols)
        if y_max > self.rows:
            y_max = F(self.rows)
        o.proj = rect_f(x_min, y_min, F(x_max - x_min), F(y_max - y_min))

    def update(self, o, f, code):
        """DataAssociateUpdate (Object.cc:1313-1554)."""
        if f.cls != o.cls:
            return False
        if code not in (1, 4):
            self.project_rect(o)
            r1 = o.proj
            P = np.concatenate([_positions(f.pts), _positions(o.pts)])
            u, v = project(self.T, P, self.K)
            x_min, x_max = F(u.min()), F(u.max())
            y_min, y_max = F(v.min()), F(v.max())
            if x_min < 0:
                x_min = F(0)
            if y_min < 0:
                y_min = F(0)
            if x_max > self.cols:
                x_max = F(self.cols)
            if y_max > self.rows:
                y_max = F(self.rows)
            r2 = rect_f(x_min, y_min, F(x_max - x_min), F(y_max - y_min))
            if float(iou(r1, r2)) < 0.5 and float(former(r2, f.box)) < 0.8:
                return False
        if o.last_add != self.fid:
            o.lastlast_add = o.last_add
            o.last_add = self.fid
            o.lastlast = o.last
            o.last = f.box
            o.confidence += 1
            o.frames.append(f)
        else:
            return False
        f.mnId = o.mnId
        # step 3
        keys = set()
        for q in o.pts:
            k = _pos_key(q)
            if k is not None:
                keys.add(k)
        pose_inv = se3_inv(o.pose) if len(o.frames) >= 10 and o.cls in (56, 77) else None
        th = F(1.0) if len(o.frames) <= 5 else F(0.9)
        lim = F(th * o.rmax)
        for p in f.pts:
            d = (o.center - p.pos).astype(np.float32)
            fdis = sqrtf(F(F(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
            if fdis > lim:
                continue
            if pose_inv is not None:
                s = se3_apply(pose_inv, [float(x) for x in p.pos])
                if (abs(s[0]) > 1.2 * float(o.lenth) / 2 or abs(s[1]) > 1.2 * float(o.width) / 2
                        or abs(s[2]) > 1.2 * float(o.height) / 2):
                    continue
            p.oidv[o.mnId] = p.oidv.get(o.mnId, 0) + 1
            k = _pos_key(p)
            if k is not None and k in keys:
                continue
            o.pts.append(p)
            if k is not None:
                keys.add(k)
            self._iadd(o.sum, p.pos)
        # step 4
        x, y, w, h = f.box
        if x > 25 and y > 25 and x + w < self.cols - 25 and y + h < self.rows - 25 and o.pts:
            u, v = project(self.T, _positions(o.pts), self.K)
            keep = []
            for p, uu, vv in zip(o.pts, u.tolist(), v.tolist()):
                if p.oidv.get(o.mnId, 0) > 8:
                    keep.append(p)
                    continue
                if 0 < uu < self.cols and 0 < vv < self.rows and not contains(f.box, uu, vv):
                    self._isub(o.sum, p.pos)
                    continue
                keep.append(p)
            o.pts = keep
        self.mean_std(o)
        self.iforest(o)
        return True

    @staticmethod
    def _iadd(s, v):
        s[:] = (s + v).astype(np.float32)
        return s

    @staticmethod
    def _isub(s, v):
        s[:] = (s - v).astype(np.float32)

    def mean_std(self, o):
        """ComputeMeanAndStandard (Object.cc:967-1198)."""
        o.sum[:] = 0
        o.pts = [p for p in o.pts if not p.bad]
        for p in o.pts:
            self._iadd(o.sum, p.pos)
        n = len(o.pts)
        o.center[:] = self.mat_div(o.sum, n)  # in place: the first observation's _Pos follows
        P = _positions(o.pts)
        c = o.center.copy()
        for a in range(3):
            d = (P[:, a] - c[a]).astype(np.float32)
            s = fsum_seq((d * d).tolist())
            o.std[a] = sqrtf(fdiv(s, F(n)))
        if n == 0:
            return
        nf = len(o.frames)
        for a in range(3):
            d = [F(fr.pos[a] - o.center[a]) for fr in o.frames]
            s = fsum_seq([F(x * x) for x in d])
            o.cstd[a] = sqrtf(fdiv(s, F(nf)))
        if nf < 5:
            mn = [F(P[:, a].min()) for a in range(3)]
            mx = [F(P[:, a].max()) for a in range(3)]
            o.cc = [float(F(F(mx[a] + mn[a]) / F(2))) for a in range(3)]
            o.xyz_min, o.xyz_max = mn, mx
            o.lenth, o.width, o.height = F(mx[0] - mn[0]), F(mx[1] - mn[1]), F(mx[2] - mn[2])
        self.update_pose(o)
        inv = se3_inv(o.pose)
        Po = np.array([se3_apply(inv, [float(x) for x in p]) for p in P.tolist()]).astype(np.float32)
        mn = [float(Po[:, a].min()) for a in range(3)]
        mx = [float(Po[:, a].max()) for a in range(3)]
        # corners 1..8 (Object.cc:1094-1111)
        sel = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
        cv = [[mx[a] if s[a] else mn[a] for a in range(3)] for s in sel]
        corners = [se3_apply(o.pose, v) for v in cv]
        o.corners_w = [se3_apply(o.pose_wo, v) for v in cv]
        o.lenth, o.width, o.height = F(F(mx[0]) - F(mn[0])), F(F(mx[1]) - F(mn[1])), F(F(mx[2]) - F(mn[2]))
        o.cc = [(corners[1][a] + corners[7][a]) / 2 for a in range(3)]
        self.update_pose(o)
        rmax = F(0)
        for cn in corners:
            d = [F(o.center[a] - F(cn[a])) for a in range(3)]
            rmax = smax(rmax, sqrtf(F(F(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))
        o.rmax = rmax
        dis = F(0)
        for fr in o.frames:
            d = [F(fr.pos[a] - o.center[a]) for a in range(3)]
            dis = F(dis + sqrtf(F(F(F(d[0] * d[0]) + F(d[1] * d[1])) + F(d[2] * d[2]))))
        o.cstd_all = sqrtf(fdiv(dis, F(nf)))

    def update_pose(self, o):
        """Object_Map::UpdateObjPose (Object.cc:2193-2248)."""
        cp, sp = cosf(o.rotP), sinf(o.rotP)
        sr, cr = sinf(o.rotR), cosf(o.rotR)
        sy, cy = sinf(o.rotY), cosf(o.rotY)
        R = [[F(cp * cy), F(F(F(sr * sp) * cy) - F(cr * sy)), F(F(F(cr * sp) * cy) + F(sr * sy))],
             [F(cp * sy), F(F(F(sr * sp) * sy) + F(cr * cy)), F(F(F(cr * sp) * sy) - F(sr * cy))],
             [F(-sp), F(sr * cp), F(cr * cp)]]
        # Rcw (identity) * Ryaw as a float gemm: exact (up to the sign of zeros)
        Rr = [[float(F(F(F(F(1) * R[0][j]) + F(F(0) * R[1][j])) + F(F(0) * R[2][j]))) if i == 0 else
               float(F(F(F(F(0) * R[0][j]) + F(F(1) * R[1][j])) + F(F(0) * R[2][j]))) if i == 1 else
               float(F(F(F(F(0) * R[0][j]) + F(F(0) * R[1][j])) + F(F(1) * R[2][j])))
               for j in range(3)] for i in range(3)]
        t = [float(F(o.cc[a])) for a in range(3)]
        o.pose = se3(Rr, t)
        I3 = [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]
        o.pose_wo = se3(I3, [float(o.center[0]), float(F(o.cc[1])), float(o.center[2])])

    def iforest(self, o):
        """IsolationForestDeleteOutliers (Object.cc:1202-1309)."""
        if not self.biforest:
            return
        if o.cls in (75, 64, 65):
            return
        th = F(0.65) if o.cls == 62 else F(0.6)
        if len(o.pts) < 30:
            return
        self.stats["forests"] += 1
        scores = iforest_scores(_positions(o.pts), 50, 12345, len(o.pts) // 2)
        if scores is None:
            return
        out = set(np.nonzero(scores > float(th))[0].tolist())
        if not out:
            return
        keep = []
        for i, p in enumerate(o.pts):
            if i in out:
                self._isub(o.sum, p.pos)
            else:
                keep.append(p)
        o.pts = keep

    def whether_overlap(self, a, b):
        """Object_Map::WhetherOverlap (Object.cc:1906-1925)."""
        d = [F(abs(a.cc[k] - b.cc[k])) for k in range(3)]
        sl = F(F(a.lenth / F(2)) + F(b.lenth / F(2)))
        sw = F(F(a.width / F(2)) + F(b.width / F(2)))
        sh = F(F(a.height / F(2)) + F(b.height / F(2)))
        return d[0] < sl and d[1] < sw and d[2] < sh

    # ---- Tracking::SampleObjYaw, Tracking.cc:2622-2862
    def world_to_img(self, P):
        u, v = project(self.T, np.asarray(P, np.float32).reshape(-1, 3), self.K)
        return u, v

    def sample_yaw(self, o):
        if self.flag in ("None", "iForest"):
            return
        self.stats["yaw"] += 1
        lines = o.frames[-1].lines()
        n_all = len(lines)
        num_max = 0
        f_error = F(0)
        f_error_yaw = F(0)
        sample = F(0)
        ccf = np.array([F(x) for x in o.cc], np.float32)
        base = np.array([[F(x) for x in c] for c in o.corners_w], np.float32) - ccf
        th = F(5.0)
        lang = []
        for r in lines:
            x1, y1, x2, y2 = r
            lang.append(F(math.atan2(y2 - y1, x2 - x1)))
        for i in range(30):
            yaw = F(((0.0 - i * 3.0) if i < 15 else (0.0 + (i - 15) * 3.0)) / 180.0 * math.pi)
            cp, sp, sr, cr = cosf(0), sinf(0), sinf(0), cosf(0)
            sy, cy = sinf(yaw), cosf(yaw)
            R = np.array([[F(cp * cy), F(F(F(sr * sp) * cy) - F(cr * sy)), F(F(F(cr * sp) * cy) + F(sr * sy))],
                          [F(cp * sy), F(F(F(sr * sp) * sy) + F(cr * cy)), F(F(F(cr * sp) * sy) - F(sr * cy))],
                          [F(-sp), F(sr * cp), F(cr * cp)]], np.float32)
            C = gemm3(R, base, ccf)
            u, v = self.world_to_img(C)
            px, py = u.tolist(), v.tolist()

            def edge(a, b):
                ax, ay, bx, by = F(px[a]), F(py[a]), F(px[b]), F(py[b])
                if bx > ax:
                    ang = atan2f(F(by - ay), F(bx - ax))
                else:
                    ang = atan2f(F(ay - by), F(ax - bx))
                dy, dx = F(by - ay), F(bx - ax)
                return ang, sqrtf(F(F(dy * dy) + F(dx * dx)))

            a1, l1 = edge(4, 5)  # point5 -> point6
            a2, l2 = edge(5, 6)  # point6 -> point7
            a3, l3 = edge(1, 5)  # point2 -> point6
            num = 0
            err = F(0)
            err_yaw = F(0)
            d1s = float(F(a1 * F(180))) / math.pi
            d2s = float(F(a2 * F(180))) / math.pi
            d3s = float(F(a3 * F(180))) / math.pi
            lmin = smin(smin(l1, l2), l3)
            for ang in lang:
                s = float(F(ang * F(180))) / math.pi
                da1, da2, da3 = F(abs(s - d1s)), F(abs(s - d2s)), F(abs(s - d3s))
                if o.cls == 56:
                    if da2 < th or da3 < th:
                        num += 1
                    if da1 < th:
                        num += 3
                else:
                    if lmin == l1:
                        if da2 < th or da3 < th:
                            num += 1
                            if da2 < th:
                                err = F(err + da2)
                            if da3 < th:
                                err = F(err + da3)
                        err_yaw = F(err_yaw + smin(da2, da3))
                    if lmin == l2:
                        if da1 < th or da3 < th:
                            num += 1
                            if da1 < th:
                                err = F(err + da1)
                            if da3 < th:
                                err = F(err + da3)
                        err_yaw = F(err_yaw + smin(da3, da1))
                    if lmin == l3:
                        if da1 < th or da2 < th:
                            num += 1
                            if da1 < th:
                                err = F(err + da1)
                            if da2 < th:
                                err = F(err + da2)
                        err_yaw = F(err_yaw + smin(da2, da1))
            if num == 0:
                num = 1
                err_yaw = F(10.0)
            if num > num_max:
                num_max = num
                sample = yaw
                f_error = err
                f_error_yaw = F(float(fdiv(err_yaw, F(num))) / 10.0)
        with np.errstate(all="ignore"):
            score = F(float(fdiv(F(num_max), F(n_all))) * (1.0 - 0.1 * float(f_error_yaw)))
        if np.isinf(score):
            score = F(0)
        new = [sample, F(1), score, f_error, f_error_yaw]
        fresh = True
        for row in o.angles:
            if row[0] == new[0]:
                row[1] = F(float(row[1]) + 1.0)
                inv = F(F(1) / row[1])
                one_m = F(F(1) - inv)
                row[2] = F(F(new[2] * inv) + F(row[2] * one_m))
                row[3] = F(F(new[3] * inv) + F(row[3] * one_m))
                row[4] = F(F(new[4] * inv) + F(row[4] * one_m))
                fresh = False
        if fresh:
            o.angles.append(new)
        std_sort(o.angles, lambda a, b: a[1] > b[1])  # VIC with index = 1
        best, best_score = 0, F(0)
        for i in range(min(3, len(o.angles))):
            if o.angles[i][2] >= best_score:
                best_score = o.angles[i][2]
                best = i
        o.rotY = o.angles[best][0]
        o.err_par = o.angles[best][3]
        o.err_yaw = o.angles[best][4]

    # ---- LocalMapping, LocalMapping.cc:86-92,772-882
    def local_mapping(self):
        with np.errstate(all="ignore"):
            for o in self.objs:  # UpdateObject
                if len(o.pts) < 10 or o.bad:
                    continue
                self.mean_std(o)
            if self.flag in ("NA", "IoU", "NP"):
                return
            for o in self.objs:  # MergePotentialAssObjs
                if o.bad:
                    continue
                if len(o.frames) >= 10 and o.reobj:
                    self.whether_merge(o)
            objs = self.objs  # WhetherOverlapObject
            for i in range(len(objs)):
                a = objs[i]
                if len(a.pts) < 10 or a.bad or len(a.frames) < 10:
                    continue
                for j in range(len(objs)):
                    if i == j:
                        continue
                    b = objs[j]
                    if len(b.pts) < 10 or b.bad or len(b.frames) < 10:
                        continue
                    d = [F(abs(a.cc[k] - b.cc[k])) for k in range(3)]
                    sl = F(F(a.lenth / F(2)) + F(b.lenth / F(2)))
                    sw = F(F(a.width / F(2)) + F(b.width / F(2)))
                    sh = F(F(a.height / F(2)) + F(b.height / F(2)))
                    if d[0] < sl and d[1] < sw and d[2] < sh:
                        self.deal_overlap(a, b, F(sl - d[0]), F(sw - d[1]), F(sh - d[2]))

    def update_points(self, ids, pos=None, bad=None):
        ids = np.asarray(ids, np.int32).reshape(-1)
        if pos is not None:
            pos = np.asarray(pos, np.float32).reshape(-1, 3)
        for i, pid in enumerate(ids.tolist()):
            p = self.mps.get(pid)
            if p is None:
                continue
            if pos is not None:
                p.pos = pos[i].copy()
            if bad is not None:
                p.bad = bool(bad[i])

    def step(self, fid, f):
        out = self.frame(fid, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        if "upd_ids" in f:
            self.update_points(f["upd_ids"], f["upd_pos"], f["upd_bad"])
        if f["kf"]:
            self.local_mapping()
        return out

    def whether_merge(self, a):
        """Object_Map::WhetherMergeTwoMapObjs (Object.cc:1605-1652). DoubleSampleTtest has no
        side effects and its verdict cannot change the branch (bSametime is false there)."""
        for oid, cnt in sorted(a.reobj.items()):
            if cnt < 3:
                continue
            b = self.objs[oid]
            if b.bad:
                continue
            if oid in a.sametime:
                continue
            self.stats["merges"] += 1
            if len(a.frames) > len(b.frames):
                self.merge(a, b)
                self.mean_std(a)
                self.iforest(a)
                b.bad = True
            else:
                self.merge(b, a)
                self.mean_std(b)
                self.iforest(b)
                a.bad = True

    def merge(self, a, b):
        """Object_Map::MergeTwoMapObjs (Object.cc:1716-1901): b into a."""
        inv = se3_inv(a.pose)
        keys = set()
        for q in a.pts:
            k = _pos_key(q)
            if k is not None:
                keys.add(k)
        for p in b.pts:
            s = se3_apply(inv, [float(x) for x in p.pos])
            if (abs(s[0]) > 1.1 * float(a.lenth) / 2 or abs(s[1]) > 1.1 * float(a.width) / 2
                    or abs(s[2]) > 1.1 * float(a.height) / 2):
                continue
            p.oidv[a.mnId] = p.oidv.get(a.mnId, 0) + 1
            k = _pos_key(p)
            if k is not None and k in keys:
                continue
            a.pts.append(p)
            if k is not None:
                keys.add(k)
            self._iadd(a.sum, p.pos)
        for fr in b.frames:
            fr.mnId = a.mnId
            a.confidence += 1
            a.frames.append(fr)
        for k, v in sorted(b.sametime.items()):
            if k in a.sametime:
                a.sametime[k] += v
            else:
                a.sametime[k] = 1
        o_last, o_lastlast, o_rect = a.last_add, a.lastlast_add, a.last
        if a.last_add > b.last_add:
            if o_lastlast > b.last_add:
                pass
            else:
                a.lastlast_add = b.last_add
                a.lastlast = b.frames[-1].box
        else:
            a.last_add = b.last_add
            a.last = b.frames[-1].box
            if o_last > b.lastlast_add:
                a.lastlast_add = o_last
                a.lastlast = o_rect
            else:
                a.lastlast_add = b.lastlast_add
                a.lastlast = b.frames[-2].box if len(b.frames) >= 2 else b.frames[0].box  # Q29
        if a.cls in YAW_CLASSES:
            for rr in b.angles:
                fresh = True
                for rt in a.angles:
                    if rr[0] == rt[0]:
                        rt[1] = F(rt[1] + rr[1])
                        w_old = F(F(rt[1] - rr[1]) / rt[1])
                        w_new = F(rr[1] / rt[1])
                        rt[2] = F(F(rt[2] * w_old) + F(rr[2] * w_new))
                        rt[3] = F(F(rt[3] * w_old) + F(rr[3] * w_new))
                        rt[4] = F(F(rt[4] * w_old) + F(rr[4] * w_new))
                        fresh = False
                        break
                if fresh:
                    a.angles.append(list(rr))
            if a.angles:
                best, best_score = 0, F(0)
                for i in range(min(6, len(a.angles))):
                    if a.angles[i][2] > best_score:
                        best_score = a.angles[i][2]
                        best = i
                a.rotY = a.angles[best][0]
                a.err_par = a.angles[best][3]
                a.err_yaw = a.angles[best][4]
                self.update_pose(a)

    def deal_overlap(self, a, b, ox, oy, oz):
        """Object_Map::DealTwoOverlapObjs (Object.cc:2073-2178)."""
        va = F(F(a.lenth * a.width) * a.height)
        vb = F(F(b.lenth * b.width) * b.height)
        vo = F(F(ox * oy) * oz)
        b_iou = float(fdiv(vo, F(F(va + vb) - vo))) >= 0.3
        b_vol = va > F(2 * vb) or vb > F(2 * va)
        b_same = a.sametime.get(b.mnId, 0) > 3
        b_cls = a.cls == b.cls
        if b_iou and not b_vol and not b_same and b_cls:
            self.stats["overlap_merges"] += 1
            if len(a.frames) >= len(b.frames):
                self.merge(a, b)
                b.bad = True
            else:
                self.merge(b, a)
                a.bad = True
        elif b_vol and not b_same and b_cls:
            if len(a.frames) >= len(b.frames) and va > vb:
                b.bad = True
            elif len(a.frames) < len(b.frames) and va < vb:
                a.bad = True
        elif b_iou and not b_vol and b_same and b_cls:
            self.divide(a, b, ox, oy, oz)
            self.divide(b, b, ox, oy, oz)  # the reference passes OverlapObj to itself (:2145)
            self.mean_std(a)
            self.mean_std(b)
        elif not b_iou and b_vol and b_same and not b_cls:
            if va > vb:
                self.big_to_small(a, b)
            elif va < vb:
                self.big_to_small(b, a)
        elif b_iou and not b_same and b_cls:
            if len(a.frames) // 2 >= len(b.frames):
                self.merge(a, b)
                b.bad = True
            elif len(b.frames) // 2 >= len(a.frames):
                self.merge(b, a)
                a.bad = True

    def divide(self, a, other, ox, oy, oz):
        """DivideEquallyTwoObjs (Object.cc:2040-2069)."""
        half = [F(F(other.lenth / F(2)) - F(ox / F(2))), F(F(other.width / F(2)) - F(oy / F(2))),
                F(F(other.height / F(2)) - F(oz / F(2)))]
        lo = [other.cc[k] - float(half[k]) for k in range(3)]
        hi = [other.cc[k] + float(half[k]) for k in range(3)]
        keep = []
        for p in a.pts:
            x = [float(v) for v in p.pos]
            if all(lo[k] < x[k] < hi[k] for k in range(3)):
                continue
            keep.append(p)
        a.pts = keep

    def big_to_small(self, a, small):
        """BigToSmall (Object.cc:1929-2036): only the point removal and the recomputation
        have an effect (the direction flags are assigned, never compared)."""
        keep = []
        for p in a.pts:
            if all(small.xyz_min[k] < p.pos[k] < small.xyz_max[k] for k in range(3)):
                continue
            keep.append(p)
        a.pts = keep
        self.mean_std(a)

    # ---- readout, layout of pyoracle.Replay.objects
    def objects(self):
        n = len(self.objs)
        ints = np.zeros((n, 8), np.int32)
        fl = np.zeros((n, 20), np.float32)
        pts = []
        for i, o in enumerate(self.objs):
            ints[i] = (o.mnId, o.cls, int(o.bad), len(o.frames), len(o.pts), o.last_add, len(o.reobj),
                       len(o.sametime))
            fl[i, 0:3] = o.center
            fl[i, 3:6] = o.std
            fl[i, 6:9] = o.cstd
            fl[i, 9:14] = (o.lenth, o.width, o.height, o.rmax, o.cstd_all)
            fl[i, 14:20] = (o.proj[0], o.proj[2], o.rotY, len(o.angles), o.err_par, o.err_yaw)
            pts.append(np.array([p.id for p in o.pts], np.int32))
        return ints, fl, pts
