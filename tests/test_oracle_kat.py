"""CPU known-answer tests of the oracle (the CPU restatement under oracle/).

The oracle is the checker for every GPU parity test, so it is pinned here
before it is trusted:
  * against the reference's own data file (tests/golden/t_test.txt) and the
    constants SURVEY.md §8c / Appendix A derive from the reference sources,
  * against the C++ standard's mt19937 known answer and against THIS
    toolchain's libstdc++ (<random>, std::shuffle) through a small program of
    our own (tests/native/std_rng_kat.cpp) -- the library the reference's
    include/isolation_forest.h draws from,
  * against independent numpy restatements of the same formulas (box filter
    mechanics, Hamming popcount, rectangle overlaps, the Wilcoxon counts of
    Object.cc NoParaDataAssociation, the isolation forest).
"""
import math
import os
import subprocess

import numpy as np
import pytest

import pyoracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
KAT = os.path.join(NATIVE, "_build", "std_rng_kat")


@pytest.fixture(scope="module")
def kat():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "_build/std_rng_kat"])
    return KAT


def run_kat(kat, *args, dtype=np.uint32, stdin=None):
    out = subprocess.run([kat] + [str(a) for a in args], input=stdin, stdout=subprocess.PIPE, check=True).stdout
    return np.frombuffer(out, dtype)


# ---------------------------------------------------------------- ORB constants
def test_level_quotas_and_scales():
    # ORBextractor::ORBextractor (src/ORBextractor.cc:420-470), 1000 features, 1.2, 8 levels
    p = orc.orb_params(1000, 1.2, 8)
    assert p["quotas"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    sc = [np.float32(1.0)]
    for _ in range(7):
        sc.append(np.float32(sc[-1] * np.float32(1.2)))
    assert np.array_equal(p["scale"], np.array(sc, np.float32))
    assert np.array_equal(p["sigma2"], np.array(sc, np.float32) * np.array(sc, np.float32))
    assert np.allclose(p["inv_scale"], 1.0 / np.array(sc, np.float64), rtol=1e-7)


def test_umax_table():
    # ORBextractor.cc:480-495: umax for the 31x31 patch (HALF_PATCH_SIZE 15)
    hp = 15
    umax = [0] * (hp + 1)
    vmax = int(math.floor(hp * math.sqrt(2.0) / 2 + 1))
    vmin = int(math.ceil(hp * math.sqrt(2.0) / 2))
    for v in range(vmax + 1):
        umax[v] = int(round(math.sqrt(hp * hp - v * v)))
    v0 = 0
    for v in range(hp, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    assert orc.orb_params()["umax"].tolist() == umax


def test_level_sizes_640x480():
    sizes = orc.level_sizes(640, 480)
    s = np.float32(1.0)
    for l in range(8):
        inv = np.float32(1.0) / s
        # cvRound(w * invScale) in float, Size(cvRound(..), cvRound(..))
        assert sizes[l] == (int(np.rint(np.float32(640) * inv)), int(np.rint(np.float32(480) * inv)))
        s = np.float32(s * np.float32(1.2))
    assert sizes[1] == (533, 400) and sizes[7] == (179, 134)


def _blur7_numpy(img):
    # GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on 8U, fixed point (Appendix A)
    k = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)
    p = np.pad(img.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == REFLECT_101
    h = sum(k[i] * p[:, i:i + img.shape[1]] for i in range(7))
    v = sum(k[i] * h[i:i + img.shape[0], :] for i in range(7))
    return np.clip((v + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


def test_gaussian_blur_mechanics():
    rng = np.random.default_rng(1)
    for shape in [(48, 64), (37, 53), (7, 7)]:
        img = rng.integers(0, 256, shape).astype(np.uint8)
        assert np.array_equal(orc.blur7(img), _blur7_numpy(img))


def test_fast_atan2_accuracy():
    rng = np.random.default_rng(2)
    for y, x in rng.normal(size=(2000, 2)).astype(np.float32):
        a = orc.fast_atan2(y, x)
        ref = math.degrees(math.atan2(y, x)) % 360.0
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.3  # cv::fastAtan2 documented accuracy
    assert orc.fast_atan2(0.0, 0.0) == 0.0


def test_hamming_popcount():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (200, 32)).astype(np.uint8)
    b = rng.integers(0, 256, (200, 32)).astype(np.uint8)
    ref = np.unpackbits(a ^ b, axis=1).sum(1)
    got = [orc.hamming(a[i], b[i]) for i in range(200)]
    assert got == ref.tolist()


def _rect_and(a, b):
    x1, y1 = max(a[0], b[0]), max(a[1], b[1])
    w = min(a[0] + a[2], b[0] + b[2]) - x1
    h = min(a[1] + a[3], b[1] + b[3]) - y1
    return 0 if w <= 0 or h <= 0 else w * h


def test_bbox_overlaps():
    # Converter::bboxOverlapratio / Former / Latter (src/Converter.cc:194-212)
    rng = np.random.default_rng(4)
    for _ in range(500):
        a = [int(v) for v in rng.integers(0, 300, 2)] + [int(v) for v in rng.integers(1, 200, 2)]
        b = [int(v) for v in rng.integers(0, 300, 2)] + [int(v) for v in rng.integers(1, 200, 2)]
        o = _rect_and(a, b)
        assert orc.bbox("iou", a, b) == np.float32(o) / np.float32(a[2] * a[3] + b[2] * b[3] - o)
        assert orc.bbox("former", a, b) == np.float32(o) / np.float32(a[2] * a[3])
        assert orc.bbox("latter", a, b) == np.float32(o) / np.float32(b[2] * b[3])


# ---------------------------------------------------------------- t-test table
def test_t_table_fixture():
    # the reference's data file (data/t_test.txt): row 0 is the alpha header,
    # read into the same 122x9 table as the 121 degree-of-freedom rows
    rows = [r.split() for r in open(os.path.join(HERE, "golden", "t_test.txt")).read().strip().splitlines()]
    body = [[float(v) for v in r] for r in rows]
    assert len(body) == 122 and all(len(r) == 9 for r in body)
    inc = open(os.path.join(os.path.dirname(HERE), "eao-slam_amd", "csrc", "t_table.inc")).read()
    body_txt = "\n".join(l for l in inc.splitlines() if not l.lstrip().startswith("//"))
    nums = [float(v.strip().rstrip("f")) for v in body_txt.replace("{", "").replace("}", "").split(",") if v.strip()]
    assert np.allclose(np.array(nums, np.float32).reshape(122, 9), np.array(body, np.float32), rtol=0, atol=0)


# ---------------------------------------------------------------- NP test
def _np_bruteforce(fp, fv, op, ov):
    """Object_2D::NoParaDataAssociation (src/Object.cc:714-930), O(m*n) counts."""
    F = fp[fv.astype(bool)]
    m = len(F)
    if m < 20:
        return 0, None
    O = op[ov.astype(bool)]
    n = len(O)
    if n < 20:
        return 2, None
    nt = len(op)
    sub = n > 3 * m
    step = nt // (3 * m) if sub else 1
    ws = []
    for a in range(3):
        ys = np.sort(O[:, a])
        if sub:
            ys = ys[::step]
        nn = len(ys)
        x = F[:, a][:, None]
        gt = int((ys[None, :] < x).sum())
        lt = int((ys[None, :] > x).sum())
        eq = int((ys[None, :] == x).sum())
        mm = np.float32(m * (m + 1) // 2)
        nn2 = np.float32(nn * (nn + 1) // 2)
        w = min(np.float32(gt) + mm, np.float32(lt) + nn2) + np.float32(eq) / np.float32(2)
        ws.append(np.float32(w))
    prod = np.int32(np.uint32(m) * np.uint32(nn) * np.uint32(m + nn + 1))  # Q4 wrap
    q = int(prod) // 12 if prod >= 0 else -((-int(prod)) // 12)
    base = 0.5 * m * (m + nn + 1)
    spread = 1.282 * math.sqrt(q) if q >= 0 else float("nan")
    r1, r2 = np.float32(base - spread), np.float32(base + spread)
    add = sum(1 for w in ws if r1 < w < r2)
    return (1 if add == 3 else 2), (ws, r1, r2)


@pytest.mark.parametrize("seed", range(8))
def test_np_counts_match_bruteforce(seed):
    rng = np.random.default_rng(100 + seed)
    m = int(rng.integers(10, 120))
    n = int(rng.integers(15, 600))
    c = rng.normal(0, 0.1, 3)
    fp = (rng.normal(0, 0.05, (m, 3)) + c).astype(np.float32)
    op = (rng.normal(0, 0.05, (n, 3)) + c + rng.normal(0, 0.02, 3)).astype(np.float32)
    op[: n // 10] = np.round(op[: n // 10], 2)  # ties
    fp[: m // 10] = np.round(fp[: m // 10], 2)
    fv = (rng.random(m) > 0.1).astype(np.uint8)
    ov = (rng.random(n) > 0.1).astype(np.uint8)
    verdict, extra = _np_bruteforce(fp, fv, op, ov)
    r = orc.np_test(fp, fv, op, ov)
    assert r["verdict"] == verdict
    if extra is not None:
        ws, r1, r2 = extra
        assert np.array_equal(r["w"], np.array(ws, np.float32))
        assert r["r1"] == r1 and r["r2"] == r2


# ---------------------------------------------------------------- random streams
def test_mt19937_standard_known_answer():
    # [rand.predef]: the 10000th output of a default-constructed mt19937
    assert orc.mt_stream(5489, 10000)[-1] == 4123659995


def test_mt19937_matches_libstdcxx(kat):
    for seed in (0, 1, 12345, 0xDEADBEEF):
        assert np.array_equal(orc.mt_stream(seed, 2000), run_kat(kat, "mt", seed, 2000))


@pytest.mark.parametrize("rng_", [2, 3, 7, 1000, 6 * 7, 2001 * 2002, 4001 * 4002, 0x7fffffff])
def test_uniform_int_matches_libstdcxx(kat, rng_):
    assert np.array_equal(orc.lemire(777, 3000, rng_), run_kat(kat, "lemire", 777, 3000, rng_))


@pytest.mark.parametrize("n", [1, 2, 3, 30, 31, 500, 2001, 4000])
def test_shuffle_matches_libstdcxx(kat, n):
    for seed in (12345, 99):
        assert np.array_equal(orc.shuffle(seed, n), run_kat(kat, "shuffle", seed, n))


def test_uniform_real_matches_libstdcxx(kat):
    for lo, hi in [(0.0, 1.0), (-2.5, 3.25), (1.9990001, 2.0)]:
        got = orc.canonical(4321, 5000, lo, hi)
        ref = run_kat(kat, "real", 4321, 5000, repr(lo), repr(hi), dtype=np.float32)
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("n", [30, 101, 640])
def test_iforest_matches_libstdcxx_forest(kat, n):
    rng = np.random.default_rng(n)
    pts = rng.normal([0, 0, 2], [0.05, 0.08, 0.03], (n, 3)).astype(np.float32)
    pts[: n // 20] += rng.uniform(-0.5, 0.5, (n // 20, 3)).astype(np.float32)
    ref = run_kat(kat, "iforest", n, 50, 12345, n // 2, dtype=np.float64, stdin=pts.tobytes())
    assert np.array_equal(orc.iforest(pts), ref)


@pytest.mark.parametrize("cn,rgb", [(3, True), (3, False), (4, True), (4, False)])
def test_color_to_gray_fixed_point(cn, rgb):
    """cvtColor(CV_{RGB,BGR}[A]2GRAY), OpenCV 3.2 RGB2Gray<uchar>: the oracle's
    table form equals the closed fixed-point formula, and the TUM3 case
    (Camera.RGB: 1 on BGR bytes, Q20) weights the first byte by R2Y."""
    rng = np.random.default_rng(cn * 2 + rgb)
    img = rng.integers(0, 256, (37, 53, cn), dtype=np.uint8)
    g = orc.color_to_gray(img, rgb)
    c0, c2 = (4899, 1868) if rgb else (1868, 4899)
    ref = ((img[..., 0].astype(np.int64) * c0 + img[..., 1].astype(np.int64) * 9617 +
            img[..., 2].astype(np.int64) * c2 + 8192) >> 14).astype(np.uint8)
    assert np.array_equal(g, ref)
    white = np.full((2, 2, cn), 255, np.uint8)
    assert (orc.color_to_gray(white, rgb) == 255).all() and (orc.color_to_gray(0 * white, rgb) == 0).all()


def test_iforest_erase_threshold_matches_libm_pow():
    """eao_iforest_erase_threshold: the engine erases a point when x = -E[h]/c(psi) >= x0,
    x0 the smallest double with pow(2, x) > th under glibc (what the reference's
    2^(-E[h]/c) > 0.6 / 0.65 comparison evaluates, Object.cc:1284-1300)."""
    import ctypes
    import math
    import eao_accel as ea
    L = ea.lib()
    for th in (0.6, 0.65):
        x0 = ctypes.c_double()
        assert L.eao_iforest_erase_threshold(ctypes.c_float(th), ctypes.byref(x0)) == 0
        thd = float(np.float32(th))
        x = x0.value
        assert math.pow(2.0, x) > thd
        below = x
        for _ in range(64):
            below = math.nextafter(below, -math.inf)
            assert math.pow(2.0, below) <= thd
        assert abs(x - math.log2(thd)) < 1e-12


def test_np_bounds_int32_wrap_q4():
    """The oracle's NoParaDataAssociation bounds against an independent restatement of
    Object.cc:905-911 with int32 two's-complement products."""
    def wrap(x):
        return (x + 2 ** 31) % 2 ** 32 - 2 ** 31
    rng = np.random.default_rng(5)
    for m, n in ((564, 1692), (600, 1800), (800, 2400), (100, 300)):
        f = rng.normal(0, 0.1, (m, 3)).astype(np.float32)
        o = rng.normal(0, 0.1, (n, 3)).astype(np.float32)
        r = orc.np_test(f, np.ones(m, np.uint8), o, np.ones(n, np.uint8))
        q = int(np.fix(wrap(m * n * (m + n + 1)) / 12))  # C integer division truncates
        base = 0.5 * m * (m + n + 1)
        sp = 1.282 * np.sqrt(np.float64(q)) if q >= 0 else np.nan
        assert np.allclose([r["r1"], r["r2"]], [np.float32(base - sp), np.float32(base + sp)], rtol=1e-7, equal_nan=True)


def test_line_oracle_properties():
    """The line restatement on a frame with one bright axis-aligned rectangle: the
    rectangle's four sides come out (EDLine's border rule only drops lines within 10 px
    of the image border), each about as long as the side, in the reference's
    start / end orientation convention (dark side on the left of the direction)."""
    img = np.full((480, 640), 40, np.uint8)
    img[149:331, 199:461] = 120  # half-intensity boundary pixels: the gradient peaks on one
    img[150:330, 200:460] = 200  # pixel row / column, so the edges carry anchors
    L = orc.edlines(img)
    assert 3 <= len(L) <= 8
    lengths = sorted(L[:, 5])
    assert lengths[-1] > 240  # a 260-px side
    for sx, sy, ex, ey, ang, ln in L:
        assert abs(np.hypot(ex - sx, ey - sy) - ln) < 1e-3
        assert -np.pi <= ang <= np.pi
    blur, dx, dy, g, d = orc.line_maps(img)
    # the 8U fixed-point taps cvRound(256 k) of getGaussianKernel(5, 1) are 14, 63, 103,
    # 63, 14 (sum 257, not renormalised -- the same rule as the 7x7 ORB blur): a flat
    # region of v blurs to (257^2 v + 2^15) >> 16
    assert blur[240, 320] == (257 * 257 * 200 + (1 << 15)) >> 16 and blur[20, 20] == (257 * 257 * 40 + (1 << 15)) >> 16
    assert dx[240, 200] > 0 and dy[150, 300] > 0  # dark -> bright steps


def test_line_oracle_color_input():
    """detectImpl's COLOR_BGR2GRAY (binary_descriptor.cpp:490-495): the colour entry equals the
    BGR-code conversion followed by the gray detector, and differs from the RGB code's gray."""
    import pyoracle as orc
    from tools import synth
    g = synth.line_frames(1, seed=0xEA7)[0]
    c = np.ascontiguousarray(np.stack([255 - g, g, g], 2))
    bgr = orc.color_to_gray(c, rgb=False)
    assert np.array_equal(orc.edlines_color(c), orc.edlines(bgr))
    assert np.array_equal(orc.edlines_color(g), orc.edlines(g))
    assert not np.array_equal(bgr, orc.color_to_gray(c, rgb=True))
    # OpenCV's fixed-point BGR2GRAY on a few pixels, restated independently
    b, gg, r = c[..., 0].astype(np.int64), c[..., 1].astype(np.int64), c[..., 2].astype(np.int64)
    assert np.array_equal(bgr, ((b * 1868 + gg * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8))
