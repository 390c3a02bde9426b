"""GPU association kernels vs the CPU restatement.

NoParaDataAssociation (src/Object.cc:714-930): counts bit-exact, W/r within
1e-5 (north-star tolerance), verdicts identical. Isolation forest
(include/isolation_forest.h): scores within 1e-5. ComputeProjectRectFrame
(src/Object.cc:1558-1603): rects identical.
"""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu


def _cloud(rng, n, center, spread, quant=None):
    p = rng.normal(center, spread, (n, 3)).astype(np.float32)
    if quant:
        p = (np.round(p / quant) * quant).astype(np.float32)
    return p


def test_np_pairs():
    rng = np.random.default_rng(21)
    fs, os_, exp = [], [], []
    for k in range(40):
        m = int(rng.integers(5, 300))
        n = int(rng.integers(5, 2500))
        same = rng.random() < 0.5
        f = _cloud(rng, m, [1, 2, 3], 0.1, quant=0.01 if k % 3 == 0 else None)
        o = _cloud(rng, n, [1, 2, 3] if same else [1.05, 2, 3.1], 0.1, quant=0.01 if k % 3 == 0 else None)
        fv = (rng.random(m) > 0.05).astype(np.uint8)
        ov = (rng.random(n) > 0.05).astype(np.uint8)
        fs.append((f, fv))
        os_.append((o, ov))
        exp.append(orc.np_test(f, fv, o, ov))
    a = ea.Assoc()
    got = a.np_batch(fs, os_)
    for g, o in zip(got, exp):
        assert g["verdict"] == o["verdict"]
        if o["verdict"] == 0:
            continue
        assert g["m"] == o["m"] and g["n"] == o["n"]
        if o["verdict"] in (1, 2) and o["n"] >= 20:
            assert np.array_equal(g["cnt_gt"], o["cnt_gt"]) and np.array_equal(g["cnt_lt"], o["cnt_lt"])
            assert np.array_equal(g["cnt_eq"], o["cnt_eq"])
            assert np.allclose(g["w"], o["w"], rtol=1e-5, atol=1e-5)
            assert np.allclose([g["r1"], g["r2"]], [o["r1"], o["r2"]], rtol=1e-5, atol=1e-5)


def test_np_pairs_direct_counts():
    """Pairs with m * n up to the direct-count threshold (131072) are counted by brute force
    against the compacted object values (no sort): with and without the n > 3m subsampling, ties
    (quantised clouds, frame values equal to object values), +-inf coordinates, invalid points on
    both sides, a NaN frame value (no count on its axis), tail quads (n % 4 != 0), one wave of
    frame points (m <= 64: 16 chunks) and up to 1024 (one chunk), and pairs just past the
    threshold (the sort path) in the same launch. (A NaN object value sends a pair to the sort
    path, whose order of NaN need not match std::sort's: map-point positions are finite, and that
    case is not pinned.)"""
    rng = np.random.default_rng(0xD1C7)
    cases = [(20, 20), (21, 61), (22, 63), (40, 121), (64, 2047), (65, 2016), (88, 195), (100, 1300),
             (128, 1024), (300, 437), (500, 262), (1000, 131), (1024, 128), (60, 2000), (120, 1093),
             (128, 1025), (400, 330), (30, 3000), (70, 1800)]
    fs, os_, exp = [], [], []
    for k, (m, n) in enumerate(cases):
        q = 0.01 if k % 3 == 0 else None
        f = _cloud(rng, m, [1, 2, 3], 0.1, quant=q)
        o = _cloud(rng, n, [1, 2, 3] if k % 2 else [1.03, 2, 3.04], 0.1, quant=q)
        fv = (rng.random(m) > 0.1).astype(np.uint8)
        ov = (rng.random(n) > 0.1).astype(np.uint8)
        if k == 4:
            f[:12] = o[:12]
        if k == 5:
            o[:3, 0], o[3:6, 2], f[:2, 1] = np.inf, -np.inf, np.inf
        if k == 6:
            f[5, 1] = np.nan
        if k == 8:
            fv[:] = 1
            ov[:] = 1
        fs.append((f, fv))
        os_.append((o, ov))
        exp.append(orc.np_test(f, fv, o, ov))
    got = ea.Assoc().np_batch(fs, os_)
    for k, (g, o) in enumerate(zip(got, exp)):
        info = (k, cases[k], {x: g[x] for x in ("verdict", "m", "n", "cnt_gt", "cnt_lt", "cnt_eq")},
                {x: o[x] for x in ("verdict", "m", "n", "cnt_gt", "cnt_lt", "cnt_eq")})
        assert g["verdict"] == o["verdict"] and g["m"] == o["m"] and g["n"] == o["n"], info
        assert np.array_equal(g["cnt_gt"], o["cnt_gt"]) and np.array_equal(g["cnt_lt"], o["cnt_lt"]), info
        assert np.array_equal(g["cnt_eq"], o["cnt_eq"]), info
        assert np.allclose(g["w"], o["w"], rtol=1e-5, atol=1e-5), info


def test_np_pairs_rank_path():
    """Large objects against small detections take the rank path of k_np_pairs (the m
    frame values sorted, the object streamed through binary searches): the counts must
    equal the sorted-sample search's, with ties (quantised clouds), +-inf coordinates,
    invalid points and NaN (which falls back to the sort path)."""
    rng = np.random.default_rng(0x4e50)
    fs, os_, exp = [], [], []
    cases = [(30, 8000, None), (100, 5000, 0.05), (250, 600, None), (64, 2048, 0.01), (300, 7000, 0.002),
             (21, 4000, None), (500, 8192, 0.02), (200, 3000, 0.5), (200, 1200, None), (40, 3000, None),
             (40, 3000, None)]
    for k, (m, n, q) in enumerate(cases):
        f = _cloud(rng, m, [1, 2, 3], 0.1, quant=q)
        o = _cloud(rng, n, [1, 2, 3] if k % 2 else [1.02, 2, 3.05], 0.1, quant=q)
        if k == 2:
            o[:5, 0] = np.inf
            o[5:9, 1] = -np.inf
            f[:2, 2] = np.inf
        if k == 3:
            f[:10] = o[:10]  # frame values equal to object values
        fv = (rng.random(m) > 0.05).astype(np.uint8)
        ov = (rng.random(n) > (0.85 if k == 8 else 0.05)).astype(np.uint8)  # k 8: few valid object points
        if k == 9:
            o[7, 1] = np.nan  # a NaN object value: the sort path
        if k == 10:
            f[3, 0] = np.nan  # a NaN frame value: the sort path after the frame pass
        fs.append((f, fv))
        os_.append((o, ov))
        exp.append(orc.np_test(f, fv, o, ov))
    got = ea.Assoc().np_batch(fs, os_)
    for k, (g, o) in enumerate(zip(got, exp)):
        info = (k, {x: g[x] for x in ("verdict", "m", "n", "cnt_gt", "cnt_lt", "cnt_eq")},
                {x: o[x] for x in ("verdict", "m", "n", "cnt_gt", "cnt_lt", "cnt_eq")})
        assert g["verdict"] == o["verdict"] and g["m"] == o["m"] and g["n"] == o["n"], info
        assert np.array_equal(g["cnt_gt"], o["cnt_gt"]) and np.array_equal(g["cnt_lt"], o["cnt_lt"]), info
        assert np.array_equal(g["cnt_eq"], o["cnt_eq"]), info
        assert np.allclose(g["w"], o["w"], rtol=1e-5, atol=1e-5), info


def test_iforest_scores():
    rng = np.random.default_rng(31)
    clouds = []
    for n in (30, 31, 64, 200, 777, 2000):
        c = _cloud(rng, n, [0, 0, 2], 0.05)
        c[: max(1, n // 20)] += rng.uniform(-0.5, 0.5, (max(1, n // 20), 3)).astype(np.float32)
        clouds.append(c)
    a = ea.Assoc()
    got = a.iforest(clouds)
    for c, g in zip(clouds, got):
        o = orc.iforest(c)
        assert np.allclose(g, o, rtol=1e-5, atol=1e-9)
        assert np.array_equal(g > 0.6, o > 0.6)


def test_iforest_mask_path_boundaries():
    """The forest kernel's mask path (nodes of more than 64 items as slot bits over a sample of
    at most 1024 items): samples just above 64 (one / two slots), at 1024 (16 slots), clouds with
    ties and duplicated points (min == max in a dimension, equal keys across a split), a cloud of
    one repeated point (the root is a leaf) and a flat cloud (one dimension constant), in one
    launch and alone; the same scores as the restatement."""
    rng = np.random.default_rng(0x3A5C)
    clouds = []
    for n in (129, 130, 131, 257, 1024, 2047, 2048):
        c = _cloud(rng, n, [0, 0, 2], 0.05)
        c[: max(1, n // 30)] += rng.uniform(-0.5, 0.5, (max(1, n // 30), 3)).astype(np.float32)
        clouds.append(c)
    lat = np.round(_cloud(rng, 600, [0, 0, 2], 0.05) * 50) / 50  # many equal keys
    clouds.append(lat.astype(np.float32))
    dup = _cloud(rng, 300, [0, 0, 2], 0.05)
    dup[100:] = dup[:200]  # every point twice or three times
    clouds.append(dup)
    clouds.append(np.tile(np.float32([[0.1, -0.2, 2.0]]), (400, 1)))  # one point repeated
    flat = _cloud(rng, 500, [0, 0, 2], 0.05)
    flat[:, 1] = 0.25  # a constant dimension
    clouds.append(flat)
    a = ea.Assoc(max_points=40000)
    for batch in (clouds, [[c] for c in clouds]):
        got = a.iforest(batch) if isinstance(batch[0], np.ndarray) else [a.iforest(b)[0] for b in batch]
        for c, g in zip(clouds, got):
            o = orc.iforest(c)
            assert np.allclose(g, o, rtol=1e-5, atol=1e-9, equal_nan=True), len(c)
            assert np.array_equal(g > 0.6, o > 0.6), len(c)


def test_iforest_one_wave_small_batches():
    """Batches whose samples all have <= 64 items run the one-wave forest kernel (k_iforest_tree<64>:
    build and score by the same wave): sizes around the register / rank-space subtree boundary
    (sample 7 / 8) and the 64-item limit (n = 128, 129), ties, duplicated and repeated points, the
    sample from the table and drawn in the kernel (sample n / 3), batched and alone."""
    rng = np.random.default_rng(0x51A11)
    clouds = []
    for n in (2, 3, 5, 14, 15, 16, 17, 18, 31, 63, 64, 65, 100, 127, 128, 129):
        c = _cloud(rng, n, [0, 0, 2], 0.05)
        c[: max(1, n // 10)] += rng.uniform(-0.5, 0.5, (max(1, n // 10), 3)).astype(np.float32)
        clouds.append(c)
    lat = np.round(_cloud(rng, 120, [0, 0, 2], 0.05) * 40) / 40  # many equal keys
    clouds.append(lat.astype(np.float32))
    dup = _cloud(rng, 90, [0, 0, 2], 0.05)
    dup[30:] = dup[:60]
    clouds.append(dup)
    clouds.append(np.tile(np.float32([[0.1, -0.2, 2.0]]), (50, 1)))  # one point repeated
    a = ea.Assoc(max_points=40000)
    for batch in (clouds, [[c] for c in clouds]):
        got = a.iforest(batch) if isinstance(batch[0], np.ndarray) else [a.iforest(b)[0] for b in batch]
        for c, g in zip(clouds, got):
            o = orc.iforest(c)
            assert np.allclose(g, o, rtol=1e-5, atol=1e-9, equal_nan=True), len(c)
            assert np.array_equal(g > 0.6, o > 0.6), len(c)
    samples = [max(1, len(c) // 3) for c in clouds]
    for c, m, g in zip(clouds, samples, a.iforest(clouds, samples=samples)):
        o = orc.iforest(c, sample=m)
        assert np.allclose(g, o, rtol=1e-5, atol=1e-9, equal_nan=True), (len(c), m)


def test_iforest_sample_table_and_drawn_paths():
    """The engine takes a forest's sample from its table (k_iforest_sample) when the cloud
    has at most IF_TAB_N = 4096 points and the sample is n / 2, and draws it in the kernel
    otherwise: both must equal the restatement. Sizes around the shuffle's 624-draw twists
    (n / 2 near 624 and 1248), odd sizes, the table's last size, one beyond it, and other
    sample sizes."""
    rng = np.random.default_rng(0x7AB)
    sizes = (1247, 1248, 1249, 2495, 2497, 4095, 4096, 4097, 5001)
    clouds = []
    for n in sizes:
        c = _cloud(rng, n, [0, 0, 2], 0.05)
        c[: n // 25] += rng.uniform(-0.5, 0.5, (n // 25, 3)).astype(np.float32)
        clouds.append(c)
    a = ea.Assoc(max_points=40000)
    for c, g in zip(clouds, a.iforest(clouds)):  # sample n / 2: table up to 4096, drawn beyond
        o = orc.iforest(c)
        assert np.allclose(g, o, rtol=1e-5, atol=1e-9), len(c)
        assert np.array_equal(g > 0.6, o > 0.6), len(c)
    sub = clouds[:4]
    samples = [len(c) // 3 for c in sub]  # drawn in the kernel whatever the size
    for c, m, g in zip(sub, samples, a.iforest(sub, samples=samples)):
        o = orc.iforest(c, sample=m)
        assert np.allclose(g, o, rtol=1e-5, atol=1e-9), (len(c), m)


def test_project_rects(frames):
    _, poses = frames
    rng = np.random.default_rng(41)
    clouds = [_cloud(rng, int(rng.integers(1, 500)), [0.2 * k - 0.5, 0.1, 2.0], 0.15) for k in range(12)]
    a = ea.Assoc()
    got, ok = a.rects(ea.camera(), poses[1], clouds)
    for c, g in zip(clouds, got):
        assert np.array_equal(g, orc.project_rect(orc.cam(), poses[1], c))
    assert ok.all()


def test_np_pairs_int32_wrap_q4():
    """NoParaDataAssociation's bounds use int products (Object.cc:905-911): m*n*(m+n+1)
    overflows int32 from m = 564 with n = 3m. Engine and oracle define the
    wrap as two's complement: a negative product gives NaN bounds (verdict 2), a product
    past 2^32 wraps positive (finite, shifted bounds). Counts and bounds must agree."""
    rng = np.random.default_rng(0x64)
    fs, os_, exp = [], [], []
    for m, n in ((564, 1692), (600, 1800), (800, 2400), (700, 900)):
        f = _cloud(rng, m, [1, 2, 3], 0.1)
        o = _cloud(rng, n, [1, 2, 3], 0.1)
        fs.append((f, np.ones(m, np.uint8)))
        os_.append((o, np.ones(n, np.uint8)))
        exp.append(orc.np_test(f, fs[-1][1], o, os_[-1][1]))
    got = ea.Assoc().np_batch(fs, os_)
    for g, o in zip(got, exp):
        assert g["verdict"] == o["verdict"] and g["m"] == o["m"] and g["n"] == o["n"]
        assert np.array_equal(g["cnt_gt"], o["cnt_gt"]) and np.array_equal(g["cnt_lt"], o["cnt_lt"])
        assert np.array_equal(g["cnt_eq"], o["cnt_eq"])
        assert np.allclose([g["r1"], g["r2"]], [o["r1"], o["r2"]], rtol=1e-6, equal_nan=True)
    assert np.isnan(exp[0]["r1"]) and exp[0]["verdict"] == 2  # 564*1692*2257 wraps negative


def test_biforest_state_per_replay_q6():
    """Object.cc's biForest is a process global that flag "None" clears for good (SURVEY
    Q6); a mono_tum process runs one flag, and a replay models one such process: a "None"
    replay launches no isolation forest, and a later "EAO" replay in the same process
    starts with biForest set, as a fresh mono_tum EAO run does."""
    frames = synth.assoc_stream(40)
    a = ea.Assoc()
    none = ea.Replay(a, "None")
    none.run(ea.Replay.pack(frames))
    prof = np.zeros(24)
    ea.lib().eao_replay_profile(none.h, ea.P(prof))
    assert prof[2] == 0  # no forest launched
    none.close()
    eao = ea.Replay(a, "EAO")
    det = eao.run(ea.Replay.pack(frames))
    ea.lib().eao_replay_profile(eao.h, ea.P(prof))
    assert prof[2] > 0
    o = orc.Replay("EAO")
    ref = []
    for i, f in enumerate(frames):
        ref.append(o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"]))
        if f["kf"]:
            o.local_mapping()
    assert np.array_equal(det, np.concatenate(ref))
