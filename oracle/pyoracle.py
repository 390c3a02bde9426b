"""ctypes binding of the CPU restatement (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker -- never by the product.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
NP_DTYPE = np.dtype([("verdict", "<i4"), ("m", "<i4"), ("n", "<i4"), ("w", "<f4", 3), ("r1", "<f4"),
                     ("r2", "<f4"), ("cnt_gt", "<f4", 3), ("cnt_lt", "<f4", 3), ("cnt_eq", "<f4", 3)])


class Cam(ctypes.Structure):
    _fields_ = [("img_w", ctypes.c_int), ("img_h", ctypes.c_int), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def use_native():
    """Switch to the -O3 -march=native build of the same sources (bench.py's timed CPU
    baseline), compiling it on this machine first; must precede the first lib() call."""
    global LIB_PATH
    native = os.path.join(HERE, "_build_native", "liboracle.so")
    if _lib is not None:
        if LIB_PATH == native:
            return LIB_PATH  # already the native build
        raise RuntimeError("pyoracle: library already loaded")
    subprocess.check_call(["make", "-s", "-j4", "-C", HERE, "native"])
    LIB_PATH = native
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_fast_atan2.restype = ctypes.c_float
        for f in ("orc_bbox_iou", "orc_bbox_former", "orc_bbox_latter"):
            getattr(_lib, f).restype = ctypes.c_float
        _lib.orc_replay_create.restype = ctypes.c_void_p
        _lib.orc_extract_match_mt.restype = ctypes.c_double
        _lib.orc_replay_destroy.argtypes = [ctypes.c_void_p]
        for f in ("orc_replay_frame", "orc_replay_local_mapping", "orc_replay_num_objects",
                  "orc_replay_object", "orc_replay_object_points", "orc_replay_update_points"):
            getattr(_lib, f).argtypes = None
    return _lib


def P(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def cam(w=640, h=480, K=(535.4, 539.2, 320.1, 247.6)):
    return Cam(w, h, *[float(k) for k in K])


def orb_params(nfeatures=1000, scale=1.2, nlevels=8):
    sc, inv, s2, is2 = [np.zeros(nlevels, np.float32) for _ in range(4)]
    q = np.zeros(nlevels, np.int32)
    umax = np.zeros(16, np.int32)
    lib().orc_orb_params(nfeatures, ctypes.c_float(scale), nlevels, P(sc), P(inv), P(s2), P(is2), P(q), P(umax))
    return dict(scale=sc, inv_scale=inv, sigma2=s2, inv_sigma2=is2, quotas=q, umax=umax)


def level_sizes(w, h, scale=1.2, nlevels=8):
    s = np.zeros(2 * nlevels, np.int32)
    lib().orc_orb_level_sizes(w, h, ctypes.c_float(scale), nlevels, P(s))
    return [(int(s[2 * i]), int(s[2 * i + 1])) for i in range(nlevels)]


def pyramid(img, scale=1.2, nlevels=8):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    sizes = level_sizes(w, h, scale, nlevels)
    out = np.zeros(sum(a * b for a, b in sizes), np.uint8)
    lib().orc_orb_pyramid(P(img), w, h, ctypes.c_float(scale), nlevels, P(out))
    levels, o = [], 0
    for lw, lh in sizes:
        levels.append(out[o:o + lw * lh].reshape(lh, lw))
        o += lw * lh
    return levels


def extract(img, nfeatures=1000, scale=1.2, nlevels=8, ini=20, mn=7):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = nfeatures + 64 * nlevels + 64
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int()
    rc = lib().orc_orb_extract(P(img), w, h, nfeatures, ctypes.c_float(scale), nlevels, ini, mn, P(kps), P(desc),
                               cap, ctypes.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def extract_match_mt(frames, Tcw, has, mpos, scales, threads, th=15, check_ori=1, nfeatures=1000, scale=1.2,
                     nlevels=8, ini=20, mn=7, c=None):
    """Frame-parallel extraction of frames (n, h, w) then motion matching of every pair
    (t-1, t) over `threads` std::threads (baseline_mt.cpp); returns (seconds, kps, desc,
    nkp, match, nmatch). has/mpos: map state of each frame's keypoints, cap slots."""
    frames = np.ascontiguousarray(frames, np.uint8)
    n, h, w = frames.shape
    cap = has.shape[1]  # keypoint slots per frame: the caller's map-state row stride
    assert has.shape == (n, cap) and mpos.shape == (n, cap, 3)
    kps = np.zeros((n, cap), KP_DTYPE)
    desc = np.zeros((n, cap, 32), np.uint8)
    nkp = np.zeros(n, np.int32)
    match = np.full((n, cap), -1, np.int32)
    nmatch = np.zeros(n, np.int32)
    c = cam(w, h) if c is None else c
    sec = lib().orc_extract_match_mt(P(frames), n, w, h, nfeatures, ctypes.c_float(scale), nlevels, ini, mn,
                                     ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)),
                                     P(np.ascontiguousarray(has, np.uint8)), P(np.ascontiguousarray(mpos, np.float32)),
                                     ctypes.c_float(th), int(check_ori), P(np.ascontiguousarray(scales, np.float32)),
                                     cap, int(threads), P(kps), P(desc), P(nkp), P(match), P(nmatch))
    return sec, kps, desc, nkp, match, nmatch


def color_to_gray(img, rgb=True):
    """cvtColor(CV_RGB2GRAY / CV_BGR2GRAY [A]) of an (h, w, 3|4) u8 image."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w, cn = img.shape
    out = np.zeros((h, w), np.uint8)
    lib().orc_color_to_gray(P(img), w, h, w * cn, cn, 1 if rgb else 0, P(out))
    return out


def blur7(img):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros_like(img)
    lib().orc_gaussian_blur7(P(img), img.shape[1], img.shape[0], P(out))
    return out


def fast_atan2(y, x):
    return lib().orc_fast_atan2(ctypes.c_float(y), ctypes.c_float(x))


def hamming(a, b):
    return lib().orc_descriptor_distance(P(np.ascontiguousarray(a, np.uint8)), P(np.ascontiguousarray(b, np.uint8)))


def match_motion(c, Tcw, th, check_ori, last_kps, has_mp, mp_pos, mp_desc, cur_kps, cur_desc, scales):
    out = np.full(len(cur_kps), -1, np.int32)
    n = lib().orc_search_by_projection_motion(
        ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)), ctypes.c_float(th), int(check_ori),
        len(last_kps), P(last_kps), P(np.ascontiguousarray(has_mp, np.uint8)),
        P(np.ascontiguousarray(mp_pos, np.float32)), P(np.ascontiguousarray(mp_desc, np.uint8)), len(cur_kps),
        P(cur_kps), P(np.ascontiguousarray(cur_desc, np.uint8)), len(scales),
        P(np.ascontiguousarray(scales, np.float32)), P(out))
    return n, out


def frustum(c, Tcw, pos, normal, mind, maxd, vclim, logsf):
    n = len(pos)
    inv = np.zeros(n, np.uint8)
    proj = np.zeros((n, 2), np.float32)
    lvl = np.zeros(n, np.int32)
    vc = np.zeros(n, np.float32)
    cnt = lib().orc_is_in_frustum(ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)), n,
                                  P(np.ascontiguousarray(pos, np.float32)),
                                  P(np.ascontiguousarray(normal, np.float32)),
                                  P(np.ascontiguousarray(mind, np.float32)),
                                  P(np.ascontiguousarray(maxd, np.float32)), ctypes.c_float(vclim),
                                  ctypes.c_float(logsf), P(inv), P(proj), P(lvl), P(vc))
    return cnt, inv, proj, lvl, vc


def match_local(c, th, nnratio, inv, proj, lvl, vc, mp_desc, cur_kps, cur_desc, pre, scales):
    out = np.full(len(cur_kps), -1, np.int32)
    n = lib().orc_search_by_projection_local(
        ctypes.byref(c), ctypes.c_float(th), ctypes.c_float(nnratio), len(inv), P(inv), P(proj), P(lvl), P(vc),
        P(np.ascontiguousarray(mp_desc, np.uint8)), len(cur_kps), P(cur_kps),
        P(np.ascontiguousarray(cur_desc, np.uint8)), P(pre) if pre is not None else None, len(scales),
        P(np.ascontiguousarray(scales, np.float32)), P(out))
    return n, out


def match_keyframe(c, Tcw, th, orb_dist, check_ori, kf_kps, valid, pos, desc, mind, maxd, logsf,
                   cur_kps, cur_desc, pre, scales):
    """SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist), ORBmatcher.cc:1472-1599."""
    out = np.full(len(cur_kps), -1, np.int32)
    n = lib().orc_search_by_projection_keyframe(
        ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)), ctypes.c_float(th), int(orb_dist),
        int(check_ori), len(kf_kps), P(kf_kps), P(np.ascontiguousarray(valid, np.uint8)),
        P(np.ascontiguousarray(pos, np.float32)), P(np.ascontiguousarray(desc, np.uint8)),
        P(np.ascontiguousarray(mind, np.float32)), P(np.ascontiguousarray(maxd, np.float32)),
        ctypes.c_float(logsf), len(cur_kps), P(cur_kps), P(np.ascontiguousarray(cur_desc, np.uint8)),
        P(np.ascontiguousarray(pre, np.int32)) if pre is not None else None, len(scales),
        P(np.ascontiguousarray(scales, np.float32)), P(out))
    return n, out


def match_init(c, nnratio, check_ori, kps1, desc1, kps2, desc2, prev_xy, window):
    m12 = np.full(len(kps1), -1, np.int32)
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    n = lib().orc_search_for_initialization(ctypes.byref(c), ctypes.c_float(nnratio), int(check_ori), len(kps1),
                                            P(kps1), P(np.ascontiguousarray(desc1, np.uint8)), len(kps2), P(kps2),
                                            P(np.ascontiguousarray(desc2, np.uint8)), P(prev), window, P(m12))
    return n, m12, prev


def np_test(fpts, fvalid, opts, ovalid):
    fpts = np.ascontiguousarray(fpts, np.float32)
    opts = np.ascontiguousarray(opts, np.float32)
    out = np.zeros(1, NP_DTYPE)
    lib().orc_np_test(len(fpts), P(fpts), P(None if fvalid is None else np.ascontiguousarray(fvalid, np.uint8)),
                      len(opts), P(opts), P(None if ovalid is None else np.ascontiguousarray(ovalid, np.uint8)),
                      P(out))
    return out[0]


def iforest(pts, trees=50, seed=12345, sample=None):
    pts = np.ascontiguousarray(pts, np.float32)
    n = len(pts)
    sample = n // 2 if sample is None else sample
    s = np.zeros(n, np.float64)
    rc = lib().orc_iforest_scores(P(pts), n, trees, seed, sample, P(s))
    assert rc == 0
    return s


def mt_stream(seed, n):
    o = np.zeros(n, np.uint32)
    lib().orc_mt19937_stream(ctypes.c_uint32(seed), n, P(o))
    return o


def lemire(seed, n, rng):
    o = np.zeros(n, np.uint32)
    lib().orc_lemire_u32(ctypes.c_uint32(seed), n, ctypes.c_uint32(rng), P(o))
    return o


def shuffle(seed, n):
    o = np.zeros(n, np.uint32)
    lib().orc_shuffle_ids(ctypes.c_uint32(seed), n, P(o))
    return o


def canonical(seed, n, lo, hi):
    o = np.zeros(n, np.float32)
    lib().orc_canonical_float(ctypes.c_uint32(seed), n, ctypes.c_float(lo), ctypes.c_float(hi), P(o))
    return o


def bbox(fn, a, b):
    a = np.asarray(a, np.int32)
    b = np.asarray(b, np.int32)
    return getattr(lib(), "orc_bbox_" + fn)(P(a), P(b))


def project_rect(c, Tcw, pts):
    pts = np.ascontiguousarray(pts, np.float32)
    r = np.zeros(4, np.int32)
    rc = lib().orc_project_rect(ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)), len(pts), P(pts), P(r))
    return r if rc == 0 else None


class Replay:
    """CPU restatement of the association replay (oracle/assoc_ref.cpp)."""

    def __init__(self, flag="iForest", w=640, h=480, K=(535.4, 539.2, 320.1, 247.6)):
        K4 = np.asarray(K, np.float32)
        self.h = lib().orc_replay_create(flag.encode(), w, h, P(K4))

    def close(self):
        if self.h:
            lib().orc_replay_destroy(self.h)
            self.h = None

    __del__ = close

    def lines(self, sets):
        """Stage frame line segments (list of (L, 4) arrays, one per upcoming frame)."""
        nl = np.array([len(np.asarray(x).reshape(-1, 4)) for x in sets], np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(x, np.float32).reshape(-1, 4) for x in sets])
                                    if len(sets) else np.zeros((0, 4), np.float32), np.float32)
        lib().orc_replay_lines(ctypes.c_void_p(self.h), len(sets), P(nl), P(flat))

    def frame(self, fid, T, boxes, ids, pos, uv, bad=None, lines=None):
        boxes = np.ascontiguousarray(boxes, np.int32).reshape(-1, 5)
        out = np.zeros((len(boxes), 4), np.int32)
        bad = np.zeros(len(ids), np.uint8) if bad is None else np.ascontiguousarray(bad, np.uint8)
        if lines is not None:
            self.lines([lines])
        lib().orc_replay_frame(ctypes.c_void_p(self.h), int(fid), P(np.ascontiguousarray(T, np.float32)),
                               len(boxes), P(boxes), len(ids), P(np.ascontiguousarray(ids, np.int32)),
                               P(np.ascontiguousarray(pos, np.float32)), P(np.ascontiguousarray(uv, np.float32)),
                               P(bad), P(out))
        return out

    def local_mapping(self):
        lib().orc_replay_local_mapping(ctypes.c_void_p(self.h))

    def update_points(self, ids, pos=None, bad=None):
        """LocalMapping's map-point changes (BA positions, culled / replaced points as bad)."""
        ids = np.ascontiguousarray(ids, np.int32)
        pos = None if pos is None else np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        bad = None if bad is None else np.ascontiguousarray(bad, np.uint8)
        lib().orc_replay_update_points(ctypes.c_void_p(self.h), len(ids), P(ids), P(pos), P(bad))

    def step(self, fid, f):
        """One frame of a stream dict (synth): the frame, its map-point record, its local mapping."""
        out = self.frame(fid, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        if "upd_ids" in f:
            self.update_points(f["upd_ids"], f["upd_pos"], f["upd_bad"])
        if f["kf"]:
            self.local_mapping()
        return out

    def objects(self):
        n = lib().orc_replay_num_objects(ctypes.c_void_p(self.h))
        ints = np.zeros((n, 8), np.int32)
        fl = np.zeros((n, 20), np.float32)
        pts = []
        for i in range(n):
            lib().orc_replay_object(ctypes.c_void_p(self.h), i, P(ints[i]), P(fl[i]))
            ids = np.zeros(max(1, ints[i, 4]), np.int32)
            k = lib().orc_replay_object_points(ctypes.c_void_p(self.h), i, P(ids), len(ids))
            pts.append(ids[:k].copy())
        return ints, fl, pts


# ---- per-frame line detection (lines_ref.cpp)
def line_maps(gray):
    """(blur u8, dx i16, dy i16, g i16, dir u8) of EDLine on GaussianBlur(5x5, 1)."""
    g8 = np.ascontiguousarray(gray, np.uint8)
    h, w = g8.shape
    blur = np.zeros((h, w), np.uint8)
    dx, dy, gg = (np.zeros((h, w), np.int16) for _ in range(3))
    dr = np.zeros((h, w), np.uint8)
    lib().orc_line_maps(P(g8), w, h, P(blur), P(dx), P(dy), P(gg), P(dr))
    return blur, dx, dy, gg, dr


def edge_chains(gray, cap_px=1 << 18, cap_edges=1 << 14):
    """EdgeDrawing chains: (xy [n_px][2] u32, sid [n_edges + 1] u32)."""
    g8 = np.ascontiguousarray(gray, np.uint8)
    h, w = g8.shape
    xy = np.zeros((cap_px, 2), np.uint32)
    sid = np.zeros(cap_edges + 1, np.uint32)
    npx, ne = ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_edge_chains(P(g8), w, h, P(xy), cap_px, P(sid), cap_edges, ctypes.byref(npx), ctypes.byref(ne))
    assert rc == 0 and npx.value <= cap_px and ne.value <= cap_edges
    return xy[:npx.value].copy(), sid[:ne.value + 1].copy()


def ed_edge_map(gray, grad_th, anchor_th, scan, min_line_len, gdiv, fit_err=1.6):
    """The restatement's kept EdgeDrawing chains as a 255/0 map under other knobs (pinning only)."""
    g8 = np.ascontiguousarray(gray, np.uint8)
    h, w = g8.shape
    ip = np.array([grad_th, anchor_th, scan, min_line_len, gdiv, 1], np.int32)
    m = np.zeros((h, w), np.uint8)
    n = ctypes.c_int()
    rc = lib().orc_ed_edge_map(P(g8), w, h, P(ip), ctypes.c_double(fit_err), P(m), ctypes.byref(n))
    assert rc == 0, rc
    return m, n.value


def ed_segments(gray, grad_th, anchor_th, scan, min_line_len, gdiv, fit_err=1.6, validate=1, cap=1 << 14):
    """EDline's raw segments [n][4] (x1, y1, x2, y2) under other knobs (pinning only)."""
    g8 = np.ascontiguousarray(gray, np.uint8)
    h, w = g8.shape
    ip = np.array([grad_th, anchor_th, scan, min_line_len, gdiv, validate], np.int32)
    out = np.zeros((cap, 4), np.float32)
    n = ctypes.c_int()
    rc = lib().orc_ed_segments(P(g8), w, h, P(ip), ctypes.c_double(fit_err), P(out), cap, ctypes.byref(n))
    assert rc == 0, rc
    return out[:n.value].copy()


def edlines(gray, min_length=50.0, cap=4096):
    """detect_raw_lines + filter_lines: [n][6] float32 (sx, sy, ex, ey, angle, length)."""
    g8 = np.ascontiguousarray(gray, np.uint8)
    h, w = g8.shape
    out = np.zeros((cap, 6), np.float32)
    n = ctypes.c_int()
    rc = lib().orc_edlines(P(g8), w, h, ctypes.c_float(min_length), P(out), cap, ctypes.byref(n))
    assert rc == 0, rc
    return out[:n.value].copy()


def edlines_color(img, min_length=50.0, cap=4096):
    """The same on the colour frame detectImpl receives ([h][w][3 or 4] BGR bytes, converted with
    COLOR_BGR2GRAY first; [h][w] is gray)."""
    a = np.ascontiguousarray(img, np.uint8)
    h, w = a.shape[:2]
    cn = 1 if a.ndim == 2 else a.shape[2]
    out = np.zeros((cap, 6), np.float32)
    n = ctypes.c_int()
    rc = lib().orc_edlines_color(P(a), w, h, w * cn, cn, ctypes.c_float(min_length), P(out), cap, ctypes.byref(n))
    assert rc == 0, rc
    return out[:n.value].copy()


def pose_optimization(c, Tcw, kps_un, has_mp, mp_pos, inv_level_sigma2):
    """Optimizer::PoseOptimization (monocular): -> (n_inliers, Tcw_out [4][4], outlier u8[n])."""
    n = len(kps_un)
    To = np.zeros((4, 4), np.float32)
    out = np.zeros(n, np.uint8)
    ni = ctypes.c_int()
    rc = lib().orc_pose_optimization(ctypes.byref(c), P(np.ascontiguousarray(Tcw, np.float32)), n,
                                     P(np.ascontiguousarray(kps_un)), P(np.ascontiguousarray(has_mp, np.uint8)),
                                     P(np.ascontiguousarray(mp_pos, np.float32)),
                                     P(np.ascontiguousarray(inv_level_sigma2, np.float32)), P(To), P(out),
                                     ctypes.byref(ni))
    assert rc == 0
    return ni.value, To, out


class Vocab:
    """orc_vocab_create over a tools/synth.vocabulary dict (arrays kept alive here)."""

    def __init__(self, voc):
        self.voc = {k: np.ascontiguousarray(voc[k]) for k in ("desc", "parent", "word", "weight")}
        lib().orc_vocab_create.restype = ctypes.c_void_p
        self.h = ctypes.c_void_p(lib().orc_vocab_create(len(self.voc["parent"]), P(self.voc["desc"]),
                                                        P(self.voc["parent"]), P(self.voc["word"]),
                                                        P(self.voc["weight"]), int(voc["L"])))

    def __del__(self):
        if self.h:
            lib().orc_vocab_destroy(self.h)
            self.h = None


def bow_transform(voc, desc, levelsup=4):
    """DBoW2 transform (TF_IDF + L1): -> (word_ids, word_weights, node_ids, node_start, node_feats).
    voc: a Vocab (or a synth.vocabulary dict, wrapped per call)."""
    if not isinstance(voc, Vocab):
        voc = Vocab(voc)
    n = len(desc)
    wid = np.zeros(max(n, 1), np.int32)
    ww = np.zeros(max(n, 1), np.float64)
    nid = np.zeros(max(n, 1), np.int32)
    ns = np.zeros(n + 2, np.int32)
    nf = np.zeros(max(n, 1), np.int32)
    nw, nn = ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_bow_transform(voc.h, n, P(np.ascontiguousarray(desc, np.uint8)),
                                 levelsup, P(wid), P(ww), ctypes.byref(nw), P(nid), P(ns), P(nf),
                                 ctypes.byref(nn))
    assert rc == 0
    k = nn.value
    return wid[:nw.value].copy(), ww[:nw.value].copy(), nid[:k].copy(), ns[:k + 1].copy(), nf[:ns[k]].copy()


def search_by_bow(nnratio, check_ori, kf_kps, kf_desc, kf_valid, kf_fv, f_kps, f_desc, f_fv):
    """SearchByBoW(KF, F): fv = (node_ids, node_start, node_feats); -> (nmatches, f_match)."""
    m = np.full(len(f_kps), -1, np.int32)
    a = [np.ascontiguousarray(x, np.int32) for x in kf_fv]
    b = [np.ascontiguousarray(x, np.int32) for x in f_fv]
    n = lib().orc_search_by_bow(ctypes.c_float(nnratio), int(check_ori), len(kf_kps), P(np.ascontiguousarray(kf_kps)),
                                P(np.ascontiguousarray(kf_desc, np.uint8)), P(np.ascontiguousarray(kf_valid, np.uint8)),
                                len(a[0]), P(a[0]), P(a[1]), P(a[2]), len(f_kps), P(np.ascontiguousarray(f_kps)),
                                P(np.ascontiguousarray(f_desc, np.uint8)), len(b[0]), P(b[0]), P(b[1]), P(b[2]), P(m))
    return n, m


def search_by_bow_kf(nnratio, check_ori, kps1, desc1, valid1, fv1, kps2, desc2, valid2, fv2):
    """SearchByBoW(KF1, KF2): fv = (node_ids, node_start, node_feats); -> (nmatches, match12)."""
    m = np.full(len(kps1), -1, np.int32)
    a = [np.ascontiguousarray(x, np.int32) for x in fv1]
    b = [np.ascontiguousarray(x, np.int32) for x in fv2]
    n = lib().orc_search_by_bow_kf(ctypes.c_float(nnratio), int(check_ori), len(kps1), P(np.ascontiguousarray(kps1)),
                                   P(np.ascontiguousarray(desc1, np.uint8)), P(np.ascontiguousarray(valid1, np.uint8)),
                                   len(a[0]), P(a[0]), P(a[1]), P(a[2]), len(kps2), P(np.ascontiguousarray(kps2)),
                                   P(np.ascontiguousarray(desc2, np.uint8)), P(np.ascontiguousarray(valid2, np.uint8)),
                                   len(b[0]), P(b[0]), P(b[1]), P(b[2]), P(m))
    return n, m
