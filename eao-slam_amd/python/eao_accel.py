"""ctypes binding of the MI355X engine's C ABI (include/eao_accel.h).

This is a thin harness binding used by tests/, bench.py and __graft_entry__;
the product is the shared library eao-slam_amd/lib/libeao_accel.so. There is
no fallback: if the library or a gfx950 device is missing, calls raise.
"""
import atexit
import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EAO_ACCEL_LIB") or os.path.join(os.path.dirname(HERE), "lib", "libeao_accel.so")

EAO_OK, EAO_E_ARG, EAO_E_NODEVICE, EAO_E_HIP, EAO_E_CAPACITY, EAO_E_STATE = 0, -1, -2, -3, -4, -5

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
NP_DTYPE = np.dtype([("verdict", "<i4"), ("m", "<i4"), ("n", "<i4"), ("w", "<f4", 3), ("r1", "<f4"),
                     ("r2", "<f4"), ("cnt_gt", "<f4", 3), ("cnt_lt", "<f4", 3), ("cnt_eq", "<f4", 3)])


class EaoError(RuntimeError):
    pass


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int32), ("scale_factor", ctypes.c_float),
                ("nlevels", ctypes.c_int32), ("ini_th_fast", ctypes.c_int32),
                ("min_th_fast", ctypes.c_int32), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("max_batch", ctypes.c_int32)]


class Camera(ctypes.Structure):
    _fields_ = [("img_w", ctypes.c_int32), ("img_h", ctypes.c_int32), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EaoError("engine library not built: %s (run __graft_entry__.build())" % LIB_PATH)
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.eao_version.restype = ctypes.c_char_p
        _lib.eao_last_error.restype = ctypes.c_char_p
    return _lib


def P(a):
    """numpy array -> void pointer (None passes NULL)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


def check(rc, what):
    if rc < 0:
        raise EaoError("%s failed (%d): %s" % (what, rc, lib().eao_last_error().decode()))
    return rc


# Handle lifetime: every handle keeps the destroy function it needs (no lookup through the
# module at interpreter teardown) and is closed at exit in dependency order (replays before
# the association engine they return their resources to).
_open_handles = weakref.WeakSet()


class _Handle:
    _DESTROY = None
    _EXIT_ORDER = 1
    h = None

    def _opened(self):
        self._destroy = getattr(lib(), self._DESTROY)
        _open_handles.add(self)

    def close(self):
        h = self.h
        if h:
            self.h = ctypes.c_void_p()
            self._destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- nothing to report to at collection time
            pass


@atexit.register
def _close_all():
    for o in sorted(list(_open_handles), key=lambda x: x._EXIT_ORDER):
        try:
            o.close()
        except Exception:  # noqa: BLE001
            pass


def rccl_unique_id():
    """eao_rccl_unique_id: 128-byte RCCL communicator id (one rank creates it)."""
    out = np.zeros(128, np.uint8)
    check(lib().eao_rccl_unique_id(P(out)), "eao_rccl_unique_id")
    return out.tobytes()


def rccl_selftest(device=0, nbytes=1000):
    """eao_rccl_selftest: one-rank RCCL all-gathers through the replay's exchanger."""
    check(lib().eao_rccl_selftest(int(device), int(nbytes)), "eao_rccl_selftest")


def lane_selftest(device=0):
    """eao_lane_selftest: the HSA launch lanes' completion markers, barrier lifetimes and ring-end
    commits; returns the packets written."""
    out = np.zeros(1, np.int32)
    check(lib().eao_lane_selftest(int(device), P(out)), "eao_lane_selftest")
    return int(out[0])


def device_ok(dev=0):
    return bool(lib().eao_device_ok(dev))


def camera(w=640, h=480, K=(535.4, 539.2, 320.1, 247.6)):
    return Camera(w, h, *[float(k) for k in K])


class Orb(_Handle):
    """ORBextractor replacement (reference src/ORBextractor.cc)."""
    _DESTROY = "eao_orb_destroy"

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7,
                 width=640, height=480, max_batch=1, device=0):
        self.p = OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th, width, height, max_batch)
        self.h = ctypes.c_void_p()
        check(lib().eao_orb_create(ctypes.byref(self.p), device, ctypes.byref(self.h)), "eao_orb_create")
        self._opened()
        self.nlevels = nlevels
        self.cap = check(lib().eao_orb_frame_capacity(self.h), "eao_orb_frame_capacity")


    def scale_tables(self):
        t = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        check(lib().eao_orb_scale_tables(self.h, *[P(x) for x in t]), "scale_tables")
        return t

    def quotas(self):
        q = np.zeros(self.nlevels, np.int32)
        check(lib().eao_orb_level_quotas(self.h, P(q)), "level_quotas")
        return q

    def extract(self, gray):
        gray = np.ascontiguousarray(gray, np.uint8)
        h, w = gray.shape
        kps = np.zeros(self.cap, KP_DTYPE)
        desc = np.zeros((self.cap, 32), np.uint8)
        n = ctypes.c_int()
        check(lib().eao_orb_extract(self.h, P(gray), w, h, w, P(kps), P(desc), self.cap, ctypes.byref(n)),
              "eao_orb_extract")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def pyramid(self, gray):
        gray = np.ascontiguousarray(gray, np.uint8)
        tot = 0
        sizes = []
        for l in range(self.nlevels):
            s = 1.0
            for _ in range(l):
                s = float(np.float32(np.float64(np.float32(s)) * np.float64(np.float32(self.p.scale_factor))))
            inv = np.float32(1.0) / np.float32(s)
            lw = int(np.rint(np.float32(gray.shape[1]) * inv))
            lh = int(np.rint(np.float32(gray.shape[0]) * inv))
            sizes.append((lw, lh))
            tot += lw * lh
        out = np.zeros(tot, np.uint8)
        check(lib().eao_orb_debug_pyramid(self.h, P(gray), P(out)), "debug_pyramid")
        levels, o = [], 0
        for lw, lh in sizes:
            levels.append(out[o:o + lw * lh].reshape(lh, lw))
            o += lw * lh
        return levels

    def set_timing(self, on=True):
        check(lib().eao_orb_set_timing(self.h, int(on)), "eao_orb_set_timing")

    def stage_ms(self):
        ms = np.zeros(8, np.float32)
        n = check(lib().eao_orb_stage_ms(self.h, P(ms), len(ms)), "eao_orb_stage_ms")
        return ms[:n]

    def extract_batch_device(self, frames_ptr, nframes, pitch, kps_ptr, desc_ptr, counts_ptr, cap, stream=None):
        check(lib().eao_orb_extract_batch_device(self.h, ctypes.c_void_p(frames_ptr), nframes, pitch,
                                                 ctypes.c_void_p(kps_ptr), ctypes.c_void_p(desc_ptr),
                                                 ctypes.c_void_p(counts_ptr), cap,
                                                 ctypes.c_void_p(stream) if stream else None),
              "eao_orb_extract_batch_device")


def color_to_gray_batch_device(color_ptr, nframes, w, h, pitch, channels, rgb, gray_ptr, gray_pitch, device=0,
                               stream=None):
    """eao_color_to_gray_batch_device: cvtColor(CV_RGB2GRAY | CV_BGR2GRAY [A]) of HBM-resident frames."""
    v = ctypes.c_void_p
    check(lib().eao_color_to_gray_batch_device(v(color_ptr), nframes, w, h, pitch, channels, 1 if rgb else 0,
                                               v(gray_ptr), gray_pitch, device, v(stream) if stream else None),
          "eao_color_to_gray_batch_device")


class Matcher(_Handle):
    """ORBmatcher + Frame grid replacement (reference src/ORBmatcher.cc, src/Frame.cc)."""
    _DESTROY = "eao_matcher_destroy"

    def __init__(self, max_kps=4096, max_batch=2, device=0):
        self.h = ctypes.c_void_p()
        check(lib().eao_matcher_create(device, max_kps, max_batch, ctypes.byref(self.h)), "eao_matcher_create")
        self._opened()


    def motion(self, cam, Tcw, th, check_ori, last_kps, has_mp, mp_pos, mp_desc, cur_kps, cur_desc, scales):
        cur_match = np.full(len(cur_kps), -1, np.int32)
        T = np.ascontiguousarray(Tcw, np.float32)
        n = check(lib().eao_match_motion(self.h, ctypes.byref(cam), P(T), ctypes.c_float(th), int(check_ori),
                                         len(last_kps), P(last_kps), P(np.ascontiguousarray(has_mp, np.uint8)),
                                         P(np.ascontiguousarray(mp_pos, np.float32)),
                                         P(np.ascontiguousarray(mp_desc, np.uint8)), len(cur_kps), P(cur_kps),
                                         P(np.ascontiguousarray(cur_desc, np.uint8)), len(scales),
                                         P(np.ascontiguousarray(scales, np.float32)), P(cur_match)),
                  "eao_match_motion")
        return n, cur_match

    def frustum(self, cam, Tcw, pos, normal, mind, maxd, vclim, logsf):
        n = len(pos)
        inv = np.zeros(n, np.uint8)
        proj = np.zeros((n, 2), np.float32)
        lvl = np.zeros(n, np.int32)
        vc = np.zeros(n, np.float32)
        c = check(lib().eao_is_in_frustum(self.h, ctypes.byref(cam), P(np.ascontiguousarray(Tcw, np.float32)), n,
                                          P(np.ascontiguousarray(pos, np.float32)),
                                          P(np.ascontiguousarray(normal, np.float32)),
                                          P(np.ascontiguousarray(mind, np.float32)),
                                          P(np.ascontiguousarray(maxd, np.float32)), ctypes.c_float(vclim),
                                          ctypes.c_float(logsf), P(inv), P(proj), P(lvl), P(vc)),
                  "eao_is_in_frustum")
        return c, inv, proj, lvl, vc

    def local(self, cam, th, nnratio, inv, proj, lvl, vc, mp_desc, cur_kps, cur_desc, pre, scales):
        out = np.full(len(cur_kps), -1, np.int32)
        n = check(lib().eao_match_local(self.h, ctypes.byref(cam), ctypes.c_float(th), ctypes.c_float(nnratio),
                                        len(inv), P(inv), P(proj), P(lvl), P(vc),
                                        P(np.ascontiguousarray(mp_desc, np.uint8)), len(cur_kps), P(cur_kps),
                                        P(np.ascontiguousarray(cur_desc, np.uint8)),
                                        P(pre) if pre is not None else None, len(scales),
                                        P(np.ascontiguousarray(scales, np.float32)), P(out)),
                  "eao_match_local")
        return n, out

    def keyframe(self, cam, Tcw, th, orb_dist, check_ori, kf_kps, valid, pos, desc, mind, maxd, logsf,
                 cur_kps, cur_desc, pre, scales):
        """SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1472-1599)."""
        out = np.full(len(cur_kps), -1, np.int32)
        n = check(lib().eao_match_keyframe(
            self.h, ctypes.byref(cam), P(np.ascontiguousarray(Tcw, np.float32)), ctypes.c_float(th), int(orb_dist),
            int(check_ori), len(kf_kps), P(kf_kps), P(np.ascontiguousarray(valid, np.uint8)),
            P(np.ascontiguousarray(pos, np.float32)), P(np.ascontiguousarray(desc, np.uint8)),
            P(np.ascontiguousarray(mind, np.float32)), P(np.ascontiguousarray(maxd, np.float32)),
            ctypes.c_float(logsf), len(cur_kps), P(cur_kps), P(np.ascontiguousarray(cur_desc, np.uint8)),
            P(np.ascontiguousarray(pre, np.int32)) if pre is not None else None, len(scales),
            P(np.ascontiguousarray(scales, np.float32)), P(out)), "eao_match_keyframe")
        return n, out

    def init(self, cam, nnratio, check_ori, kps1, desc1, kps2, desc2, prev_xy, window):
        m12 = np.full(len(kps1), -1, np.int32)
        prev = np.ascontiguousarray(prev_xy, np.float32).copy()
        n = check(lib().eao_match_init(self.h, ctypes.byref(cam), ctypes.c_float(nnratio), int(check_ori),
                                       len(kps1), P(kps1), P(np.ascontiguousarray(desc1, np.uint8)), len(kps2),
                                       P(kps2), P(np.ascontiguousarray(desc2, np.uint8)), P(prev), window, P(m12)),
                  "eao_match_init")
        return n, m12, prev

    def hamming(self, q, t, qi, ti):
        out = np.zeros(len(qi), np.int32)
        check(lib().eao_hamming_pairs(self.h, P(np.ascontiguousarray(q, np.uint8)), len(q),
                                      P(np.ascontiguousarray(t, np.uint8)), len(t),
                                      P(np.ascontiguousarray(qi, np.int32)), P(np.ascontiguousarray(ti, np.int32)),
                                      len(qi), P(out)), "eao_hamming_pairs")
        return out

    def motion_batch_device(self, cam, nframes, cap, T_ptr, th, check_ori, kps_ptr, desc_ptr, counts_ptr,
                            has_mp_ptr, mp_pos_ptr, mp_desc_ptr, scales, match_ptr, nmatch_ptr, stream=None):
        sc = np.ascontiguousarray(scales, np.float32)
        v = ctypes.c_void_p
        check(lib().eao_match_motion_batch_device(self.h, ctypes.byref(cam), nframes, cap, v(T_ptr),
                                                  ctypes.c_float(th), int(check_ori), v(kps_ptr), v(desc_ptr),
                                                  v(counts_ptr), v(has_mp_ptr), v(mp_pos_ptr), v(mp_desc_ptr),
                                                  len(sc), P(sc), v(match_ptr), v(nmatch_ptr),
                                                  v(stream) if stream else None),
              "eao_match_motion_batch_device")


    # batched HBM-resident single-frame searches: the arguments are device pointers
    # (ints), slot strides q_cap / cap; see include/eao_accel.h
    def local_batch_device(self, cam, nsearch, th, nnratio, mp_cap, n_mp, inv, proj, lvl, vc, mp_desc, cap, n_cur,
                           cur_kps, cur_desc, pre, scales, match, nmatch, stream=None):
        sc = np.ascontiguousarray(scales, np.float32)
        v = ctypes.c_void_p
        check(lib().eao_match_local_batch_device(
            self.h, ctypes.byref(cam), nsearch, ctypes.c_float(th), ctypes.c_float(nnratio), mp_cap, v(n_mp), v(inv),
            v(proj), v(lvl), v(vc), v(mp_desc), cap, v(n_cur), v(cur_kps), v(cur_desc), v(pre) if pre else None,
            len(sc), P(sc), v(match), v(nmatch), v(stream) if stream else None), "eao_match_local_batch_device")

    def keyframe_batch_device(self, cam, nsearch, T, th, orb_dist, check_ori, kf_cap, n_kf, kf_kps, valid, pos, desc,
                              mind, maxd, logsf, cap, n_cur, cur_kps, cur_desc, pre, scales, match, nmatch,
                              stream=None):
        sc = np.ascontiguousarray(scales, np.float32)
        v = ctypes.c_void_p
        check(lib().eao_match_keyframe_batch_device(
            self.h, ctypes.byref(cam), nsearch, v(T), ctypes.c_float(th), int(orb_dist), int(check_ori), kf_cap,
            v(n_kf), v(kf_kps), v(valid), v(pos), v(desc), v(mind), v(maxd), ctypes.c_float(logsf), cap, v(n_cur),
            v(cur_kps), v(cur_desc), v(pre) if pre else None, len(sc), P(sc), v(match), v(nmatch),
            v(stream) if stream else None), "eao_match_keyframe_batch_device")

    def init_batch_device(self, cam, nsearch, nnratio, check_ori, cap1, n1, kps1, desc1, cap2, n2, kps2, desc2, prev,
                          window, m12, nmatch, stream=None):
        v = ctypes.c_void_p
        check(lib().eao_match_init_batch_device(
            self.h, ctypes.byref(cam), nsearch, ctypes.c_float(nnratio), int(check_ori), cap1, v(n1), v(kps1),
            v(desc1), cap2, v(n2), v(kps2), v(desc2), v(prev), int(window), v(m12), v(nmatch),
            v(stream) if stream else None), "eao_match_init_batch_device")


class Pose(_Handle):
    """Optimizer::PoseOptimization replacement (reference src/Optimizer.cc:243-457), monocular edges."""
    _DESTROY = "eao_pose_destroy"

    def __init__(self, max_kps=4096, max_batch=1, device=0):
        self.h = ctypes.c_void_p()
        check(lib().eao_pose_create(device, max_kps, max_batch, ctypes.byref(self.h)), "eao_pose_create")
        self._opened()


    def optimize(self, cam, Tcw, kps_un, has_mp, mp_pos, inv_level_sigma2, outlier=None):
        """-> (n_inliers, Tcw_out [4][4] float32, outlier u8[n])."""
        n = len(kps_un)
        T = np.ascontiguousarray(Tcw, np.float32)
        To = np.zeros((4, 4), np.float32)
        out = np.zeros(n, np.uint8) if outlier is None else np.array(outlier, np.uint8)
        inv = np.ascontiguousarray(inv_level_sigma2, np.float32)
        ni = ctypes.c_int32()
        check(lib().eao_pose_optimization(self.h, ctypes.byref(cam), P(T), n, P(np.ascontiguousarray(kps_un)),
                                          P(np.ascontiguousarray(has_mp, np.uint8)),
                                          P(np.ascontiguousarray(mp_pos, np.float32)), P(inv), len(inv), P(To),
                                          P(out), ctypes.byref(ni)), "eao_pose_optimization")
        return ni.value, To, out

    def optimize_batch_device(self, cam, nframes, cap, d_T, d_counts, d_kps, d_has, d_pos, inv_level_sigma2,
                              d_Tout, d_outlier, d_ninl, stream=None):
        """HBM-resident batch; d_* are device pointers (ints)."""
        inv = np.ascontiguousarray(inv_level_sigma2, np.float32)
        v = ctypes.c_void_p
        check(lib().eao_pose_optimization_batch_device(self.h, ctypes.byref(cam), nframes, cap, v(d_T), v(d_counts),
                                                       v(d_kps), v(d_has), v(d_pos), P(inv), len(inv), v(d_Tout),
                                                       v(d_outlier), v(d_ninl), v(stream) if stream else None),
              "eao_pose_optimization_batch_device")


class Vocab(_Handle):
    """DBoW2 ORB vocabulary on the GPU: ComputeBoW's transform and SearchByBoW
    (reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1271, src/ORBmatcher.cc:159-288).
    voc: dict with desc [n][32] u8, parent i32, word i32, weight f64, L (tools/synth.vocabulary)."""
    _DESTROY = "eao_vocab_destroy"

    def __init__(self, voc, max_kps=4096, max_batch=1, device=0):
        self.h = ctypes.c_void_p()
        self.max_kps = max_kps
        a = {k: np.ascontiguousarray(voc[k]) for k in ("desc", "parent", "word", "weight")}
        check(lib().eao_vocab_create(device, len(a["parent"]), P(a["desc"]), P(a["parent"]), P(a["word"]),
                                     P(a["weight"]), int(voc["L"]), max_kps, max_batch, ctypes.byref(self.h)),
              "eao_vocab_create")
        self._opened()


    def transform(self, desc, levelsup=4):
        """-> (word_ids, word_weights, node_ids, node_start, node_feats)."""
        n = len(desc)
        m = max(n, 1)
        wid, ww = np.zeros(m, np.int32), np.zeros(m, np.float64)
        nid, ns, nf = np.zeros(m, np.int32), np.zeros(m + 1, np.int32), np.zeros(m, np.int32)
        nw, nn = ctypes.c_int32(), ctypes.c_int32()
        check(lib().eao_bow_transform(self.h, n, P(np.ascontiguousarray(desc, np.uint8)), levelsup, P(wid), P(ww),
                                      ctypes.byref(nw), P(nid), P(ns), P(nf), ctypes.byref(nn)), "eao_bow_transform")
        k = nn.value
        return wid[:nw.value].copy(), ww[:nw.value].copy(), nid[:k].copy(), ns[:k + 1].copy(), nf[:ns[k]].copy()

    def search(self, nnratio, check_ori, kf_kps, kf_desc, kf_valid, kf_fv, f_kps, f_desc, f_fv):
        """SearchByBoW: fv = (node_ids, node_start, node_feats) -> (nmatches, f_match)."""
        m = np.full(len(f_kps), -1, np.int32)
        a = [np.ascontiguousarray(x, np.int32) for x in kf_fv]
        b = [np.ascontiguousarray(x, np.int32) for x in f_fv]
        n = check(lib().eao_search_by_bow(self.h, ctypes.c_float(nnratio), int(check_ori), len(kf_kps),
                                          P(np.ascontiguousarray(kf_kps)), P(np.ascontiguousarray(kf_desc, np.uint8)),
                                          P(np.ascontiguousarray(kf_valid, np.uint8)), len(a[0]), P(a[0]), P(a[1]),
                                          P(a[2]), len(f_kps), P(np.ascontiguousarray(f_kps)),
                                          P(np.ascontiguousarray(f_desc, np.uint8)), len(b[0]), P(b[0]), P(b[1]),
                                          P(b[2]), P(m)), "eao_search_by_bow")
        return n, m

    def search_kf(self, nnratio, check_ori, kps1, desc1, valid1, fv1, kps2, desc2, valid2, fv2):
        """SearchByBoW(KF1, KF2): fv = (node_ids, node_start, node_feats) -> (nmatches, match12)."""
        m = np.full(len(kps1), -1, np.int32)
        a = [np.ascontiguousarray(x, np.int32) for x in fv1]
        b = [np.ascontiguousarray(x, np.int32) for x in fv2]
        n = check(lib().eao_search_by_bow_kf(self.h, ctypes.c_float(nnratio), int(check_ori), len(kps1),
                                             P(np.ascontiguousarray(kps1)), P(np.ascontiguousarray(desc1, np.uint8)),
                                             P(np.ascontiguousarray(valid1, np.uint8)), len(a[0]), P(a[0]), P(a[1]),
                                             P(a[2]), len(kps2), P(np.ascontiguousarray(kps2)),
                                             P(np.ascontiguousarray(desc2, np.uint8)),
                                             P(np.ascontiguousarray(valid2, np.uint8)), len(b[0]), P(b[0]), P(b[1]),
                                             P(b[2]), P(m)), "eao_search_by_bow_kf")
        return n, m

    def search_kf_batch_device(self, nnratio, check_ori, nsearch, cap, d_n1, kf1, kf2, d_match, d_nm, stream=None):
        """kf1 / kf2: (kps, desc, valid, nn, node_ids, node_start, node_feats) device pointers."""
        v = ctypes.c_void_p
        check(lib().eao_search_by_bow_kf_batch_device(self.h, ctypes.c_float(nnratio), int(check_ori), nsearch, cap,
                                                      v(d_n1), *[v(x) for x in kf1], *[v(x) for x in kf2], v(d_match),
                                                      v(d_nm), v(stream) if stream else None),
              "eao_search_by_bow_kf_batch_device")

    def transform_batch_device(self, nframes, cap, d_counts, d_desc, levelsup, d_wid, d_ww, d_nw, d_nid, d_ns, d_nf,
                               d_nn, stream=None):
        v = ctypes.c_void_p
        check(lib().eao_bow_transform_batch_device(self.h, nframes, cap, v(d_counts), v(d_desc), levelsup, v(d_wid),
                                                   v(d_ww), v(d_nw), v(d_nid), v(d_ns), v(d_nf), v(d_nn),
                                                   v(stream) if stream else None), "eao_bow_transform_batch_device")

    def search_batch_device(self, nnratio, check_ori, nsearch, cap, kf, fr, d_match, d_nm, stream=None):
        """kf = (kps, desc, valid, nn, node_ids, node_start, node_feats) device pointers;
        fr = (n_f, kps, desc, nn, node_ids, node_start, node_feats)."""
        v = ctypes.c_void_p
        check(lib().eao_search_by_bow_batch_device(self.h, ctypes.c_float(nnratio), int(check_ori), nsearch, cap,
                                                   *[v(x) for x in kf], *[v(x) for x in fr], v(d_match), v(d_nm),
                                                   v(stream) if stream else None), "eao_search_by_bow_batch_device")


class Lines(_Handle):
    """Per-frame line detection (line_lbd_detect::detect_raw_lines + filter_lines,
    reference src/Frame.cc:324-328) on the GPU."""
    _DESTROY = "eao_lines_destroy"

    def __init__(self, w=640, h=480, max_batch=1, device=0):
        self.h = ctypes.c_void_p()
        self.w, self.hh = w, h
        check(lib().eao_lines_create(device, w, h, max_batch, ctypes.byref(self.h)), "eao_lines_create")
        self._opened()


    def detect(self, gray, min_length=50.0, cap=4096):
        """[n][6] float32: (startX, startY, endX, endY, angle, lineLength)."""
        g8 = np.ascontiguousarray(gray, np.uint8)
        out = np.zeros((cap, 6), np.float32)
        n = ctypes.c_int()
        check(lib().eao_lines_detect(self.h, P(g8), g8.shape[1], ctypes.c_float(min_length), P(out), cap,
                                     ctypes.byref(n)), "eao_lines_detect")
        return out[:n.value].copy()

    def detect_color(self, img, min_length=50.0, cap=4096):
        """eao_lines_detect_color: the colour frame ([h][w][3 or 4] BGR bytes, rawImage) converted with
        COLOR_BGR2GRAY inside the blur kernel, as BinaryDescriptor::detectImpl does."""
        a = np.ascontiguousarray(img, np.uint8)
        cn = 1 if a.ndim == 2 else a.shape[2]
        out = np.zeros((cap, 6), np.float32)
        n = ctypes.c_int()
        check(lib().eao_lines_detect_color(self.h, P(a), a.shape[1] * cn, cn, ctypes.c_float(min_length), P(out), cap,
                                           ctypes.byref(n)), "eao_lines_detect_color")
        return out[:n.value].copy()

    def detect_color_start(self, img, min_length=50.0, cap=4096):
        """eao_lines_detect_color_start: stage the frame and enqueue the detection, return at once."""
        a = np.ascontiguousarray(img, np.uint8)
        cn = 1 if a.ndim == 2 else a.shape[2]
        check(lib().eao_lines_detect_color_start(self.h, P(a), a.shape[1] * cn, cn, ctypes.c_float(min_length), cap),
              "eao_lines_detect_color_start")
        self._pending_cap = cap

    def detect_finish(self):
        """eao_lines_detect_finish: wait for the started frame, its lines."""
        cap = getattr(self, "_pending_cap", 0)
        out = np.zeros((max(cap, 1), 6), np.float32)
        n = ctypes.c_int()
        check(lib().eao_lines_detect_finish(self.h, P(out), ctypes.byref(n)), "eao_lines_detect_finish")
        return out[:n.value].copy()

    def detect_color_batch_device(self, img_ptr, nframes, pitch, channels, min_length, lines_ptr, counts_ptr, cap,
                                  stream=None):
        v = ctypes.c_void_p
        check(lib().eao_lines_detect_color_batch_device(self.h, v(img_ptr), nframes, pitch, channels,
                                                        ctypes.c_float(min_length), v(lines_ptr), v(counts_ptr), cap,
                                                        v(stream) if stream else None),
              "eao_lines_detect_color_batch_device")

    def debug_maps(self):
        blur = np.zeros((self.hh, self.w), np.uint8)
        dx, dy = np.zeros((self.hh, self.w), np.int16), np.zeros((self.hh, self.w), np.int16)
        code = np.zeros((self.hh, self.w), np.uint16)
        check(lib().eao_lines_debug_maps(self.h, P(blur), P(dx), P(dy), P(code)), "eao_lines_debug_maps")
        return blur, dx, dy, code

    def detect_batch_device(self, gray_ptr, nframes, pitch, min_length, lines_ptr, counts_ptr, cap, stream=None):
        v = ctypes.c_void_p
        check(lib().eao_lines_detect_batch_device(self.h, v(gray_ptr), nframes, pitch, ctypes.c_float(min_length),
                                                  v(lines_ptr), v(counts_ptr), cap, v(stream) if stream else None),
              "eao_lines_detect_batch_device")


class Assoc(_Handle):
    """Object_2D / Object_Map math replacement (reference src/Object.cc, isolation_forest.h)."""
    _DESTROY = "eao_assoc_destroy"

    def __init__(self, max_points=65536, device=0):
        self.h = ctypes.c_void_p()
        check(lib().eao_assoc_create(device, max_points, ctypes.byref(self.h)), "eao_assoc_create")
        self._opened()


    def np_batch(self, frame_sets, obj_sets):
        """frame_sets/obj_sets: lists of (pts (n,3) f32, valid (n,) u8 or None)."""
        def cat(sets):
            pts = [np.asarray(p, np.float32).reshape(-1, 3) for p, _ in sets]
            val = [np.ones(len(p), np.uint8) if v is None else np.asarray(v, np.uint8) for (_, v), p in zip(sets, pts)]
            lens = np.array([len(p) for p in pts], np.int32)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int32)
            allp = np.concatenate(pts) if len(pts) else np.zeros((0, 3), np.float32)
            allv = np.concatenate(val) if len(val) else np.zeros(0, np.uint8)
            return np.ascontiguousarray(allp), np.ascontiguousarray(allv), offs, lens
        fp, fv, fo, fl = cat(frame_sets)
        op, ov, oo, ol = cat(obj_sets)
        out = np.zeros(len(frame_sets), NP_DTYPE)
        check(lib().eao_np_test_batch(self.h, len(frame_sets), P(fp), P(fv), P(fo), P(fl), P(op), P(ov), P(oo),
                                      P(ol), P(out)), "eao_np_test_batch")
        return out

    def iforest(self, clouds, trees=50, seed=12345, samples=None):
        pts = [np.asarray(c, np.float32).reshape(-1, 3) for c in clouds]
        lens = np.array([len(p) for p in pts], np.int32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int32)
        if samples is None:
            samples = lens // 2
        samples = np.asarray(samples, np.uint32)
        allp = np.ascontiguousarray(np.concatenate(pts))
        scores = np.zeros(len(allp), np.float64)
        check(lib().eao_iforest_scores_batch(self.h, len(pts), P(allp), P(offs), P(lens), trees, seed, P(samples),
                                             P(scores)), "eao_iforest_scores_batch")
        return [scores[o:o + l] for o, l in zip(offs, lens)]

    def rects(self, cam, Tcw, clouds):
        pts = [np.asarray(c, np.float32).reshape(-1, 3) for c in clouds]
        lens = np.array([len(p) for p in pts], np.int32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int32)
        allp = np.ascontiguousarray(np.concatenate(pts)) if len(pts) else np.zeros((0, 3), np.float32)
        rect = np.zeros((len(pts), 4), np.int32)
        ok = np.zeros(len(pts), np.uint8)
        check(lib().eao_project_rects(self.h, ctypes.byref(cam), P(np.ascontiguousarray(Tcw, np.float32)),
                                      len(pts), P(allp), P(offs), P(lens), P(rect), P(ok)), "eao_project_rects")
        return rect, ok


class Replay(_Handle):
    """Deterministic association replay on the engine:
    the object section of Tracking::TrackWithMotionModel + LocalMapping object
    maintenance, with NP / iForest / projected rects on the GPU."""
    _DESTROY = "eao_replay_destroy"
    _EXIT_ORDER = 0

    def __init__(self, assoc, flag="iForest", w=640, h=480, K=(535.4, 539.2, 320.1, 247.6)):
        self.assoc = assoc
        self.h = ctypes.c_void_p()
        K4 = np.asarray(K, np.float32)
        check(lib().eao_replay_create(assoc.h, flag.encode(), w, h, P(K4), ctypes.byref(self.h)),
              "eao_replay_create")
        self._opened()


    def lines(self, sets):
        """Stage frame line segments (eao_replay_lines): a list of (L, 4) arrays, one per upcoming frame."""
        nl = np.array([len(np.asarray(x).reshape(-1, 4)) for x in sets], np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(x, np.float32).reshape(-1, 4) for x in sets])
                                    if len(sets) else np.zeros((0, 4), np.float32), np.float32)
        check(lib().eao_replay_lines(self.h, len(sets), P(nl), P(flat)), "eao_replay_lines")

    def frame(self, fid, T, boxes, ids, pos, uv, bad=None, lines=None):
        boxes = np.ascontiguousarray(boxes, np.int32).reshape(-1, 5)
        out = np.zeros((len(boxes), 4), np.int32)
        bad = np.zeros(len(ids), np.uint8) if bad is None else np.ascontiguousarray(bad, np.uint8)
        if lines is not None:
            self.lines([lines])
        check(lib().eao_replay_frame(self.h, int(fid), P(np.ascontiguousarray(T, np.float32)), len(boxes),
                                     P(boxes), len(ids), P(np.ascontiguousarray(ids, np.int32)),
                                     P(np.ascontiguousarray(pos, np.float32)),
                                     P(np.ascontiguousarray(uv, np.float32)), P(bad), P(out)),
              "eao_replay_frame")
        return out

    def frame_begin(self, fid, T, boxes, ids, pos, uv, bad=None):
        """eao_replay_frame_begin: the frame up to its line-dependent tail (the caller's line
        detection may still be running); finish with frame_end(lines)."""
        boxes = np.ascontiguousarray(boxes, np.int32).reshape(-1, 5)
        self._open = boxes
        bad = np.zeros(len(ids), np.uint8) if bad is None else np.ascontiguousarray(bad, np.uint8)
        check(lib().eao_replay_frame_begin(self.h, int(fid), P(np.ascontiguousarray(T, np.float32)), len(boxes),
                                           P(boxes), len(ids), P(np.ascontiguousarray(ids, np.int32)),
                                           P(np.ascontiguousarray(pos, np.float32)),
                                           P(np.ascontiguousarray(uv, np.float32)), P(bad)),
              "eao_replay_frame_begin")

    def frame_end(self, lines=None):
        """eao_replay_frame_end after staging the frame's lines: the detections' [n][4] rows."""
        out = np.zeros((len(self._open), 4), np.int32)
        if lines is not None:
            self.lines([lines])
        check(lib().eao_replay_frame_end(self.h, P(out)), "eao_replay_frame_end")
        return out

    def local_mapping(self):
        check(lib().eao_replay_local_mapping(self.h), "eao_replay_local_mapping")

    def update_points(self, ids, pos=None, bad=None):
        """eao_replay_update_points: LocalMapping's map-point changes (BA positions, culled /
        replaced points as bad) for the points the replay holds."""
        ids = np.ascontiguousarray(ids, np.int32)
        pos = None if pos is None else np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        bad = None if bad is None else np.ascontiguousarray(bad, np.uint8)
        check(lib().eao_replay_update_points(self.h, len(ids), P(ids), P(pos), P(bad)), "eao_replay_update_points")

    def held_points(self):
        n = check(lib().eao_replay_held_points(self.h, None, 0), "eao_replay_held_points")
        ids = np.zeros(max(1, n), np.int32)
        n = check(lib().eao_replay_held_points(self.h, P(ids), len(ids)), "eao_replay_held_points")
        return ids[:n].copy()

    def step(self, fid, f):
        """One frame of a stream dict (tools/synth): the frame, its map-point record, its local mapping."""
        out = self.frame(fid, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        if "upd_ids" in f:
            self.update_points(f["upd_ids"], f["upd_pos"], f["upd_bad"])
        if f["kf"]:
            self.local_mapping()
        return out

    ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

    def shard(self, rank, world, allgather=None, unique_id=None):
        """Object-sharded association (eao_replay_shard_*): call
        before the first frame on every rank with the same stream.
        allgather(bytes) -> bytes (world x len, rank order) selects the callback
        exchanger (e.g. gloo); otherwise unique_id (128 bytes, eao_rccl_unique_id
        on one rank, broadcast) selects RCCL."""
        if allgather is not None:
            def cb(ctx, send, recv, nbytes):
                try:
                    data = allgather(ctypes.string_at(send, nbytes))
                    if len(data) != nbytes * world:
                        return -1
                    ctypes.memmove(recv, data, len(data))
                    return 0
                except Exception:  # noqa: BLE001 -- reported through the C status
                    return -1
            self._cb = Replay.ALLGATHER(cb)
            check(lib().eao_replay_shard_callback(self.h, rank, world, self._cb, None), "eao_replay_shard_callback")
        else:
            uid = np.frombuffer(bytes(unique_id), np.uint8).copy()
            assert uid.size == 128
            check(lib().eao_replay_shard_rccl(self.h, rank, world, P(uid)), "eao_replay_shard_rccl")

    def shard_stats(self):
        out = np.zeros(3, np.float64)
        check(lib().eao_replay_shard_stats(self.h, P(out)), "eao_replay_shard_stats")
        return dict(exchanges=int(out[0]), bytes_per_rank=float(out[1]), exchange_us=float(out[2]))

    @staticmethod
    def pack(frames, first_id=1):
        """Concatenate a list of per-frame dicts (T, boxes, ids, pos, uv, bad, kf) for run()."""
        n = len(frames)
        return dict(
            n=n, ids=np.arange(first_id, first_id + n, dtype=np.int32),
            T=np.ascontiguousarray(np.stack([f["T"] for f in frames]), np.float32).reshape(n, 16),
            nb=np.array([len(f["boxes"]) for f in frames], np.int32),
            boxes=np.ascontiguousarray(np.concatenate([np.asarray(f["boxes"], np.int32).reshape(-1, 5) for f in frames])),
            npt=np.array([len(f["ids"]) for f in frames], np.int32),
            mp=np.ascontiguousarray(np.concatenate([f["ids"] for f in frames]), np.int32),
            pos=np.ascontiguousarray(np.concatenate([f["pos"] for f in frames]), np.float32),
            uv=np.ascontiguousarray(np.concatenate([f["uv"] for f in frames]), np.float32),
            bad=np.ascontiguousarray(np.concatenate([f["bad"] for f in frames]), np.uint8),
            kf=np.array([1 if f["kf"] else 0 for f in frames], np.uint8),
            lines=[f["lines"] for f in frames] if all("lines" in f for f in frames) else None,
            **Replay._pack_updates(frames))

    @staticmethod
    def _pack_updates(frames):
        """The frames' map-point records (keys upd_ids / upd_pos / upd_bad), if any frame has one."""
        if not any("upd_ids" in f for f in frames):
            return {}
        z = (np.zeros(0, np.int32), np.zeros((0, 3), np.float32), np.zeros(0, np.uint8))
        rec = [(f["upd_ids"], f["upd_pos"], f["upd_bad"]) if "upd_ids" in f else z for f in frames]
        return dict(nupd=np.array([len(r[0]) for r in rec], np.int32),
                    upd_ids=np.ascontiguousarray(np.concatenate([r[0] for r in rec]), np.int32),
                    upd_pos=np.ascontiguousarray(np.concatenate([np.reshape(r[1], (-1, 3)) for r in rec]), np.float32),
                    upd_bad=np.ascontiguousarray(np.concatenate([r[2] for r in rec]), np.uint8))

    def run(self, pk):
        """eao_replay_run over a packed stream; returns det_out (total boxes x 4)."""
        out = np.zeros((int(pk["nb"].sum()), 4), np.int32)
        if pk.get("lines") is not None:
            self.lines(pk["lines"])
        if "nupd" in pk:
            check(lib().eao_replay_run_updates(
                self.h, pk["n"], P(pk["ids"]), P(pk["T"]), P(pk["nb"]), P(pk["boxes"]), P(pk["npt"]), P(pk["mp"]),
                P(pk["pos"]), P(pk["uv"]), P(pk["bad"]), P(pk["kf"]), P(pk["nupd"]), P(pk["upd_ids"]),
                P(pk["upd_pos"]), P(pk["upd_bad"]), P(out)), "eao_replay_run_updates")
            return out
        check(lib().eao_replay_run(self.h, pk["n"], P(pk["ids"]), P(pk["T"]), P(pk["nb"]), P(pk["boxes"]),
                                   P(pk["npt"]), P(pk["mp"]), P(pk["pos"]), P(pk["uv"]), P(pk["bad"]), P(pk["kf"]),
                                   P(out)), "eao_replay_run")
        return out

    def objects(self):
        n = check(lib().eao_replay_num_objects(self.h), "eao_replay_num_objects")
        ints = np.zeros((n, 8), np.int32)
        fl = np.zeros((n, 20), np.float32)
        pts = []
        for i in range(n):
            check(lib().eao_replay_object(self.h, i, P(ints[i]), P(fl[i])), "eao_replay_object")
            ids = np.zeros(max(1, ints[i, 4]), np.int32)
            k = check(lib().eao_replay_object_points(self.h, i, P(ids), len(ids)), "eao_replay_object_points")
            pts.append(ids[:k].copy())
        return ints, fl, pts


# ---------------------------------------------------------------- frame input stage
def yolo_parse(text):
    """eao_yolo_parse: one data/yolo_txts file's text -> (n, 6) int32 rows
    {class, x, y, w, h, score} as Tracking::GrabImageMonocular reads them."""
    b = text.encode() if isinstance(text, str) else bytes(text)
    cap = max(16, b.count(b"\n") + 1)
    out = np.zeros((cap, 6), np.int32)
    n = ctypes.c_int()
    buf = ctypes.create_string_buffer(b, len(b))
    check(lib().eao_yolo_parse(buf, ctypes.c_size_t(len(b)), P(out), cap, ctypes.byref(n)), "eao_yolo_parse")
    return out[:n.value].copy()


def gt_lookup(gt, timestamps):
    """eao_gt_lookup: (row index or -1, Twc float32 (n, 4, 4)) per timestamp."""
    gt = np.ascontiguousarray(gt, np.float64).reshape(-1, 8)
    ts = np.ascontiguousarray(timestamps, np.float64).reshape(-1)
    idx = np.zeros(len(ts), np.int32)
    T = np.zeros((len(ts), 4, 4), np.float32)
    check(lib().eao_gt_lookup(P(gt), len(gt), P(ts), len(ts), P(idx), P(T)), "eao_gt_lookup")
    return idx, T

