"""ORACLE — test infrastructure only (CPU restatement of the reference hot path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as the
checker / CPU baseline. The product package (gtsfm_amd) never imports it.

Loads oracle/liboracle.so (built by oracle/Makefile, see __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib: Optional[ctypes.CDLL] = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> str:
    """Compiles the oracle restatement (gcc, no reference sources involved)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.oracle_twoway_match.restype = ctypes.c_int
        _lib.oracle_twoway_match.argtypes = [_f32p, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_double, _u32p]
        _lib.oracle_oneway_top2.restype = None
        _lib.oracle_oneway_top2.argtypes = [_f32p, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int,
                                            _f32p, _f32p, _i32p]
        _register_optional(_lib)
    return _lib


def _register_optional(l: ctypes.CDLL) -> None:
    """Registers symbols of the restatements that exist in this build (ransac / sift)."""
    if hasattr(l, "oracle_ransac_E"):
        l.oracle_ransac_E.restype = ctypes.c_int
        l.oracle_ransac_E.argtypes = [_f64p, _f64p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _f64p, _u8p, _f64p, _f64p,
                                      ctypes.POINTER(ctypes.c_int)]
        l.oracle_ransac_E_gc.restype = ctypes.c_int
        l.oracle_ransac_E_gc.argtypes = [_f64p, _f64p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_int, ctypes.c_int, _f64p, _u8p, _f64p, _f64p,
                                         ctypes.POINTER(ctypes.c_int)]
        l.oracle_gc_label_q.restype = ctypes.c_int
        l.oracle_gc_label_q.argtypes = [np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS"),
                                        np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS"), ctypes.c_int,
                                        ctypes.c_int64, ctypes.c_int64, _u8p]
        l.oracle_five_point.restype = ctypes.c_int
        l.oracle_five_point.argtypes = [_f64p, _f64p, _f64p]
        l.oracle_sample5.restype = ctypes.c_int
        l.oracle_sample5.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p]
        l.oracle_sampson_sq.restype = None
        l.oracle_sampson_sq.argtypes = [_f64p, _f64p, _f64p, ctypes.c_int, ctypes.c_int, _f64p]
        l.oracle_recover_pose.restype = ctypes.c_int
        l.oracle_recover_pose.argtypes = [_f64p, _f64p, _f64p, ctypes.c_void_p, ctypes.c_int, _f64p, _f64p]
    if hasattr(l, "oracle_ba2"):
        l.oracle_ba2.restype = ctypes.c_int
        l.oracle_ba2.argtypes = [_f64p, _f64p, ctypes.c_int, _f64p, _f64p, _f64p, _f64p, ctypes.c_int, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, _f64p, _f64p, _u8p,
                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
        l.oracle_between_eval.restype = None
        l.oracle_between_eval.argtypes = [_f64p, _f64p, _f64p, ctypes.c_void_p, _f64p, ctypes.c_void_p]
    if hasattr(l, "oracle_ransac_F"):
        l.oracle_ransac_F.restype = ctypes.c_int
        l.oracle_ransac_F.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_uint64, ctypes.c_int, _f64p, _u8p, ctypes.POINTER(ctypes.c_int)]
        l.oracle_seven_point.restype = ctypes.c_int
        l.oracle_seven_point.argtypes = [_f32p, _i32p, _f64p]
        l.oracle_sample7.restype = ctypes.c_int
        l.oracle_sample7.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _i32p]
        l.oracle_f_error.restype = ctypes.c_float
        l.oracle_f_error.argtypes = [_f64p, _f32p]
    if hasattr(l, "oracle_sift_detect_describe"):
        l.oracle_sift_detect_describe.restype = ctypes.c_int
        l.oracle_sift_detect_describe.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p,
                                                  ctypes.POINTER(ctypes.c_int)]
        l.oracle_sift_detect_describe_masked.restype = ctypes.c_int
        l.oracle_sift_detect_describe_masked.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                                         _f32p, ctypes.POINTER(ctypes.c_int)]
        l.oracle_rgb_to_gray.restype = None
        l.oracle_rgb_to_gray.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, _u8p]
        l.oracle_sift_pyramid_level.restype = ctypes.c_int
        l.oracle_sift_pyramid_level.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]


def twoway_match(d1: np.ndarray, d2: np.ndarray, ratio: Optional[float]) -> np.ndarray:
    """Mutual NN + ratio matching; returns (M,2) uint32 ordered like the reference."""
    d1 = np.ascontiguousarray(d1, dtype=np.float32)
    d2 = np.ascontiguousarray(d2, dtype=np.float32)
    if d1.ndim == 1:
        d1 = d1.reshape(-1, 1)
    if d2.ndim == 1:
        d2 = d2.reshape(-1, 1)
    n1, D = d1.shape
    n2 = d2.shape[0]
    out = np.zeros((max(1, min(n1, n2)), 2), dtype=np.uint32)
    m = lib().oracle_twoway_match(d1, n1, d2, n2, D, -1.0 if ratio is None else float(ratio), out)
    return out[:m].copy()


def oneway_top2(q: np.ndarray, t: np.ndarray):
    q = np.ascontiguousarray(q, dtype=np.float32)
    t = np.ascontiguousarray(t, dtype=np.float32)
    nq, D = q.shape
    d1 = np.zeros(nq, np.float32)
    d2 = np.zeros(nq, np.float32)
    j1 = np.zeros(nq, np.int32)
    lib().oracle_oneway_top2(q, nq, t, t.shape[0], D, d1, d2, j1)
    return d1, d2, j1


RANSAC_SEED = 0x5EED5EED
SCORING_RANSAC = 0  # == GTSFM_RANSAC_SCORING_RANSAC
SCORING_MSAC = 1  # == GTSFM_RANSAC_SCORING_MSAC


def five_point(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    """All essential matrices (k,3,3) from 5 normalized correspondences (Nister)."""
    Es = np.zeros(90, np.float64)
    n = lib().oracle_five_point(np.ascontiguousarray(x1, np.float64).ravel(),
                                np.ascontiguousarray(x2, np.float64).ravel(), Es)
    return Es[: 9 * n].reshape(n, 3, 3)


def sample5(pair: int, h: int, M: int, seed: int = RANSAC_SEED) -> Optional[np.ndarray]:
    idx = np.zeros(5, np.int32)
    return idx if lib().oracle_sample5(seed, pair, h, M, idx) else None


def ransac_E(x1n: np.ndarray, x2n: np.ndarray, thr: float, prob: float = 0.999999, max_iters: int = 1000,
             seed: int = RANSAC_SEED, pair_id: int = 0, scoring: int = SCORING_MSAC):
    """Returns (E (3,3), inlier mask (M,) uint8, R (3,3), t (3,), n_inliers, n_hypotheses) or None.
    scoring: SCORING_RANSAC (most inliers, cv2 RANSAC) or SCORING_MSAC (truncated quadratic, USAC_ACCURATE)."""
    x1n = np.ascontiguousarray(x1n, np.float64)
    x2n = np.ascontiguousarray(x2n, np.float64)
    M = x1n.shape[0]
    E = np.zeros(9)
    R = np.zeros(9)
    t = np.zeros(3)
    mask = np.zeros(max(M, 1), np.uint8)
    nh = ctypes.c_int(0)
    n = lib().oracle_ransac_E(x1n.ravel(), x2n.ravel(), M, thr, prob, max_iters, seed, pair_id, int(scoring), E, mask,
                              R, t, ctypes.byref(nh))
    if n < 0:
        return None
    return E.reshape(3, 3), mask[:M].copy(), R.reshape(3, 3), t, n, nh.value


def ransac_E_gc(x1n: np.ndarray, x2n: np.ndarray, thr: float, gc_iters: int, gc_cell: float, gc_lambda=(39, 40),
                prob: float = 0.999999, max_iters: int = 1000, seed: int = RANSAC_SEED, pair_id: int = 0,
                scoring: int = SCORING_MSAC):
    """ransac_E followed by the graph-cut LO stage (oracle/ransac.c gc_label): gc_cell in normalised units,
    gc_lambda = (num, den) of the spatial-coherence weight. Same return tuple as ransac_E."""
    x1n = np.ascontiguousarray(x1n, np.float64)
    x2n = np.ascontiguousarray(x2n, np.float64)
    M = x1n.shape[0]
    E, R, t = np.zeros(9), np.zeros(9), np.zeros(3)
    mask = np.zeros(max(M, 1), np.uint8)
    nh = ctypes.c_int(0)
    n = lib().oracle_ransac_E_gc(x1n.ravel(), x2n.ravel(), M, thr, prob, max_iters, seed, pair_id, int(scoring),
                                 int(gc_iters), float(gc_cell), int(gc_lambda[0]), int(gc_lambda[1]), E, mask, R, t,
                                 ctypes.byref(nh))
    if n < 0:
        return None
    return E.reshape(3, 3), mask[:M].copy(), R.reshape(3, 3), t, n, nh.value


def gc_label_q(q: np.ndarray, key: np.ndarray, lam=(39, 40)) -> np.ndarray:
    """Graph-cut labelling (oracle/ransac.c oracle_gc_label_q) of points with MSAC terms q and cell keys."""
    q = np.ascontiguousarray(q, np.uint32)
    key = np.ascontiguousarray(key, np.int64)
    lab = np.zeros(max(len(q), 1), np.uint8)
    lib().oracle_gc_label_q(q, key, len(q), int(lam[0]), int(lam[1]), lab)
    return lab[: len(q)].astype(bool)


def sampson_sq(F: np.ndarray, x1: np.ndarray, x2: np.ndarray, precision: int = 0) -> np.ndarray:
    """Squared Sampson distances (n,) of x1[i] <-> x2[i] under F: 0 = double, 1 = the verifier's float32 expression."""
    x1 = np.ascontiguousarray(x1, np.float64).reshape(-1, 2)
    x2 = np.ascontiguousarray(x2, np.float64).reshape(-1, 2)
    out = np.zeros(len(x1), np.float64)
    lib().oracle_sampson_sq(np.ascontiguousarray(F, np.float64).ravel(), x1.ravel(), x2.ravel(), len(x1), precision,
                            out)
    return out


def seven_point(x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    """All fundamental matrices (k,3,3), k <= 3, through 7 pixel correspondences (x1, x2: (7,2))."""
    pts = np.ascontiguousarray(np.hstack([x1, x2]), np.float32)
    Fs = np.zeros(27, np.float64)
    n = lib().oracle_seven_point(pts.ravel(), np.arange(7, dtype=np.int32), Fs)
    return Fs[: 9 * n].reshape(n, 3, 3)


def f_errors(F: np.ndarray, x1: np.ndarray, x2: np.ndarray) -> np.ndarray:
    """Per-correspondence max squared point-to-epipolar-line distance (float32), as the F verifier scores it."""
    pts = np.ascontiguousarray(np.hstack([x1, x2]), np.float32)
    Fd = np.ascontiguousarray(F, np.float64).ravel()
    return np.array([lib().oracle_f_error(Fd, pts[i].copy()) for i in range(len(pts))], np.float32)


def ransac_F(x1: np.ndarray, x2: np.ndarray, thr_px: float, prob: float = 0.999999, max_iters: int = 1000000,
             seed: int = RANSAC_SEED, pair_id: int = 0):
    """F path on pixel coordinates: (F (3,3), mask (M,) uint8, n_inliers, n_hypotheses) or None."""
    x1 = np.ascontiguousarray(x1, np.float32)
    x2 = np.ascontiguousarray(x2, np.float32)
    M = x1.shape[0]
    F = np.zeros(9)
    mask = np.zeros(max(M, 1), np.uint8)
    nh = ctypes.c_int(0)
    n = lib().oracle_ransac_F(x1.ravel(), x2.ravel(), M, thr_px, prob, max_iters, seed, pair_id, F, mask,
                              ctypes.byref(nh))
    if n < 0:
        return None
    return F.reshape(3, 3), mask[:M].copy(), n, nh.value


def verify_F(x1: np.ndarray, x2: np.ndarray, K1: np.ndarray, K2: np.ndarray, thr_px: float, **kw):
    """opencv_verifier_base.verify with use_intrinsics_in_verification=False: F, E = K2^T F K1, recoverPose on
    the K-normalised inliers. Returns (R, t, mask, n_inliers) or None."""
    r = ransac_F(x1, x2, thr_px, **kw)
    if r is None:
        return None
    F, mask, n, _ = r
    E = K2.T @ F @ K1
    sel = mask.astype(bool)
    n1 = (np.asarray(x1, np.float64)[sel] - K1[:2, 2]) / K1[0, 0]
    n2 = (np.asarray(x2, np.float64)[sel] - K2[:2, 2]) / K2[0, 0]
    R, t, _ = recover_pose(E, n1, n2)
    return R, t, mask, n


def recover_pose(E: np.ndarray, x1n: np.ndarray, x2n: np.ndarray):
    R = np.zeros(9)
    t = np.zeros(3)
    x1n = np.ascontiguousarray(x1n, np.float64)
    x2n = np.ascontiguousarray(x2n, np.float64)
    good = lib().oracle_recover_pose(np.ascontiguousarray(E, np.float64).ravel(), x1n.ravel(), x2n.ravel(), None,
                                     x1n.shape[0], R, t)
    return R.reshape(3, 3), t, good


def ba2(uv1: np.ndarray, uv2: np.ndarray, K1, K2, R: np.ndarray, t: np.ndarray, max_iters: int = 100,
        reproj_thresh: float = 0.5, tri_thresh: float = 100.0, prior_R: Optional[np.ndarray] = None,
        prior_t: Optional[np.ndarray] = None, prior_sigmas: Optional[np.ndarray] = None):
    """Two-view triangulation + bundle adjustment (oracle/ba2.c). K = (f, u0, v0). Returns
    (status, R_out, t_out, valid (n,) bool, LM iterations, final error); status 0 ok / 1 no track / 2 none valid.
    prior_R / prior_t / prior_sigmas: an i2Ti1 relative-pose prior (PosePrior value and sigmas, rotation first)."""
    uv1 = np.ascontiguousarray(uv1, np.float64).reshape(-1, 2)
    uv2 = np.ascontiguousarray(uv2, np.float64).reshape(-1, 2)
    n = len(uv1)
    Ro, to = np.zeros(9), np.zeros(3)
    valid = np.zeros(max(n, 1), np.uint8)
    it, err = ctypes.c_int(0), ctypes.c_double(0)
    prt = psg = None
    if prior_R is not None:
        prt = np.concatenate([np.asarray(prior_R, np.float64).ravel(), np.asarray(prior_t, np.float64).ravel()])
        psg = np.ascontiguousarray(prior_sigmas, np.float64).ravel()
    st = lib().oracle_ba2(uv1.ravel(), uv2.ravel(), n, np.asarray(K1, np.float64), np.asarray(K2, np.float64),
                          np.ascontiguousarray(R, np.float64).ravel(), np.ascontiguousarray(t, np.float64).ravel(),
                          max_iters, reproj_thresh, tri_thresh, None if prt is None else prt.ctypes.data,
                          None if psg is None else psg.ctypes.data, Ro, to, valid, ctypes.byref(it),
                          ctypes.byref(err))
    return st, Ro.reshape(3, 3), to, valid[:n].astype(bool), it.value, err.value


def rgb_to_gray(rgb: np.ndarray) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.uint8)
    H, W, _ = rgb.shape
    g = np.zeros((H, W), np.uint8)
    lib().oracle_rgb_to_gray(rgb.ravel(), H, W, g.ravel())
    return g


def sift(gray: np.ndarray, max_kpts: int = 5000, with_desc: bool = True, mask: Optional[np.ndarray] = None):
    """SIFT restatement on a u8 gray image: (kp (N,5) [x, y, size, angle, response], desc (N,128), n_detected).
    mask: optional (H, W) u8; keypoints whose rounded pixel is 0 are dropped before the top-k (runByPixelsMask)."""
    gray = np.ascontiguousarray(gray, np.uint8)
    H, W = gray.shape
    kp = np.zeros((max_kpts, 5), np.float32)
    desc = np.zeros((max_kpts, 128), np.float32)
    nd = ctypes.c_int(0)
    if mask is not None:
        m = np.ascontiguousarray(mask, np.uint8)
        assert m.shape == (H, W)
        n = lib().oracle_sift_detect_describe_masked(gray.ravel(), m.ravel(), H, W, max_kpts, kp.ravel(), desc.ravel(),
                                                     ctypes.byref(nd))
        return kp[:n].copy(), desc[:n].copy(), nd.value
    n = lib().oracle_sift_detect_describe(gray.ravel(), H, W, max_kpts, kp.ravel(), desc.ravel(), ctypes.byref(nd))
    return kp[:n].copy(), desc[:n].copy(), nd.value


def sift_level(gray: np.ndarray, o: int, i: int) -> np.ndarray:
    gray = np.ascontiguousarray(gray, np.uint8)
    H, W = gray.shape
    out = np.zeros((2 * H) * (2 * W), np.float32)
    Ho, Wo = ctypes.c_int(0), ctypes.c_int(0)
    lib().oracle_sift_pyramid_level(gray.ravel(), H, W, o, i, out, ctypes.byref(Ho), ctypes.byref(Wo))
    return out[: Ho.value * Wo.value].reshape(Ho.value, Wo.value).copy()


# ---- f3 retrieval (numpy; netvlad_retriever.py). Parity unpinned against the reference module itself: importing it
# needs gtsam (absent here); pinned instead against the reference test's hand-made descriptors and expected pairs.
def retrieval_similarity(desc: np.ndarray, blocksize: int) -> np.ndarray:
    """netvlad_retriever.py:77-149: per block pair (bi <= bj) the f32 einsum "id,jd->ij", aggregated into zeros."""
    desc = np.asarray(desc, np.float32)
    n = desc.shape[0]
    sim = np.zeros((n, n), np.float32)
    nb = -(-n // blocksize)
    for bi in range(nb):
        for bj in range(bi, nb):
            i0, i1 = bi * blocksize, min((bi + 1) * blocksize, n)
            j0, j1 = bj * blocksize, min((bj + 1) * blocksize, n)
            sim[i0:i1, j0:j1] = (desc[i0:i1].astype(np.float64) @ desc[j0:j1].astype(np.float64).T).astype(np.float32)
    return sim


def retrieval_select_row(row: np.ndarray, bad: np.ndarray, k: int, min_score: Optional[float]) -> list:
    """One row of pairs_from_score_matrix (netvlad_retriever.py:218-228): the columns of the finite entries of
    topk(row masked by `bad` and min_score, k) in rank order -- NaN first, then value descending, equal values by
    ascending column."""
    row = np.asarray(row, np.float32).copy()
    bad = np.asarray(bad, bool).copy()
    if min_score is not None:
        bad |= row < min_score
    row[bad] = -np.inf
    nan = np.isnan(row)
    order = np.lexsort((np.arange(row.shape[0]), -np.where(nan, 0, row), ~nan))
    return [int(j) for j in order[:k] if np.isfinite(row[j])]


def retrieval_pairs(scores: np.ndarray, num_select: int, min_score: Optional[float],
                    invalid: Optional[np.ndarray] = None) -> list:
    """netvlad_retriever.py:196-228 (+ the strict-upper mask of :164-167 when `invalid` is None): rows concatenated."""
    scores = np.asarray(scores, np.float32)
    n1, n2 = scores.shape
    k = min(num_select, n1)
    if invalid is None:
        invalid = ~np.triu(np.ones((n1, n2), bool), 1)
    return [(i, j) for i in range(n1) for j in retrieval_select_row(scores[i], invalid[i], k, min_score)]
