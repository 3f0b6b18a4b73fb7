"""Device-resident batched entry points over the C ABI (include/gtsfm_hip.h).

torch provides HBM allocations and the stream; every computation is a libgtsfm_hip.so kernel. Tensors passed
in must already live on the GPU; nothing here copies to the host or synchronises (except the measurement hook
match_pairs(stats=...)).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch

from gtsfm_amd import native


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def match_pairs(desc: torch.Tensor, counts: torch.Tensor, pairs: torch.Tensor, ratio: Optional[float],
                mode: int = native.GTSFM_MATCH_INT_F16, stream: Optional[torch.cuda.Stream] = None,
                groups: Optional[torch.Tensor] = None,
                out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                stats: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mutual-NN + ratio matching of every (i1, i2) row of `pairs`.

    Args:
        desc: (n_img, kmax, dim) float32 descriptors on the GPU (rows >= counts[i] are ignored).
        counts: (n_img,) int32 valid rows per image.
        pairs: (P, 2) int32 image index pairs.
        ratio: ratio-test threshold, or None for plain mutual NN.
        mode: GTSFM_MATCH_INT_F16 (integer descriptors, MFMA) or GTSFM_MATCH_EXACT_F32.
        groups: optional (n_groups, G) int32 device tensor of pair indices (-1 = empty slot) for the INT_F16 kernel:
            every pair exactly once, the pairs of a group sharing image i1 (pair_groups builds one).
        out: optional caller-owned (idx (P, kmax, 2) int32, count (P,) int32) to write into (no allocation: a
            pipelined caller keeps them across steps instead of cycling cross-stream blocks through the allocator).
        stats: optional dict filled, for GTSFM_MATCH_F16_RERANK with dim <= 256, with the certificate's counts
            (gtsfm_match_rerank_stats; synchronises the stream): "keypoint_sides" (sum over pairs of both images'
            counts), "uncertified" and "uncertified_frac" (entries the fp16 shortlist did not certify, recomputed
            exactly), "tiled_frac" (entries of (pair, side)s recomputed whole by the exact tile kernel) and
            "rescan_frac" (uncertified entries rescanned one keypoint at a time).

    Returns:
        idx: (P, kmax, 2) int32 tensor holding uint32 keypoint indices, rows [0, count) valid per pair.
        count: (P,) int32.
    """
    assert desc.is_cuda and desc.dtype == torch.float32 and desc.dim() == 3 and desc.is_contiguous()
    assert counts.dtype == torch.int32 and pairs.dtype == torch.int32 and pairs.is_contiguous()
    n_img, kmax, dim = desc.shape
    n_pairs = pairs.shape[0]
    L = native.lib()
    if out is not None:
        idx, cnt = out
        assert idx.dtype == torch.int32 and idx.is_contiguous() and tuple(idx.shape) == (n_pairs, kmax, 2)
        assert cnt.dtype == torch.int32 and cnt.is_contiguous() and tuple(cnt.shape) == (n_pairs,)
        cnt.zero_()
    else:
        idx = torch.empty((max(n_pairs, 1), kmax, 2), dtype=torch.int32, device=desc.device)
        cnt = torch.zeros((max(n_pairs, 1),), dtype=torch.int32, device=desc.device)
    if n_pairs == 0:
        return idx[:0], cnt[:0]
    ws_bytes = L.gtsfm_match_workspace_bytes(n_img, kmax, dim, n_pairs, mode)
    ws = _workspace(ws_bytes, desc.device)
    if stream is not None:
        ws.record_stream(stream)  # the kernels may still read it after this function returns
    if groups is not None:
        assert groups.is_cuda and groups.dtype == torch.int32 and groups.dim() == 2 and groups.is_contiguous()
    rc = L.gtsfm_match_batched_grouped(
        _ptr(desc), _ptr(counts), n_img, kmax, dim, _ptr(pairs), n_pairs,
        _ptr(groups) if groups is not None else None, 0 if groups is None else groups.shape[0],
        0 if groups is None else groups.shape[1], -1.0 if ratio is None else float(ratio), mode, _ptr(ws),
        ws.numel(), _ptr(idx), _ptr(cnt), native.stream_handle(stream))
    native.check(rc, "gtsfm_match_batched_grouped")
    if stats is not None and mode == native.GTSFM_MATCH_F16_RERANK and dim <= 256:
        unc = np.zeros(2 * n_pairs, dtype=np.int32)
        n_unc = ctypes.c_int(0)
        native.check(L.gtsfm_match_rerank_stats(_ptr(ws), ws.numel(), n_img, kmax, dim, n_pairs, ctypes.byref(n_unc),
                                                unc.ctypes.data, native.stream_handle(stream)),
                     "gtsfm_match_rerank_stats")
        c = counts.cpu().numpy().astype(np.int64)
        pr = pairs.cpu().numpy().astype(np.int64)
        nq = np.concatenate([c[pr[:, 0]], c[pr[:, 1]]])  # side 0: rows of i1, side 1: rows of i2
        tiled = (unc > 0) & (unc.astype(np.int64) * 32 >= nq)
        total = max(int(nq.sum()), 1)
        stats.update(keypoint_sides=int(nq.sum()), uncertified=int(n_unc.value),
                     uncertified_frac=int(n_unc.value) / total, tiled_frac=int(nq[tiled].sum()) / total,
                     rescan_frac=int(unc[~tiled].sum()) / total)
    return idx, cnt


def match_group_size(kmax: int, dim: int) -> int:
    """Largest pairs-per-workgroup the INT_F16 distance GEMM holds for this kmax / dim (0: not supported)."""
    return int(native.lib().gtsfm_match_max_group(int(kmax), int(dim)))


def _split_cost(n_groups: int, group_size: int, kmax: int, n_cu: int) -> float:
    """Estimated time (in pair-passes of one workgroup) of a grouped distance-GEMM launch, with the pass split the
    library picks for it (matcher.hip pp_split: n_split in {1, 2, 4} minimising ceil(n_groups * n_split / CUs) *
    (passes / n_split))."""
    npass = -(-kmax // 512)
    best = None
    s = 1
    while s <= 4 and s <= npass:
        t = -(-(n_groups * s) // n_cu) * -(-npass // s)
        best = t if best is None or t < best else best
        s *= 2
    return float(best) * group_size


def match_plan(pairs: np.ndarray, kmax: int, dim: int, n_cu: Optional[int] = None) -> Optional[np.ndarray]:
    """Pair groups for the INT_F16 distance GEMM (gtsfm_match_batched_grouped), sized to fill the GPU: the largest
    group size (most reuse of the register operand) is kept unless a smaller one, together with the library's pass
    split, finishes in fewer estimated workgroup rounds. A rank's share of C2 at 8 GPUs (~619 pairs dealt in whole
    (i1, i2 // 4) runs, sharding.rank_pairs) has ~160 groups of 4 for 256 CUs: full groups of 2 split over pass ranges
    take 10 pair-passes of time instead of 12."""
    gmax = match_group_size(kmax, dim)
    if gmax <= 1:
        return None
    if n_cu is None:
        n_cu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count \
            if torch.cuda.is_available() else 256
    plans = [(g, pair_groups(pairs, g)) for g in range(gmax, 0, -1)]
    cost = [_split_cost(len(groups), g, kmax, n_cu) for g, groups in plans]
    # the estimate ignores what a smaller group loses (the register operand re-read per pair, more workgroups):
    # a smaller group must win by more than 10 %
    best = min(cost)
    return next(groups for (g, groups), t in zip(plans, cost) if t <= 1.1 * best)


def pair_groups(pairs: np.ndarray, group_size: int) -> np.ndarray:
    """Tile an (P, 2) pair list into groups for the INT_F16 distance GEMM: each group = up to `group_size` pairs
    (i1, i2) sharing i1 (the register operand) with i2 in one block of `group_size` consecutive image ids, ordered
    block-major, so the ~32 workgroups resident on one XCD stream the same few i2 images from its L2 while each reads
    its own i1 once. Returns (n_groups, group_size) int32 pair indices, -1 for empty slots."""
    pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    P = len(pairs)
    if P == 0 or group_size <= 1:
        return np.arange(P, dtype=np.int32).reshape(-1, 1)
    blk = pairs[:, 1] // group_size
    order = np.lexsort((pairs[:, 1], pairs[:, 0], blk))  # block-major, then i1, then i2
    key = blk[order] * (int(pairs[:, 0].max()) + 1) + pairs[order, 0]
    starts = np.flatnonzero(np.r_[True, key[1:] != key[:-1]])
    sizes = np.diff(np.r_[starts, P])
    rank = np.arange(P) - np.repeat(starts, sizes)           # position inside its (block, i1) run
    n_sub = -(-sizes // group_size)                           # groups per run (> 1 only for repeated pairs)
    first = np.r_[0, np.cumsum(n_sub)[:-1]]
    gid = np.repeat(first, sizes) + rank // group_size
    out = np.full((int(n_sub.sum()), group_size), -1, dtype=np.int32)
    out[gid, rank % group_size] = order
    return out


class RansacResult:
    """Per-pair verifier outputs (device tensors): E, R (i2Ri1), t (i2ti1), n_inliers, status, n_hyp, mask, and
    n_models (candidate models scored; E path only, else None)."""

    def __init__(self, E, R, t, n_inliers, status, n_hyp, mask, n_models=None):
        self.E, self.R, self.t = E, R, t
        self.n_inliers, self.status, self.n_hyp, self.mask = n_inliers, status, n_hyp, mask
        self.n_models = n_models


def ransac_essential(kp_xy: torch.Tensor, intrinsics: torch.Tensor, pairs: torch.Tensor, match_idx: torch.Tensor,
                     match_count: torch.Tensor, thr_px: float, prob: float = 0.999999, max_iters: int = 1000,
                     seed: int = native.RANSAC_DEFAULT_SEED, pair_id_base: int = 0,
                     pair_ids: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None,
                     scoring: int = native.GTSFM_RANSAC_SCORING_MSAC) -> RansacResult:
    """Batched 5-point RANSAC + LO + recoverPose for every pair (gtsfm_ransac_E_batched).
    scoring: GTSFM_RANSAC_SCORING_MSAC (USAC_ACCURATE, the reference's default) or _RANSAC (inlier count).

    Args:
        kp_xy: (n_img, kmax, 2) float32 keypoint pixels; intrinsics: (n_img, 3) float64 (f, u0, v0).
        pairs: (P, 2) int32; match_idx: (P, mcap, 2) int32 (uint32 values); match_count: (P,) int32.
        pair_ids: optional (P,) int32 sampler keys (default pair_id_base + p).
    """
    assert pair_ids is None or (pair_ids.dtype == torch.int32 and pair_ids.is_cuda and pair_ids.numel() == pairs.shape[0])
    assert kp_xy.is_cuda and kp_xy.dtype == torch.float32 and kp_xy.dim() == 3 and kp_xy.is_contiguous()
    assert intrinsics.dtype == torch.float64 and intrinsics.is_contiguous()
    assert match_idx.dtype == torch.int32 and match_idx.is_contiguous() and match_count.dtype == torch.int32
    n_img, kmax, _ = kp_xy.shape
    P = pairs.shape[0]
    mcap = match_idx.shape[1]
    dev = kp_xy.device
    L = native.lib()
    # outputs carved from two zeroed buffers (one fill each instead of one per output; pairs the verifier rejects keep
    # zero E / R / t, as do the mask entries past a pair's match count)
    P1 = max(P, 1)
    f64 = torch.zeros(21 * P1, dtype=torch.float64, device=dev)
    E, R, t = f64[:9 * P1].view(P1, 3, 3), f64[9 * P1:18 * P1].view(P1, 3, 3), f64[18 * P1:].view(P1, 3)
    i32 = torch.zeros(4 * P1, dtype=torch.int32, device=dev)
    n_inl, status, n_hyp, n_models = (i32[j * P1:(j + 1) * P1] for j in range(4))
    mask = torch.zeros((P1, max(mcap, 1)), dtype=torch.uint8, device=dev)
    if P > 0:
        ws = _workspace(L.gtsfm_ransac_workspace_bytes(P, mcap), dev)
        if stream is not None:
            ws.record_stream(stream)
        rc = L.gtsfm_ransac_E_batched(_ptr(kp_xy), _ptr(intrinsics), n_img, kmax, _ptr(pairs), P, _ptr(match_idx),
                                      _ptr(match_count), mcap, float(thr_px), float(prob), int(max_iters), int(scoring),
                                      int(seed),
                                      int(pair_id_base), _ptr(pair_ids), _ptr(ws), ws.numel(), _ptr(E), _ptr(R), _ptr(t),
                                      _ptr(n_inl), _ptr(status), _ptr(n_hyp), _ptr(n_models), _ptr(mask),
                                      native.stream_handle(stream))
        native.check(rc, "gtsfm_ransac_E_batched")
    return RansacResult(E[:P], R[:P], t[:P], n_inl[:P], status[:P], n_hyp[:P], mask[:P], n_models[:P])


def compact_verified(match_idx: torch.Tensor, match_count: torch.Tensor, res: "RansacResult", min_inliers: int,
                     min_inlier_ratio: float, capacity: int, out_offsets: Optional[torch.Tensor] = None,
                     out_v_corr: Optional[torch.Tensor] = None, out_isp_ok: Optional[torch.Tensor] = None,
                     stream: Optional[torch.cuda.Stream] = None, ratio_inliers: Optional[torch.Tensor] = None
                     ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Inlier rows of every pair, concatenated in pair order, + the inlier-support verdict (gtsfm_compact_verified).
    `res` supplies mask / status / n_inliers (a RansacResult, or a BA2Result for the post-BA rows); ratio_inliers
    optionally gives the counts the inlier ratio is taken on (the pre-BA ones after BA).

    Returns offsets (P + 1,) int32, v_corr (capacity, 2) int32 holding uint32 indices (rows offsets[p] ..
    offsets[p + 1] belong to pair p, matcher order), isp_ok (P,) uint8.
    """
    assert match_idx.dtype == torch.int32 and match_idx.is_contiguous() and match_idx.dim() == 3
    P, mcap = match_idx.shape[0], match_idx.shape[1]
    assert res.mask.shape[0] == P and (P == 0 or res.mask.shape[1] == mcap) and res.mask.is_contiguous()
    dev = match_idx.device
    offsets = out_offsets if out_offsets is not None else torch.empty(P + 1, dtype=torch.int32, device=dev)
    v_corr = out_v_corr if out_v_corr is not None else torch.empty((max(capacity, 1), 2), dtype=torch.int32, device=dev)
    isp_ok = out_isp_ok if out_isp_ok is not None else torch.empty(max(P, 1), dtype=torch.uint8, device=dev)
    assert offsets.numel() >= P + 1 and v_corr.shape[0] >= capacity and isp_ok.numel() >= P
    rc = native.lib().gtsfm_compact_verified(_ptr(match_idx), _ptr(match_count), mcap, _ptr(res.mask),
                                             _ptr(res.status), _ptr(res.n_inliers), _ptr(ratio_inliers), P,
                                             int(min_inliers),
                                             float(min_inlier_ratio), _ptr(offsets), _ptr(v_corr), int(capacity),
                                             _ptr(isp_ok), native.stream_handle(stream))
    native.check(rc, "gtsfm_compact_verified")
    return offsets, v_corr, isp_ok


class BA2Result:
    """Post-BA per-pair outputs (device tensors): R (i2Ri1), t (unit i2ti1), mask (P, mcap) over the putatives,
    n_inliers (its row count), ba_status (0 ok, 1 no track, 2 none valid, 3 not run), iters, and `status` = the
    verifier's status (what the reference's R is None / not None follows)."""

    def __init__(self, R, t, mask, n_inliers, ba_status, iters, status):
        self.R, self.t, self.mask, self.n_inliers = R, t, mask, n_inliers
        self.ba_status, self.iters, self.status = ba_status, iters, status


def bundle_adjust_2view(kp_xy: torch.Tensor, intrinsics: torch.Tensor, pairs: torch.Tensor, match_idx: torch.Tensor,
                        match_count: torch.Tensor, res: "RansacResult", min_inliers: int = 15, max_iters: int = 100,
                        reproj_thresh: float = 0.5, tri_thresh: float = 100.0,
                        stream: Optional[torch.cuda.Stream] = None, prior_Rt: Optional[torch.Tensor] = None,
                        prior_sigmas: Optional[torch.Tensor] = None) -> BA2Result:
    """Two-view triangulation + bundle adjustment of every verified pair (gtsfm_ba2_batched) on the verifier's
    outputs `res` (same tensors as ransac_essential took). prior_Rt (P, 12) float64 (i2Ti1 R row-major, t) and
    prior_sigmas (P, 6) float64: optional relative-pose priors (a row with sigma[0] <= 0 has none)."""
    assert kp_xy.is_cuda and kp_xy.dtype == torch.float32 and kp_xy.is_contiguous()
    assert intrinsics.dtype == torch.float64 and match_idx.dtype == torch.int32 and match_idx.is_contiguous()
    assert (prior_Rt is None) == (prior_sigmas is None)
    if prior_Rt is not None:
        assert prior_Rt.dtype == torch.float64 and prior_Rt.is_contiguous() and prior_Rt.is_cuda
        assert prior_sigmas.dtype == torch.float64 and prior_sigmas.is_contiguous() and prior_sigmas.is_cuda
        assert tuple(prior_Rt.shape) == (match_idx.shape[0], 12) and tuple(prior_sigmas.shape) == (match_idx.shape[0], 6)
    n_img, kmax = kp_xy.shape[0], kp_xy.shape[1]
    P, mcap = match_idx.shape[0], match_idx.shape[1]
    dev = kp_xy.device
    L = native.lib()
    R = torch.zeros((max(P, 1), 3, 3), dtype=torch.float64, device=dev)
    t = torch.zeros((max(P, 1), 3), dtype=torch.float64, device=dev)
    mask = torch.zeros((max(P, 1), max(mcap, 1)), dtype=torch.uint8, device=dev)
    n_out = torch.zeros(max(P, 1), dtype=torch.int32, device=dev)
    st = torch.zeros_like(n_out)
    iters = torch.zeros_like(n_out)
    if P > 0:
        ws = _workspace(L.gtsfm_ba2_workspace_bytes(P, mcap), dev)
        if stream is not None:
            ws.record_stream(stream)
        rc = L.gtsfm_ba2_batched(_ptr(kp_xy), _ptr(intrinsics), n_img, kmax, _ptr(pairs), P, _ptr(match_idx),
                                 _ptr(match_count), mcap, _ptr(res.mask), _ptr(res.R.contiguous()),
                                 _ptr(res.t.contiguous()), _ptr(res.status), _ptr(prior_Rt), _ptr(prior_sigmas),
                                 int(min_inliers), int(max_iters),
                                 float(reproj_thresh), float(tri_thresh), _ptr(ws), ws.numel(), _ptr(R), _ptr(t),
                                 _ptr(mask), _ptr(n_out), _ptr(st), _ptr(iters), native.stream_handle(stream))
        native.check(rc, "gtsfm_ba2_batched")
    return BA2Result(R[:P], t[:P], mask[:P], n_out[:P], st[:P], iters[:P], res.status)


def sampson_sq(F: torch.Tensor, row_pair: torch.Tensor, x1: torch.Tensor, x2: torch.Tensor,
               precision: int = native.GTSFM_SAMPSON_F64, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """Squared Sampson distance of row r = (x1[r], x2[r]) under F[row_pair[r]] (gtsfm_sampson_sq_batched).

    F: (n_mats, 3, 3) float64; row_pair: (N,) int32; x1, x2: (N, 2) float64. Returns (N,) float64.
    """
    assert F.dtype == torch.float64 and F.is_contiguous() and F.is_cuda
    assert x1.dtype == torch.float64 and x2.dtype == torch.float64 and x1.is_contiguous() and x2.is_contiguous()
    assert row_pair.dtype == torch.int32 and row_pair.numel() == x1.shape[0] == x2.shape[0]
    out = torch.empty(max(x1.shape[0], 1), dtype=torch.float64, device=F.device)
    rc = native.lib().gtsfm_sampson_sq_batched(_ptr(F), F.shape[0], _ptr(row_pair), _ptr(x1), _ptr(x2), x1.shape[0],
                                               int(precision), _ptr(out), native.stream_handle(stream))
    native.check(rc, "gtsfm_sampson_sq_batched")
    return out[: x1.shape[0]]


class FundamentalResult(RansacResult):
    """Per-pair F-path outputs: F plus everything RansacResult holds (E = K2^T F K1)."""

    def __init__(self, F, E, R, t, n_inliers, status, n_hyp, mask):
        super().__init__(E, R, t, n_inliers, status, n_hyp, mask)
        self.F = F


def ransac_fundamental(kp_xy: torch.Tensor, intrinsics: torch.Tensor, pairs: torch.Tensor, match_idx: torch.Tensor,
                       match_count: torch.Tensor, thr_px: float, prob: float = 0.999999, max_iters: int = 1000000,
                       seed: int = native.RANSAC_DEFAULT_SEED, pair_id_base: int = 0,
                       pair_ids: Optional[torch.Tensor] = None,
                       stream: Optional[torch.cuda.Stream] = None) -> FundamentalResult:
    """Batched 7-point RANSAC / LMedS F estimation + 8-point refit + E + recoverPose (gtsfm_ransac_F_batched).

    Same tensor conventions as ransac_essential; thr_px is in pixels (no focal-length scaling).
    """
    assert kp_xy.is_cuda and kp_xy.dtype == torch.float32 and kp_xy.dim() == 3 and kp_xy.is_contiguous()
    assert intrinsics.dtype == torch.float64 and intrinsics.is_contiguous()
    assert match_idx.dtype == torch.int32 and match_idx.is_contiguous() and match_count.dtype == torch.int32
    assert pair_ids is None or (pair_ids.dtype == torch.int32 and pair_ids.is_cuda and pair_ids.numel() == pairs.shape[0])
    n_img, kmax, _ = kp_xy.shape
    P = pairs.shape[0]
    mcap = match_idx.shape[1]
    dev = kp_xy.device
    L = native.lib()
    F = torch.zeros((max(P, 1), 3, 3), dtype=torch.float64, device=dev)
    E, R = torch.zeros_like(F), torch.zeros_like(F)
    t = torch.zeros((max(P, 1), 3), dtype=torch.float64, device=dev)
    n_inl = torch.zeros((max(P, 1),), dtype=torch.int32, device=dev)
    status, n_hyp = torch.zeros_like(n_inl), torch.zeros_like(n_inl)
    mask = torch.zeros((max(P, 1), max(mcap, 1)), dtype=torch.uint8, device=dev)
    if P > 0:
        ws = _workspace(L.gtsfm_ransac_F_workspace_bytes(P, mcap), dev)
        if stream is not None:
            ws.record_stream(stream)
        rc = L.gtsfm_ransac_F_batched(_ptr(kp_xy), _ptr(intrinsics), n_img, kmax, _ptr(pairs), P, _ptr(match_idx),
                                      _ptr(match_count), mcap, float(thr_px), float(prob), int(max_iters), int(seed),
                                      int(pair_id_base), _ptr(pair_ids), _ptr(ws), ws.numel(), _ptr(F), _ptr(E),
                                      _ptr(R), _ptr(t), _ptr(n_inl), _ptr(status), _ptr(n_hyp), _ptr(mask),
                                      native.stream_handle(stream))
        native.check(rc, "gtsfm_ransac_F_batched")
    return FundamentalResult(F[:P], E[:P], R[:P], t[:P], n_inl[:P], status[:P], n_hyp[:P], mask[:P])


class SiftResult:
    """Per-image SIFT outputs (device tensors): xy (n,k,2), attr (n,k,3) size/angle/response, desc (n,k,128),
    count (n,), n_detected (n,)."""

    def __init__(self, xy, attr, desc, count, n_detected):
        self.xy, self.attr, self.desc, self.count, self.n_detected = xy, attr, desc, count, n_detected


def sift_extract(images: torch.Tensor, max_kpts: int, stream: Optional[torch.cuda.Stream] = None,
                 out: Optional[SiftResult] = None, workspace: Optional[torch.Tensor] = None,
                 masks: Optional[torch.Tensor] = None) -> SiftResult:
    """SIFT + top-k on a batch of same-sized uint8 images (n, H, W) gray or (n, H, W, 3) RGB (gtsfm_sift_batched).
    masks: optional (n, H, W) uint8; keypoints on zero pixels are dropped before the top-k."""
    assert images.is_cuda and images.dtype == torch.uint8 and images.is_contiguous()
    assert masks is None or (masks.is_cuda and masks.dtype == torch.uint8 and masks.is_contiguous()
                             and tuple(masks.shape) == tuple(images.shape[:3]))
    n = images.shape[0]
    H, W = images.shape[1], images.shape[2]
    C = 1 if images.dim() == 3 else images.shape[3]
    dev = images.device
    L = native.lib()
    if out is None:
        out = SiftResult(torch.empty((n, max_kpts, 2), dtype=torch.float32, device=dev),
                         torch.empty((n, max_kpts, 3), dtype=torch.float32, device=dev),
                         torch.empty((n, max_kpts, 128), dtype=torch.float32, device=dev),
                         torch.empty((n,), dtype=torch.int32, device=dev),
                         torch.empty((n,), dtype=torch.int32, device=dev))
    nbytes = L.gtsfm_sift_workspace_bytes(n, H, W, max_kpts)
    ws = workspace if workspace is not None and workspace.numel() >= nbytes else _workspace(nbytes, dev)
    if stream is not None:
        ws.record_stream(stream)
    rc = L.gtsfm_sift_batched(_ptr(images), _ptr(masks), n, H, W, C, max_kpts, _ptr(ws), ws.numel(), _ptr(out.xy),
                              _ptr(out.attr),
                              _ptr(out.desc), _ptr(out.count), _ptr(out.n_detected), native.stream_handle(stream))
    native.check(rc, "gtsfm_sift_batched")
    return out


class SuperPointResult:
    """Per-image SuperPoint outputs (device tensors): xy (n,k,2) float32 (x, y), scores (n,k), desc (n,k,256),
    count (n,), n_detected (n,)."""

    def __init__(self, xy, scores, desc, count, n_detected):
        self.xy, self.scores, self.desc, self.count, self.n_detected = xy, scores, desc, count, n_detected


def superpoint_extract(images: torch.Tensor, weights: torch.Tensor, max_kpts: int, keypoint_threshold: float = 0.005,
                       nms_radius: int = 4, remove_borders: int = 4,
                       stream: Optional[torch.cuda.Stream] = None, out: Optional[SuperPointResult] = None,
                       workspace: Optional[torch.Tensor] = None, masks: Optional[torch.Tensor] = None
                       ) -> SuperPointResult:
    """SuperPoint on a batch of same-sized uint8 images (n, H, W) gray or (n, H, W, 3) RGB (gtsfm_superpoint_batched).

    weights: the packed fp32 blob (gtsfm_amd.frontend.detector_descriptor.superpoint.pack_superpoint_weights).
    out: optional preallocated outputs (xy (n,k,2), scores (n,k), desc (n,k,256), count, n_detected; rows past a
    count are unspecified); workspace: optional device buffer of at least gtsfm_superpoint_workspace_bytes.
    masks: optional (n, H, W) uint8 device tensor; a detection at (x, y) is kept iff masks[i, y, x] == 1 (the
    reference's Keypoints.filter_by_mask), before the top-k.
    """
    assert images.is_cuda and images.dtype == torch.uint8 and images.is_contiguous()
    assert weights.is_cuda and weights.dtype == torch.float32 and weights.is_contiguous()
    L = native.lib()
    assert weights.numel() == L.gtsfm_superpoint_weights_floats()
    n, H, W = images.shape[0], images.shape[1], images.shape[2]
    C = 1 if images.dim() == 3 else images.shape[3]
    dev = images.device
    if out is None:
        out = SuperPointResult(torch.zeros((n, max_kpts, 2), dtype=torch.float32, device=dev),
                               torch.zeros((n, max_kpts), dtype=torch.float32, device=dev),
                               torch.empty((n, max_kpts, 256), dtype=torch.float32, device=dev),
                               torch.zeros((n,), dtype=torch.int32, device=dev),
                               torch.zeros((n,), dtype=torch.int32, device=dev))
    for t, shape in ((out.xy, (n, max_kpts, 2)), (out.scores, (n, max_kpts)), (out.desc, (n, max_kpts, 256))):
        assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == shape
    if n == 0:
        return out
    need = L.gtsfm_superpoint_workspace_bytes(n, H, W, max_kpts)
    ws = workspace if workspace is not None and workspace.numel() >= need else _workspace(need, dev)
    if stream is not None:
        ws.record_stream(stream)
    if masks is not None:
        assert masks.is_cuda and masks.dtype == torch.uint8 and masks.is_contiguous()
        assert tuple(masks.shape) == (n, H, W), (tuple(masks.shape), (n, H, W))
    rc = L.gtsfm_superpoint_batched(_ptr(images), _ptr(masks) if masks is not None else None, n, H, W, C,
                                    _ptr(weights), max_kpts, float(keypoint_threshold),
                                    int(nms_radius), int(remove_borders), _ptr(ws), ws.numel(), _ptr(out.xy),
                                    _ptr(out.scores), _ptr(out.desc), _ptr(out.count), _ptr(out.n_detected),
                                    native.stream_handle(stream))
    native.check(rc, "gtsfm_superpoint_batched")
    return out


def superglue_match(kp: torch.Tensor, scores: torch.Tensor, desc: torch.Tensor, counts: torch.Tensor,
                    image_hw: torch.Tensor, pairs: torch.Tensor, weights: torch.Tensor, n_layers: int = 18,
                    sinkhorn_iters: int = 20, match_threshold: float = 0.2,
                    stream: Optional[torch.cuda.Stream] = None, workspace: Optional[torch.Tensor] = None
                    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """SuperGlue over every pair (gtsfm_superglue_batched).

    Args: kp (n_img, kmax, 2) f32, scores (n_img, kmax) f32, desc (n_img, kmax, 256) f32, counts (n_img,) int32,
    image_hw (n_img, 2) int32 (H, W), pairs (P, 2) int32, weights: the packed blob. kmax must be a multiple of 64.
    Returns idx (P, kmax, 2) int32 (uint32 values, i ascending), count (P,) int32, mscores0 (P, kmax) f32.
    """
    for t in (kp, scores, desc, weights):
        assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
    assert counts.dtype == torch.int32 and image_hw.dtype == torch.int32 and pairs.dtype == torch.int32
    n_img, kmax = kp.shape[0], kp.shape[1]
    assert kmax % 64 == 0 and desc.shape == (n_img, kmax, 256) and scores.shape == (n_img, kmax)
    L = native.lib()
    assert weights.numel() == L.gtsfm_superglue_weights_floats(n_layers)
    P = pairs.shape[0]
    dev = kp.device
    idx = torch.zeros((max(P, 1), kmax, 2), dtype=torch.int32, device=dev)
    cnt = torch.zeros((max(P, 1),), dtype=torch.int32, device=dev)
    ms = torch.zeros((max(P, 1), kmax), dtype=torch.float32, device=dev)
    if P > 0:
        need = L.gtsfm_superglue_workspace_bytes(P, kmax)
        ws = workspace if workspace is not None and workspace.numel() >= need else _workspace(need, dev)
        if stream is not None:
            ws.record_stream(stream)
        rc = L.gtsfm_superglue_batched(_ptr(kp), _ptr(scores), _ptr(desc), _ptr(counts), _ptr(image_hw), n_img, kmax,
                                       _ptr(pairs), P, _ptr(weights), int(n_layers), int(sinkhorn_iters),
                                       float(match_threshold), _ptr(ws), ws.numel(), _ptr(idx), _ptr(cnt), _ptr(ms),
                                       native.stream_handle(stream))
        native.check(rc, "gtsfm_superglue_batched")
    return idx[:P], cnt[:P], ms[:P]


def superglue_log_assignment(workspace: torch.Tensor, n_pairs: int, kmax: int, pair: int,
                             stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """Pair `pair`'s final log-assignment matrix (kmax + 1, kmax + 1) from the workspace of the superglue_match call
    that used `workspace` (gtsfm_superglue_log_assignment; entries past (m + 1, n + 1) are NaN)."""
    out = torch.empty((kmax + 1, kmax + 1), dtype=torch.float32, device=workspace.device)
    rc = native.lib().gtsfm_superglue_log_assignment(_ptr(workspace), workspace.numel(), n_pairs, kmax, pair, _ptr(out),
                                                     native.stream_handle(stream))
    native.check(rc, "gtsfm_superglue_log_assignment")
    return out


def retrieval_similarity(desc: torch.Tensor, blocksize: int,
                         stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """(N, N) f32 block-upper-triangular similarity of N global descriptors (N, D) f32 on the device
    (gtsfm_retrieval_similarity; netvlad_retriever.py:77-149)."""
    if desc.dim() != 2 or desc.dtype != torch.float32 or not desc.is_cuda:
        raise ValueError("desc must be a (N, D) float32 device tensor")
    desc = desc.contiguous()
    n, d = desc.shape
    sim = torch.empty((n, n), dtype=torch.float32, device=desc.device)
    if n == 0:
        return sim
    native.check(native.lib().gtsfm_retrieval_similarity(_ptr(desc), n, d, int(blocksize), _ptr(sim),
                                                         native.stream_handle(stream)),
                 "gtsfm_retrieval_similarity")
    return sim


def retrieval_pairs(scores: torch.Tensor, num_select: int, min_score: Optional[float],
                    invalid: Optional[torch.Tensor] = None,
                    stream: Optional[torch.cuda.Stream] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k valid pairs per row of a (K1, K2) f32 device score matrix (gtsfm_retrieval_pairs;
    netvlad_retriever.py:196-228). invalid: (K1, K2) bool device mask, None = every entry not strictly above the
    diagonal (:164-167). Returns (pairs (K1, k, 2) int32, row_count (K1,) int32): row i's first row_count[i] entries
    are its finite top-k pairs in rank order."""
    if scores.dim() != 2 or scores.dtype != torch.float32 or not scores.is_cuda:
        raise ValueError("scores must be a (K1, K2) float32 device tensor")
    if num_select < 0:
        raise ValueError("num_select must be >= 0")
    scores = scores.contiguous()
    n1, n2 = scores.shape
    k = min(int(num_select), n1)
    if k > n2:
        raise RuntimeError(f"selected index k={k} out of range for {n2} columns")  # torch.topk's error
    inv = None
    if invalid is not None:
        if tuple(invalid.shape) != (n1, n2):
            raise ValueError("invalid must have the shape of scores")
        inv = invalid.to(device=scores.device, dtype=torch.uint8).contiguous()
    out = torch.empty((n1, k, 2), dtype=torch.int32, device=scores.device)
    cnt = torch.zeros((n1,), dtype=torch.int32, device=scores.device)
    if n1 == 0:
        return out, cnt
    use_min = min_score is not None
    native.check(native.lib().gtsfm_retrieval_pairs(_ptr(scores), n1, n2, _ptr(inv), int(num_select),
                                                    float(min_score) if use_min else 0.0, int(use_min), _ptr(out),
                                                    _ptr(cnt), native.stream_handle(stream)),
                 "gtsfm_retrieval_pairs")
    return out, cnt


def netvlad_describe(images: torch.Tensor, weights: torch.Tensor, whiten: bool = True,
                     stream: Optional[torch.cuda.Stream] = None, workspace: Optional[torch.Tensor] = None,
                     keep_vlad: bool = False) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """NetVLAD global descriptors of a batch of same-sized (n, H, W, 3) uint8 RGB images (gtsfm_netvlad_batched).

    weights: the packed fp32 blob (gtsfm_amd.frontend.global_descriptor.netvlad_global_descriptor.pack_netvlad_weights).
    Returns (desc (n, 4096) f32 or None when whiten is False, vlad (n, 32768) f32 or None unless keep_vlad or
    not whiten): the whitened, L2-normalised descriptor and the NetVLADLayer output before whitening."""
    assert images.is_cuda and images.dtype == torch.uint8 and images.is_contiguous() and images.dim() == 4
    assert images.shape[3] == 3, "NetVLAD takes RGB images (netvlad.py:172: image.shape[1] == 3)"
    assert weights.is_cuda and weights.dtype == torch.float32 and weights.is_contiguous()
    L = native.lib()
    assert weights.numel() == L.gtsfm_netvlad_weights_floats()
    n, H, W = images.shape[0], images.shape[1], images.shape[2]
    dev = images.device
    desc = torch.empty((n, 4096), dtype=torch.float32, device=dev) if whiten else None
    vlad = torch.empty((n, 32768), dtype=torch.float32, device=dev) if (keep_vlad or not whiten) else None
    if n == 0:
        return desc, vlad
    need = L.gtsfm_netvlad_workspace_bytes(n, H, W)
    ws = workspace if workspace is not None and workspace.numel() >= need else _workspace(need, dev)
    if stream is not None:
        ws.record_stream(stream)
    rc = L.gtsfm_netvlad_batched(_ptr(images), n, H, W, 3, _ptr(weights), int(bool(whiten)), _ptr(vlad), _ptr(desc),
                                 _ptr(ws), ws.numel(), native.stream_handle(stream))
    native.check(rc, "gtsfm_netvlad_batched")
    return desc, vlad
