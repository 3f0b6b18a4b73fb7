"""All-pairs two-view front-end of one rank: images in host memory -> per-pair (R, t, v_corr, inlier count) in host
memory, the unit SURVEY.md §8(d) times.

This is the batched engine behind the drop-ins: it replaces the reference's Dask fan-out of
`DetDescCorrespondenceGenerator.generate_correspondences` (det_desc_correspondence_generator.py:31-87: one
detect_and_describe task per image, one match task per pair) followed by `run_two_view_estimator_as_futures`
(two_view_estimator.py:531-587: one verify + inlier-support task per pair), with on-device batches:

1. H2D + extraction, pipelined: the rank's images go up from pinned host memory in chunks on a copy stream while
   the detector-descriptor runs on the previous chunk (`kernels.extract`, one batched launch sequence per chunk:
   SIFT, or SuperPoint for the deep front-end).
2. The one exchange (N > 1): all-gather of the padded per-rank feature blocks (gtsfm_amd/frontend/sharding.py).
3. Per block of pairs: matching (`kernels.match`: mutual-NN + ratio, or SuperGlue), 5-point RANSAC + LO + recoverPose
   (`kernels.verify`), optionally the two-view triangulation + bundle adjustment (`kernels.bundle_adjust`,
   TwoViewEstimator's bundle_adjust_2view), then compaction of the verified rows + the inlier-support verdict
   (`kernels.compact`).
4. D2H of the compact results into pinned host buffers: fixed-size per-pair records first, then exactly the verified
   rows once their total is known.

The kernels come from an object (default `HipKernels`: SIFT + TwoWayMatcher in libgtsfm_hip.so;
`HipSuperPointKernels`: SuperPoint + TwoWayMatcher or SuperGlue, BASELINE configs C3 / C5). The control flow, the
sharding and the buffers do not depend on it, so tests drive this same class under gloo on CPU with the oracle standing in for the
device (tests/test_launcher.py). The product path has no CPU fallback: `HipKernels` fails when the library or the GPU
is missing.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from gtsfm_amd.frontend import sharding


@dataclass
class FrontEndConfig:
    kpts: int = 2048                 # SIFT max_keypoints (BASELINE configs C2 / C4)
    ratio: float = 0.8               # TwoWayMatcher ratio_test_threshold (sift_front_end.yaml)
    thresh_px: float = 4.0           # Ransac estimation_threshold_px (sift_front_end.yaml:48)
    min_inliers: int = 15            # InlierSupportProcessor min_num_inliers_est_model
    min_inlier_ratio: float = 0.1    # InlierSupportProcessor min_inlier_ratio_est_model
    extract_chunk: int = 40          # host steps: images per SIFT launch sequence (the next chunk's H2D overlaps it)
    extract_first: int = 20          # host steps: size of a smaller first chunk (less exposed H2D); 0 = extract_chunk
    resident_chunk: int = 100        # device-resident steps: images per SIFT launch sequence (bounded by workspace)
    pair_chunk: int = 131072         # pairs per match / verify / compact launch sequence (C4: 272k -> 283k pairs/s vs 32768)
    overlap: bool = True             # match of pair chunk c + 1 on a second stream while chunk c verifies
    bundle_adjust: bool = False      # TwoViewEstimator bundle_adjust_2view: two-view triangulation + BA after RANSAC
    ba_max_iters: int = 100          # bundle_adjust_2view_maxiters
    ba_reproj_thresh: float = 0.5    # ba_reproj_error_thresholds[-1]
    tri_reproj_thresh: float = 100.0  # TriangulationOptions.reproj_error_threshold (sift_front_end.yaml)


class HipKernels:
    """The product kernels of the SIFT front-end (SIFTDetectorDescriptor + TwoWayMatcher + Ransac):
    libgtsfm_hip.so through gtsfm_amd.device (no fallback).

    The kernel-set interface AllPairsFrontEnd drives: per-image attribute / descriptor widths, the fields the pair
    stages read (all-gathered over the ranks, each in its wire dtype), extract_workspace_bytes / extract, match_groups
    / match, verify, bundle_adjust, compact."""

    attr_dim, desc_dim = 3, 128  # SIFT: (size, angle, response) per keypoint, 128-D descriptors
    # SIFT descriptors are integer-valued in [0, 255]: they travel as u8 (lossless, a quarter of the f32 bytes)
    gather = (("xy", None), ("desc", torch.uint8), ("count", None))
    max_pair_chunk: Optional[int] = None  # no workspace limit below FrontEndConfig.pair_chunk

    def __init__(self):
        from gtsfm_amd import device, native

        native.require_gpu()
        native.lib()
        self._dev, self._native = device, native

    def extract_workspace_bytes(self, n: int, H: int, W: int, kpts: int) -> int:
        return int(self._native.lib().gtsfm_sift_workspace_bytes(n, H, W, kpts))

    def extract(self, images, kpts, out, workspace):
        self._dev.sift_extract(images, kpts, out=out, workspace=workspace)

    def match_groups(self, pairs: np.ndarray, kmax: int, dim: int) -> Optional[np.ndarray]:
        """Block-tiled pair groups for the distance GEMM (gtsfm_match_batched_grouped), sized to fill the GPU, or None."""
        return self._dev.match_plan(pairs, kmax, dim)

    def match(self, f: "Features", pairs, ratio, groups=None, image_hw=None, out=None):
        return self._dev.match_pairs(f.desc, f.count, pairs, ratio, self._native.GTSFM_MATCH_INT_F16, groups=groups,
                                     out=out)

    def verify(self, xy, intr, pairs, idx, cnt, thresh_px, pair_ids):
        return self._dev.ransac_essential(xy, intr, pairs, idx, cnt, thresh_px, pair_ids=pair_ids)

    def bundle_adjust(self, xy, intr, pairs, idx, cnt, res, min_inliers, max_iters, reproj_thresh, tri_thresh):
        return self._dev.bundle_adjust_2view(xy, intr, pairs, idx, cnt, res, min_inliers, max_iters, reproj_thresh,
                                             tri_thresh)

    def compact(self, idx, cnt, res, min_inliers, min_ratio, capacity, out_offsets, out_v_corr, out_isp_ok,
                ratio_inliers=None):
        self._dev.compact_verified(idx, cnt, res, min_inliers, min_ratio, capacity, out_offsets=out_offsets,
                                   out_v_corr=out_v_corr, out_isp_ok=out_isp_ok, ratio_inliers=ratio_inliers)


class HipSuperPointKernels(HipKernels):
    """The deep front-end (BASELINE configs C3 / C5): SuperPointDetectorDescriptor (superpoint.hip) with either
    TwoWayMatcher on its float descriptors (F16_RERANK: fp16 MFMA shortlist + certified exact re-rank; config C3) or
    SuperGlueMatcher (superglue.hip; config C5), then the same verifier / compaction kernels.

    superpoint_weights / superglue_weights: the packed fp32 device blobs (pack_superpoint_weights /
    pack_superglue_weights). SuperGlue's workspace is ~59 MB per pair at 2048 keypoints, so its pair chunks are
    capped at superglue_pair_chunk."""

    attr_dim, desc_dim = 1, 256  # SuperPoint: score per keypoint, 256-D unit descriptors

    def __init__(self, superpoint_weights: torch.Tensor, matcher: str = "twoway",
                 superglue_weights: Optional[torch.Tensor] = None, n_layers: int = 18, sinkhorn_iterations: int = 20,
                 match_threshold: float = 0.2, keypoint_threshold: float = 0.005, nms_radius: int = 4,
                 remove_borders: int = 4, superglue_pair_chunk: int = 1024):
        super().__init__()
        if matcher not in ("twoway", "superglue"):
            raise ValueError(f"matcher must be 'twoway' or 'superglue', not {matcher!r}")
        if matcher == "superglue" and superglue_weights is None:
            raise ValueError("the superglue matcher needs its weight blob")
        self.matcher = matcher
        self.sp_w, self.sg_w = superpoint_weights, superglue_weights
        self.n_layers, self.iters, self.match_thr = n_layers, sinkhorn_iterations, match_threshold
        self.kp_thr, self.nms, self.border = keypoint_threshold, nms_radius, remove_borders
        # float descriptors travel as f32 (no lossless narrower wire); SuperGlue also reads the keypoint scores
        self.gather = (("xy", None), ("attr", None), ("desc", None), ("count", None)) if matcher == "superglue" else \
            (("xy", None), ("desc", None), ("count", None))
        self.max_pair_chunk = superglue_pair_chunk if matcher == "superglue" else None
        self._sg_ws: Optional[torch.Tensor] = None

    def extract_workspace_bytes(self, n: int, H: int, W: int, kpts: int) -> int:
        return int(self._native.lib().gtsfm_superpoint_workspace_bytes(n, H, W, kpts))

    def extract(self, images, kpts, out, workspace):
        res = self._dev.SuperPointResult(out.xy, out.attr.select(-1, 0), out.desc, out.count, out.n_detected)
        self._dev.superpoint_extract(images, self.sp_w, kpts, self.kp_thr, self.nms, self.border, out=res,
                                     workspace=workspace)

    def match_groups(self, pairs: np.ndarray, kmax: int, dim: int) -> Optional[np.ndarray]:
        return None

    def match(self, f: "Features", pairs, ratio, groups=None, image_hw=None, out=None):
        if self.matcher == "twoway":
            return self._dev.match_pairs(f.desc, f.count, pairs, ratio, self._native.GTSFM_MATCH_F16_RERANK, out=out)
        kmax = f.desc.shape[1]
        need = int(self._native.lib().gtsfm_superglue_workspace_bytes(int(pairs.shape[0]), kmax))
        if self._sg_ws is None or self._sg_ws.numel() < need:
            self._sg_ws = torch.empty(need, dtype=torch.uint8, device=f.desc.device)
        idx, cnt, _ = self._dev.superglue_match(f.xy, f.attr.select(-1, 0).contiguous(), f.desc, f.count, image_hw,
                                                pairs, self.sg_w, self.n_layers, self.iters, self.match_thr,
                                                workspace=self._sg_ws)
        return idx, cnt


class Features:
    """Per-image extraction outputs of one rank (device tensors): xy (n,k,2), attr (n,k,A), desc (n,k,D), count (n,),
    n_detected (n,). SIFT: A = 3 (size, angle, response), D = 128 (gtsfm_amd.device.SiftResult's fields); SuperPoint:
    A = 1 (score), D = 256."""

    def __init__(self, xy, attr, desc, count, n_detected):
        self.xy, self.attr, self.desc, self.count, self.n_detected = xy, attr, desc, count, n_detected

    def rows(self, a: int, b: int) -> "Features":
        return Features(self.xy[a:b], self.attr[a:b], self.desc[a:b], self.count[a:b], self.n_detected[a:b])


@dataclass
class HostResults:
    """Per-pair results of one rank in host memory (numpy views of pinned buffers, valid until the next step).

    pairs[p] = (i1, i2) original image indices; R[p] = i2Ri1, t[p] = unit i2ti1; status[p] 0 ok / 1 too few
    putatives / 2 no model; n_inliers[p]; n_matches[p] = putatives; isp_ok[p] = passes the inlier-support filter;
    v_corr[offsets[p]:offsets[p+1]] = pair p's verified (i1 kp, i2 kp) rows in matcher order (uint32).
    kp_xy / kp_count: this rank's keypoints (local image order, sharding.local_images).
    """
    pairs: np.ndarray
    R: np.ndarray
    t: np.ndarray
    status: np.ndarray
    n_inliers: np.ndarray
    n_matches: np.ndarray
    isp_ok: np.ndarray
    offsets: np.ndarray
    v_corr: np.ndarray
    kp_xy: np.ndarray
    kp_count: np.ndarray

    def verified(self, p: int) -> np.ndarray:
        return self.v_corr[self.offsets[p]: self.offsets[p + 1]]


class AllPairsFrontEnd:
    """One rank's share of the all-pairs front-end (images i with i % world == rank, pairs p with p % world == rank)."""

    def __init__(self, host_images: torch.Tensor, intrinsics: np.ndarray, n_img: int, rank: int, world: int,
                 device: torch.device, cfg: Optional[FrontEndConfig] = None, kernels=None,
                 image_pairs: Optional[np.ndarray] = None, exchange=None, pair_limit: Optional[int] = None):
        """image_pairs: (P, 2) global (i1, i2) pairs to match and verify, e.g. a retriever's output
        (gtsfm_amd.retriever; image_pairs_generator.py:29-47); None = every pair (ExhaustiveRetriever).
        exchange: None (the collective over torch.distributed), or a sharding.EmulatedAllGather when one process runs
        rank `rank`'s share of a `world`-rank job (bench.py --emulate-world).
        pair_limit: keep only the first pair_limit pairs of this rank's share (a bounded partial run of a job whose
        full block would take minutes per step; bench.py --pair-limit)."""
        self.cfg = cfg or FrontEndConfig()
        self.exchange = exchange
        self.kern = kernels if kernels is not None else HipKernels()
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.rank, self.world, self.n_img = rank, world, n_img
        assert host_images.dtype == torch.uint8 and host_images.device.type == "cpu" and host_images.dim() in (3, 4)
        n_local = host_images.shape[0]
        if n_local != len(sharding.local_images(n_img, world, rank)):
            raise ValueError(f"rank {rank} holds {n_local} images, expected {len(sharding.local_images(n_img, world, rank))}")
        H, W = host_images.shape[1], host_images.shape[2]
        k = self.cfg.kpts
        self.n_local = n_local
        self.host_images = host_images.contiguous()
        if self.cuda and not self.host_images.is_pinned():
            self.host_images = self.host_images.pin_memory()
        self.dev_images = torch.empty_like(self.host_images, device=self.dev)
        self.n_per = sharding.images_per_rank(n_img, world)
        z = dict(device=self.dev)
        A, D = getattr(self.kern, "attr_dim", 3), getattr(self.kern, "desc_dim", 128)
        self.desc_dim = D
        self.feats = Features(torch.zeros((n_local, k, 2), dtype=torch.float32, **z),
                              torch.zeros((n_local, k, A), dtype=torch.float32, **z),
                              torch.zeros((n_local, k, D), dtype=torch.float32, **z),
                              torch.zeros((n_local,), dtype=torch.int32, **z),
                              torch.zeros((n_local,), dtype=torch.int32, **z))
        def schedule(ch: int, first: int):
            ch = max(1, ch)
            first = first if 0 < first < ch else ch
            edges = [0] + list(range(min(first, n_local), n_local, ch)) + [n_local]
            return [(a, b) for a, b in zip(edges[:-1], edges[1:]) if b > a]

        self.chunks = schedule(self.cfg.extract_chunk, self.cfg.extract_first)
        self.chunks_resident = schedule(self.cfg.resident_chunk, 0)
        big = max([b - a for a, b in self.chunks + self.chunks_resident] + [1])
        ws = self.kern.extract_workspace_bytes(big, H, W, k) if n_local else 0
        self.extract_ws = torch.empty(max(int(ws), 256), dtype=torch.uint8, **z)

        slot = sharding.global_slots(n_img, world)
        if image_pairs is None:
            pairs = sharding.all_pairs(n_img)
        else:
            pairs = np.asarray(image_pairs, dtype=np.int64).reshape(-1, 2)
            if len(pairs) and (pairs.min() < 0 or pairs.max() >= n_img or np.any(pairs[:, 0] == pairs[:, 1])):
                raise ValueError("image_pairs must hold distinct image indices in [0, n_img)")
        self.total_pairs = len(pairs)
        block = sharding.rank_pairs(pairs, world, rank)
        if pair_limit is not None:
            block = block[: max(0, int(pair_limit))]
        # the global pair index keys the RANSAC sampler (a pair's result does not depend on the world size)
        self.pair_ids = torch.from_numpy(block.astype(np.int32)).to(self.dev)
        self.my_pairs = pairs[block]
        P = len(block)
        self.P = P
        self.pairs_dev = torch.from_numpy(slot[self.my_pairs].astype(np.int32)).to(self.dev)
        intr = np.zeros((world * self.n_per, 3))
        intr[slot] = intrinsics
        self.intr = torch.from_numpy(intr).to(self.dev)
        pc = max(1, self.cfg.pair_chunk)
        if getattr(self.kern, "max_pair_chunk", None):
            pc = min(pc, int(self.kern.max_pair_chunk))
        self.image_hw = torch.tensor([[H, W]] * (world * self.n_per), dtype=torch.int32, device=self.dev)
        self.pchunks = [(a, min(a + pc, P)) for a in range(0, P, pc)]
        # per pair chunk: workgroup groups of the distance GEMM (pairs sharing i1, i2 blocked), laid out once
        slot_pairs = slot[self.my_pairs].astype(np.int32)
        self.pgroups = []
        for a, b in self.pchunks:
            g = self.kern.match_groups(slot_pairs[a:b], k, D) if hasattr(self.kern, "match_groups") else None
            self.pgroups.append(None if g is None else torch.from_numpy(g).to(self.dev))

        # compact results on the device: per chunk c, offsets rows [a + c, b + c] and verified rows from a * k
        nc = len(self.pchunks)
        self.d_offsets = torch.zeros(P + nc, dtype=torch.int32, **z)
        self.d_v_corr = torch.zeros((max(P * k, 1), 2), dtype=torch.int32, **z)
        self.d_isp_ok = torch.zeros(max(P, 1), dtype=torch.uint8, **z)
        self.d_fixed = torch.zeros((max(P, 1), 12), dtype=torch.float64, **z)  # R (9) | t (3)
        self.d_ints = torch.zeros((max(P, 1), 3), dtype=torch.int32, **z)      # status | n_inliers | n_matches
        # matcher outputs, caller-owned and kept across steps: with the matcher one chunk ahead on its own stream,
        # per-step blocks would only return to the allocator once the compute stream caught up, so device-resident
        # steps queued back to back kept growing the pool until it synchronised and released everything (C4: 5
        # queued steps ran 1.86 s each against 1.17 s for 2). Step s + 1's matcher waits on the compute stream
        # (after the all-gather), so it never overwrites rows step s still reads.
        self.d_match = (torch.empty((max(P, 1), k, 2), dtype=torch.int32, **z),
                        torch.zeros(max(P, 1), dtype=torch.int32, **z)) if self.cuda else None
        self.stats: Dict[str, torch.Tensor] = {}

        pin = dict(pin_memory=self.cuda)
        self.h_offsets = torch.zeros(P + nc, dtype=torch.int32, **pin)
        self.h_v_corr = torch.zeros((max(P * k, 1), 2), dtype=torch.int32, **pin)
        self.h_isp_ok = torch.zeros(max(P, 1), dtype=torch.uint8, **pin)
        self.h_fixed = torch.zeros((max(P, 1), 12), dtype=torch.float64, **pin)
        self.h_ints = torch.zeros((max(P, 1), 3), dtype=torch.int32, **pin)
        self.h_xy = torch.zeros((n_local, k, 2), dtype=torch.float32, **pin)
        self.h_count = torch.zeros((n_local,), dtype=torch.int32, **pin)

        if self.cuda:
            self.copy_stream = torch.cuda.Stream(device=self.dev)
            self.copy_done = [torch.cuda.Event() for _ in self.chunks]
            self.match_stream = torch.cuda.Stream(device=self.dev)
            self.match_done = [torch.cuda.Event() for _ in self.pchunks]
        self.instrument = False
        self.marks: List[Tuple[str, object]] = []
        self.copy_marks: List[Tuple[str, object]] = []

    # -- instrumentation: HIP events on the stream each phase runs on (no-ops unless self.instrument) --
    def _mark(self, name: str, stream=None):
        if not (self.instrument and self.cuda):
            return
        ev = torch.cuda.Event(enable_timing=True)
        if stream is None:
            ev.record()
            self.marks.append((name, ev))
        else:
            ev.record(stream)
            self.copy_marks.append((name, ev))

    def stage_ms(self) -> Dict[str, float]:
        """Per-phase milliseconds of the last instrumented step (call after synchronising)."""
        out: Dict[str, float] = {}
        for (_, e0), (name, e1) in zip(self.marks[:-1], self.marks[1:]):
            out[name] = out.get(name, 0.0) + e0.elapsed_time(e1)
        if len(self.copy_marks) >= 2:
            out["h2d"] = self.copy_marks[0][1].elapsed_time(self.copy_marks[-1][1])
        return out

    def _extract(self, resident: bool):
        k = self.cfg.kpts
        cs = torch.cuda.current_stream(self.dev) if self.cuda else None
        if self.cuda and not resident:
            self.copy_stream.wait_stream(cs)  # the previous step's extraction has finished reading dev_images
            self._mark("h2d_start", self.copy_stream)
        for c, (a, b) in enumerate(self.chunks_resident if resident else self.chunks):
            if not resident:
                if self.cuda:
                    with torch.cuda.stream(self.copy_stream):
                        self.dev_images[a:b].copy_(self.host_images[a:b], non_blocking=True)
                        self.copy_done[c].record(self.copy_stream)
                    cs.wait_event(self.copy_done[c])
                else:
                    self.dev_images[a:b].copy_(self.host_images[a:b])
            self.kern.extract(self.dev_images[a:b], k, self.feats.rows(a, b), self.extract_ws)
        if self.cuda and not resident:
            self._mark("h2d_end", self.copy_stream)

    def packed_features(self) -> torch.Tensor:
        """This rank's packed exchange block of the last extraction (what it contributes to the all-gather)."""
        fields = getattr(self.kern, "gather", (("xy", None), ("desc", torch.uint8), ("count", None)))
        return sharding.pack_features([getattr(self.feats, n) for n, _ in fields], self.n_per,
                                      wire=[w for _, w in fields])[0]

    def step(self, resident: bool = False) -> Optional[HostResults]:
        """One pass of the front-end over this rank's share.

        resident=False (the contracted unit): H2D of the images from pinned host memory, ..., D2H of the results;
        returns HostResults. resident=True: the images already sit in HBM from an earlier step and the results stay
        there (returns None) -- the device-resident figure, reported beside the contracted one.
        """
        cfg, k = self.cfg, self.cfg.kpts
        self.marks, self.copy_marks = [], []
        self._mark("start")
        self._extract(resident)
        self._mark("extract")
        # the one exchange: the fields the pair stages read, each in the kernel set's wire dtype (one collective)
        fields = getattr(self.kern, "gather", (("xy", None), ("desc", torch.uint8), ("count", None)))
        got = sharding.allgather_features([getattr(self.feats, n) for n, _ in fields], self.n_per,
                                          wire=[w for _, w in fields], exchange=self.exchange)
        f_all = Features(**{n: None for n in ("xy", "attr", "desc", "count", "n_detected")})
        for (n, _), t in zip(fields, got):
            setattr(f_all, n, t)
        xy_all = f_all.xy
        self._mark("allgather")
        n_hyp, n_models, n_match = [], [], []
        # With several pair chunks, the matcher runs on its own stream one chunk ahead: the distance GEMM of chunk
        # c + 1 (MFMA) overlaps the RANSAC of chunk c (fp64 VALU) and fills the verifier's launch tails. Instrumented
        # steps stay sequential so that every stage's events bracket that stage alone.
        overlap = self.cuda and cfg.overlap and not self.instrument and len(self.pchunks) > 1
        matched = {}

        def issue_match(c: int):
            a, b = self.pchunks[c]
            kw = {} if self.d_match is None else {"out": (self.d_match[0][a:b], self.d_match[1][a:b])}
            if overlap:
                with torch.cuda.stream(self.match_stream):
                    matched[c] = self.kern.match(f_all, self.pairs_dev[a:b], cfg.ratio, groups=self.pgroups[c],
                                                 image_hw=self.image_hw, **kw)
                    self.match_done[c].record(self.match_stream)
            else:
                matched[c] = self.kern.match(f_all, self.pairs_dev[a:b], cfg.ratio, groups=self.pgroups[c],
                                             image_hw=self.image_hw, **kw)

        if overlap:
            self.match_stream.wait_stream(torch.cuda.current_stream(self.dev))  # features gathered
            issue_match(0)
        for c, (a, b) in enumerate(self.pchunks):
            pairs = self.pairs_dev[a:b]
            if overlap:
                cs = torch.cuda.current_stream(self.dev)
                cs.wait_event(self.match_done[c])
                if c + 1 < len(self.pchunks):
                    issue_match(c + 1)
                idx, mcnt = matched.pop(c)
                idx.record_stream(cs)  # allocated on the match stream, read here
                mcnt.record_stream(cs)
            else:
                issue_match(c)
                idx, mcnt = matched.pop(c)
            self._mark("match")
            res = self.kern.verify(xy_all, self.intr, pairs, idx, mcnt, cfg.thresh_px, self.pair_ids[a:b])
            self._mark("verify")
            out, ratio_inl = res, None
            if cfg.bundle_adjust:
                out = self.kern.bundle_adjust(xy_all, self.intr, pairs, idx, mcnt, res, cfg.min_inliers,
                                              cfg.ba_max_iters, cfg.ba_reproj_thresh, cfg.tri_reproj_thresh)
                ratio_inl = res.n_inliers  # the post-BA report keeps the pre-BA inlier ratio
                self._mark("bundle_adjust")
            self.kern.compact(idx, mcnt, out, cfg.min_inliers, cfg.min_inlier_ratio, (b - a) * k,
                              self.d_offsets[a + c: b + c + 1], self.d_v_corr[a * k: b * k], self.d_isp_ok[a:b],
                              ratio_inliers=ratio_inl)
            self.d_fixed[a:b, :9] = out.R.reshape(-1, 9)
            self.d_fixed[a:b, 9:] = out.t
            self.d_ints[a:b, 0] = res.status
            self.d_ints[a:b, 1] = out.n_inliers
            self.d_ints[a:b, 2] = mcnt
            self._mark("compact")
            n_hyp.append(res.n_hyp)
            if res.n_models is not None:
                n_models.append(res.n_models)
            n_match.append(mcnt)
        if self.P:
            self.stats = {"n_hyp": torch.cat(n_hyp), "n_matches": torch.cat(n_match)}
            if n_models:
                self.stats["n_models"] = torch.cat(n_models)
        if resident:
            return None
        return self._to_host()

    def _to_host(self) -> HostResults:
        k = self.cfg.kpts
        P, nc = self.P, len(self.pchunks)
        nb = dict(non_blocking=self.cuda)
        self.h_fixed.copy_(self.d_fixed, **nb)
        self.h_ints.copy_(self.d_ints, **nb)
        self.h_isp_ok.copy_(self.d_isp_ok, **nb)
        self.h_offsets.copy_(self.d_offsets, **nb)
        self.h_xy.copy_(self.feats.xy, **nb)
        self.h_count.copy_(self.feats.count, **nb)
        self._mark("d2h")
        if self.cuda:
            torch.cuda.current_stream(self.dev).synchronize()
        off = self.h_offsets.numpy()
        glob = np.zeros(P + 1, dtype=np.int64)
        pos = 0
        for c, (a, b) in enumerate(self.pchunks):
            n = int(off[b + c])
            if n:
                self.h_v_corr[pos: pos + n].copy_(self.d_v_corr[a * k: a * k + n], **nb)
            glob[a: b + 1] = pos + off[a + c: b + c + 1]
            pos += n
        self._mark("d2h")
        if self.cuda:
            torch.cuda.current_stream(self.dev).synchronize()
        fixed = self.h_fixed.numpy()[:P]
        ints = self.h_ints.numpy()[:P]
        return HostResults(pairs=self.my_pairs, R=fixed[:, :9].reshape(P, 3, 3), t=fixed[:, 9:], status=ints[:, 0],
                           n_inliers=ints[:, 1], n_matches=ints[:, 2], isp_ok=self.h_isp_ok.numpy()[:P].astype(bool),
                           offsets=glob, v_corr=self.h_v_corr.numpy()[:pos].view(np.uint32),
                           kp_xy=self.h_xy.numpy(), kp_count=self.h_count.numpy())
