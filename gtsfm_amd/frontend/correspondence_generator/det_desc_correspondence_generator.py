"""Detect/describe every image, then match every requested pair — batched on the MI355X.

Drop-in for gtsfm/frontend/correspondence_generator/det_desc_correspondence_generator.py:17-87
(DetDescCorrespondenceGenerator). Same constructor (matcher, detector_descriptor), same
`generate_correspondences(client, images, image_pairs)` signature and outputs: the keypoints of every image and a
dict (i1, i2) -> (M, 2) uint32 putative correspondences (np.array([]) for a pair without matches,
twoway_matcher.py:71-72,80-81).

The reference submits one Dask task per image and one per pair (:64-80). Here the HIP plugin combinations of the
BASELINE configs run batched on the device: images of one size go through ONE batched extraction launch sequence
(per workspace-bounded group), their features stay in HBM as one padded (n, k, D) block, and the pairs go through one
batched matcher launch per chunk of pairs:
- SIFTDetectorDescriptor + TwoWayMatcher (configs C1, C2, C4): the exact-integer fp16 MFMA distance GEMM;
- SuperPointDetectorDescriptor + TwoWayMatcher (config C3): the F16_RERANK matcher on the float descriptors;
- SuperPointDetectorDescriptor + SuperGlueMatcher (config C5): batched SuperGlue (superglue.hip).
Any other combination (e.g. cacher-wrapped plugins) runs its own per-call methods in the reference's order.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.correspondence_generator.correspondence_generator_base import CorrespondenceGeneratorBase
from gtsfm_amd.frontend.detector_descriptor.detector_descriptor_base import DetectorDescriptorBase
from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor, extract_group, sift_groups
from gtsfm_amd.frontend.matcher.matcher_base import MatcherBase
from gtsfm_amd.frontend.detector_descriptor.superpoint import SuperPointDetectorDescriptor
from gtsfm_amd.frontend.matcher.superglue_matcher import MATCH_THRESHOLD, SuperGlueMatcher
from gtsfm_amd.frontend.matcher.twoway_matcher import MatchingDistanceType, TwoWayMatcher

PAIR_CHUNK = 8192  # pairs per matcher launch: (chunk, k, 2) int32 indices = 128 MiB at k = 2048


def resolve(obj):
    """Images may arrive as Dask futures (the reference's call site) or as plain objects."""
    return obj.result() if hasattr(obj, "result") and callable(obj.result) else obj


class DeviceFeatures:
    """Features of n images resident in HBM: xy (n, k, 2) f32, desc (n, k, D) f32, count (n,) int32."""

    def __init__(self, xy: torch.Tensor, desc: torch.Tensor, count: torch.Tensor, keypoints: List[Keypoints]):
        self.xy, self.desc, self.count, self.keypoints = xy, desc, count, keypoints


def extract_sift_batched(detector: SIFTDetectorDescriptor, images: Sequence[Image]) -> DeviceFeatures:
    """gtsfm_sift_batched launch sequences per image size (workspace-bounded groups); features gathered into one
    padded block."""
    native.require_gpu()
    n, k = len(images), detector.max_keypoints
    dev = torch.device("cuda")
    xy = torch.zeros((n, k, 2), dtype=torch.float32, device=dev)
    attr = torch.zeros((n, k, 3), dtype=torch.float32, device=dev)
    desc = torch.zeros((n, k, 128), dtype=torch.float32, device=dev)
    count = torch.zeros((n,), dtype=torch.int32, device=dev)
    for idx in sift_groups(list(images), k):  # same shape, workspace-bounded; masks as detectAndCompute's
        res = extract_group(list(images), idx, k)
        sel = torch.tensor(idx, dtype=torch.long, device=dev)
        xy[sel], attr[sel], desc[sel], count[sel] = res.xy, res.attr, res.desc, res.count
    cnt = count.cpu().numpy()
    xy_h, attr_h = xy.cpu().numpy(), attr.cpu().numpy()
    kps = [Keypoints(coordinates=xy_h[i, : cnt[i]].astype(np.float64), scales=attr_h[i, : cnt[i], 0].astype(np.float64),
                     responses=attr_h[i, : cnt[i], 2].astype(np.float64)) for i in range(n)]
    return DeviceFeatures(xy, desc, count, kps)


def match_pairs_batched(feats: DeviceFeatures, image_pairs: Sequence[Tuple[int, int]], ratio, mode: int,
                        chunk: int = PAIR_CHUNK) -> Dict[Tuple[int, int], np.ndarray]:
    """All pairs through gtsfm_match_batched, `chunk` pairs per launch; host dict in the reference's format."""
    out: Dict[Tuple[int, int], np.ndarray] = {}
    pairs = np.asarray(image_pairs, dtype=np.int64).reshape(-1, 2)
    dev = feats.desc.device
    G = device.match_group_size(feats.desc.shape[1], feats.desc.shape[2]) if mode == native.GTSFM_MATCH_INT_F16 else 0
    for s in range(0, len(pairs), chunk):
        blk = pairs[s: s + chunk]
        groups = torch.from_numpy(device.pair_groups(blk, G)).to(dev) if G > 1 else None
        idx, cnt = device.match_pairs(feats.desc, feats.count, torch.from_numpy(blk.astype(np.int32)).to(dev),
                                      ratio, mode, groups=groups)
        cnt_h = cnt.cpu().numpy()
        width = int(cnt_h.max()) if len(cnt_h) else 0
        idx_h = idx[:, :width].cpu().numpy().view(np.uint32)
        for j, (i1, i2) in enumerate(blk):
            m = int(cnt_h[j])
            out[(int(i1), int(i2))] = idx_h[j, :m].copy() if m else np.array([])
    return out


SP_GROUP_BYTES = 16 << 30  # SuperPoint workspace per launch (~0.75 GB per 1080p image)


def extract_superpoint_batched(detector: SuperPointDetectorDescriptor, images: Sequence[Image]) -> DeviceFeatures:
    """gtsfm_superpoint_batched per image size in workspace-bounded groups; features gathered into one padded block
    (scores kept for SuperGlue). Image masks filter the detections on the device before the top-k, as the per-call
    plugin (reference superpoint.py:68-72)."""
    native.require_gpu()
    n, k = len(images), detector.max_keypoints
    dev = torch.device("cuda")
    xy = torch.zeros((n, k, 2), dtype=torch.float32, device=dev)
    sc = torch.zeros((n, k), dtype=torch.float32, device=dev)
    desc = torch.zeros((n, k, 256), dtype=torch.float32, device=dev)
    count = torch.zeros((n,), dtype=torch.int32, device=dev)
    by_shape: Dict[tuple, List[int]] = {}
    for i, im in enumerate(images):
        by_shape.setdefault(tuple(im.value_array.shape), []).append(i)
    L = native.lib()
    for shape, idx in by_shape.items():
        per = max(1, int(L.gtsfm_superpoint_workspace_bytes(1, shape[0], shape[1], k)))
        g = max(1, SP_GROUP_BYTES // per)
        for s0 in range(0, len(idx), g):
            part = idx[s0: s0 + g]
            res = detector.extract_batch([images[i].value_array for i in part], k, masks=[images[i].mask for i in part])
            sel = torch.tensor(part, dtype=torch.long, device=dev)
            xy[sel], sc[sel], desc[sel], count[sel] = res.xy, res.scores, res.desc, res.count
    cnt = count.cpu().numpy()
    xy_h, sc_h = xy.cpu().numpy(), sc.cpu().numpy()
    kps = [Keypoints(coordinates=xy_h[i, : cnt[i]], scales=None, responses=sc_h[i, : cnt[i]]) for i in range(n)]
    out = DeviceFeatures(xy, desc, count, kps)
    out.scores = sc
    return out


def superglue_pairs_batched(matcher: SuperGlueMatcher, feats: DeviceFeatures, image_shapes: Sequence[tuple],
                            image_pairs: Sequence[Tuple[int, int]], chunk: int = 1024
                            ) -> Dict[Tuple[int, int], np.ndarray]:
    """All pairs through gtsfm_superglue_batched on the resident features, `chunk` pairs per launch sequence (the
    workspace is ~59 MB per pair at 2048 keypoints); host dict in SuperGlueMatcher.match's format."""
    out: Dict[Tuple[int, int], np.ndarray] = {}
    pairs = np.asarray(image_pairs, dtype=np.int64).reshape(-1, 2)
    dev = feats.desc.device
    kmax = feats.desc.shape[1]
    kpad = (kmax + 63) // 64 * 64
    xy, sc, desc = feats.xy, feats.scores, feats.desc
    if kpad != kmax:
        pad = kpad - kmax
        xy = torch.nn.functional.pad(xy, (0, 0, 0, pad))
        sc = torch.nn.functional.pad(sc, (0, pad))
        desc = torch.nn.functional.pad(desc, (0, 0, 0, pad))
    hw = torch.tensor([[int(s[0]), int(s[1])] for s in image_shapes], dtype=torch.int32, device=dev)
    cnt_h = feats.count.cpu().numpy()
    ws = None
    for s in range(0, len(pairs), chunk):
        blk = pairs[s: s + chunk]
        run = blk[(cnt_h[blk[:, 0]] > 0) & (cnt_h[blk[:, 1]] > 0)] if len(blk) else blk
        for i1, i2 in blk:
            out[(int(i1), int(i2))] = np.zeros((0, 2), np.uint32)
        if not len(run):
            continue
        need = int(native.lib().gtsfm_superglue_workspace_bytes(len(run), kpad))
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=dev)
        idx, c, _ = device.superglue_match(xy.contiguous(), sc.contiguous(), desc.contiguous(), feats.count, hw,
                                           torch.from_numpy(run.astype(np.int32)).to(dev), matcher.weights(),
                                           matcher._n_layers, matcher._config["sinkhorn_iterations"],
                                           MATCH_THRESHOLD, workspace=ws)
        c = c.cpu().numpy()
        w = int(c.max()) if len(c) else 0
        idx_h = idx[:, :w].cpu().numpy().view(np.uint32)
        for j, (i1, i2) in enumerate(run):
            out[(int(i1), int(i2))] = idx_h[j, : c[j]].copy()
    return out


class DetDescCorrespondenceGenerator(CorrespondenceGeneratorBase):
    """Traditional detect -> describe -> match, batched on the device when the plugins are the HIP ones."""

    def __init__(self, matcher: MatcherBase, detector_descriptor: DetectorDescriptorBase) -> None:
        self._detector_descriptor = detector_descriptor
        self._matcher = matcher
        self.device_features: DeviceFeatures | None = None  # last batched extraction (kept for reuse)

    def __repr__(self) -> str:
        return f"DetDescCorrespondenceGenerator:\n   {self._detector_descriptor}\n   {self._matcher}\n"

    def _batched(self) -> Optional[str]:
        """Which batched device path serves this plugin pair: 'sift', 'superpoint_twoway', 'superpoint_superglue',
        or None (per-call)."""
        d, m = self._detector_descriptor, self._matcher
        twoway_l2 = type(m) is TwoWayMatcher and m._distance_type is MatchingDistanceType.EUCLIDEAN
        if type(d) is SIFTDetectorDescriptor and twoway_l2:
            return "sift"
        if type(d) is SuperPointDetectorDescriptor and twoway_l2:
            return "superpoint_twoway"
        if type(d) is SuperPointDetectorDescriptor and type(m) is SuperGlueMatcher:
            return "superpoint_superglue"
        return None

    def generate_correspondences(
        self, client, images: List, image_pairs: List[Tuple[int, int]]
    ) -> Tuple[List[Keypoints], Dict[Tuple[int, int], np.ndarray]]:
        imgs = [resolve(im) for im in images]
        path = self._batched()
        if path == "sift":
            feats = extract_sift_batched(self._detector_descriptor, imgs)
            self.device_features = feats
            # SIFT descriptors are integers in [0, 255] with |d|^2 < 2^19: the exact fp16 MFMA path applies
            corr = match_pairs_batched(feats, image_pairs, self._matcher._ratio_test_threshold,
                                       native.GTSFM_MATCH_INT_F16)
            return feats.keypoints, corr
        if path is not None:
            feats = extract_superpoint_batched(self._detector_descriptor, imgs)
            self.device_features = feats
            if path == "superpoint_twoway":
                # 256-D float descriptors: fp16 MFMA shortlist + certified exact re-rank (same matches as EXACT_F32)
                corr = match_pairs_batched(feats, image_pairs, self._matcher._ratio_test_threshold,
                                           native.GTSFM_MATCH_F16_RERANK)
            else:
                corr = superglue_pairs_batched(self._matcher, feats, [im.value_array.shape for im in imgs],
                                               image_pairs)
            return feats.keypoints, corr
        features = [self._detector_descriptor.detect_and_describe(im) for im in imgs]
        corr = {}
        for (i1, i2) in image_pairs:
            corr[(i1, i2)] = self._matcher.match(features[i1][0], features[i2][0], features[i1][1],
                                                 features[i2][1], imgs[i1].shape, imgs[i2].shape)
        return [f[0] for f in features], corr
