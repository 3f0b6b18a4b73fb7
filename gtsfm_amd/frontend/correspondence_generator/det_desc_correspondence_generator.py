"""Detect/describe every image, then match every requested pair — batched on the MI355X.

Drop-in for gtsfm/frontend/correspondence_generator/det_desc_correspondence_generator.py:17-87
(DetDescCorrespondenceGenerator). Same constructor (matcher, detector_descriptor), same
`generate_correspondences(client, images, image_pairs)` signature and outputs: the keypoints of every image and a
dict (i1, i2) -> (M, 2) uint32 putative correspondences (np.array([]) for a pair without matches,
twoway_matcher.py:71-72,80-81).

The reference submits one Dask task per image and one per pair (:64-80). Here, when the plugins are the HIP SIFT
and the HIP TwoWayMatcher, images of one size go through ONE batched SIFT launch sequence, their features stay in
HBM as one padded (n, k, 128) block, and all pairs go through ONE batched matcher launch per chunk of pairs. Other
plugin combinations run their own per-call methods in the reference's order.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.correspondence_generator.correspondence_generator_base import CorrespondenceGeneratorBase
from gtsfm_amd.frontend.detector_descriptor.detector_descriptor_base import DetectorDescriptorBase
from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor, extract_group, sift_groups
from gtsfm_amd.frontend.matcher.matcher_base import MatcherBase
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


class DetDescCorrespondenceGenerator(CorrespondenceGeneratorBase):
    """Traditional detect -> describe -> match, batched on the device when the plugins are the HIP ones."""

    def __init__(self, matcher: MatcherBase, detector_descriptor: DetectorDescriptorBase) -> None:
        self._detector_descriptor = detector_descriptor
        self._matcher = matcher
        self.device_features: DeviceFeatures | None = None  # last batched extraction (kept for reuse)

    def __repr__(self) -> str:
        return f"DetDescCorrespondenceGenerator:\n   {self._detector_descriptor}\n   {self._matcher}\n"

    def _batched(self) -> bool:
        m = self._matcher
        return (isinstance(self._detector_descriptor, SIFTDetectorDescriptor) and isinstance(m, TwoWayMatcher)
                and m._distance_type is MatchingDistanceType.EUCLIDEAN)

    def generate_correspondences(
        self, client, images: List, image_pairs: List[Tuple[int, int]]
    ) -> Tuple[List[Keypoints], Dict[Tuple[int, int], np.ndarray]]:
        imgs = [resolve(im) for im in images]
        if self._batched():
            feats = extract_sift_batched(self._detector_descriptor, imgs)
            self.device_features = feats
            # SIFT descriptors are integers in [0, 255] with |d|^2 < 2^19: the exact fp16 MFMA path applies
            corr = match_pairs_batched(feats, image_pairs, self._matcher._ratio_test_threshold,
                                       native.GTSFM_MATCH_INT_F16)
            return feats.keypoints, corr
        features = [self._detector_descriptor.detect_and_describe(im) for im in imgs]
        corr = {}
        for (i1, i2) in image_pairs:
            corr[(i1, i2)] = self._matcher.match(features[i1][0], features[i2][0], features[i1][1],
                                                 features[i2][1], imgs[i1].shape, imgs[i2].shape)
        return [f[0] for f in features], corr
