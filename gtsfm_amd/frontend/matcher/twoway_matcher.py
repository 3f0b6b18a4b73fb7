"""Two-way (mutual nearest neighbour) matcher with optional ratio test, on the MI355X.

Drop-in for gtsfm/frontend/matcher/twoway_matcher.py:24-144 (TwoWayMatcher). Same constructor arguments, same
`match` signature, same output (uint32 (M,2), ordered by ascending i1->i2 distance, ties by i1 index), same
empty-input behaviour (`np.array([])`) and the same NaN-row filtering and index remapping (:71-85).

The distance / top-2 / ratio / mutual / sort work runs in libgtsfm_hip.so (gtsfm_match_batched):
integer-valued descriptors (SIFT) go through the fp16 MFMA distance GEMM, anything else through the exact
fp32 kernel. Both are bit-identical to the reference semantics restated in oracle/twoway.c.
"""
from enum import Enum
from typing import Optional, Tuple

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.matcher.matcher_base import MatcherBase

_INT_MAX_VALUE = 1023.0
_INT_MAX_NORM_SQ = float(1 << 19)


class MatchingDistanceType(Enum):
    """Distance metric (reference twoway_matcher.py:17-21). Only EUCLIDEAN is on the MI355X path."""

    HAMMING = 1
    EUCLIDEAN = 2


def select_match_mode(d1: np.ndarray, d2: np.ndarray) -> int:
    """INT_F16 (exact-integer MFMA) when every descriptor is an integer in [0, 1023] with |d|^2 < 2^19; otherwise
    F16_RERANK (fp16 MFMA shortlist + certified exact re-rank) up to 256 dims, else EXACT_F32. All three give the
    same matches."""
    kmax = max(d1.shape[0], d2.shape[0])
    float_mode = native.GTSFM_MATCH_F16_RERANK if d1.shape[1] <= 256 else native.GTSFM_MATCH_EXACT_F32
    if d1.shape[1] > 139 or kmax > 8192:
        return float_mode
    for d in (d1, d2):
        if d.size == 0:
            continue
        if d.min() < 0.0 or d.max() > _INT_MAX_VALUE or not np.array_equal(d, np.round(d)):
            return float_mode
        if float(np.max(np.sum(d.astype(np.float64) ** 2, axis=1))) >= _INT_MAX_NORM_SQ:
            return float_mode
    return native.GTSFM_MATCH_INT_F16


def match_descriptor_pair(d1: np.ndarray, d2: np.ndarray, ratio: Optional[float]) -> np.ndarray:
    """Runs the device matcher on one pair of (already NaN-free) descriptor arrays."""
    native.require_gpu()
    d1 = np.ascontiguousarray(d1, dtype=np.float32)
    d2 = np.ascontiguousarray(d2, dtype=np.float32)
    n1, dim = d1.shape
    n2 = d2.shape[0]
    kmax = max(n1, n2)
    host = np.zeros((2, kmax, dim), dtype=np.float32)
    host[0, :n1] = d1
    host[1, :n2] = d2
    dev = torch.device("cuda")
    desc = torch.from_numpy(host).to(dev)
    counts = torch.tensor([n1, n2], dtype=torch.int32, device=dev)
    pairs = torch.tensor([[0, 1]], dtype=torch.int32, device=dev)
    idx, cnt = device.match_pairs(desc, counts, pairs, ratio, select_match_mode(d1, d2))
    m = int(cnt[0].item())
    return idx[0, :m].cpu().numpy().view(np.uint32).copy()


class TwoWayMatcher(MatcherBase):
    """Mutual-NN matcher with optional ratio test, computed by HIP kernels on the MI355X."""

    def __init__(
        self,
        distance_type: MatchingDistanceType = MatchingDistanceType.EUCLIDEAN,
        ratio_test_threshold: Optional[float] = None,
    ):
        super().__init__()
        self._distance_type = distance_type
        self._ratio_test_threshold: Optional[float] = ratio_test_threshold

    def match(
        self,
        keypoints_i1: Keypoints,  # pylint: disable=unused-argument
        keypoints_i2: Keypoints,  # pylint: disable=unused-argument
        descriptors_i1: np.ndarray,
        descriptors_i2: np.ndarray,
        im_shape_i1: Tuple[int, int, int],  # pylint: disable=unused-argument
        im_shape_i2: Tuple[int, int, int],  # pylint: disable=unused-argument
    ) -> np.ndarray:
        if self._distance_type is not MatchingDistanceType.EUCLIDEAN:
            raise NotImplementedError("Only Euclidean (L2) matching runs on the MI355X path")
        if descriptors_i1.size == 0 or descriptors_i2.size == 0:
            return np.array([])
        d1 = descriptors_i1.reshape(descriptors_i1.shape[0], -1)
        d2 = descriptors_i2.reshape(descriptors_i2.shape[0], -1)
        valid1 = np.nonzero(~np.isnan(d1).any(axis=1))[0]
        valid2 = np.nonzero(~np.isnan(d2).any(axis=1))[0]
        if valid1.size == 0 or valid2.size == 0:
            return np.array([])
        match_indices = match_descriptor_pair(d1[valid1], d2[valid2], self._ratio_test_threshold)
        if match_indices.size == 0:
            return np.array([])
        match_indices[:, 0] = valid1[match_indices[:, 0]]
        match_indices[:, 1] = valid2[match_indices[:, 1]]
        return match_indices
