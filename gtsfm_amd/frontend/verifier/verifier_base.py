"""Verifier plugin interface (reference: gtsfm/frontend/verifier/verifier_base.py:17-82)."""
import abc
from typing import Optional, Tuple

import numpy as np

from gtsfm_amd.common.keypoints import Keypoints

NUM_MATCHES_REQ_E_MATRIX = 5
NUM_MATCHES_REQ_F_MATRIX = 8


class VerifierBase(metaclass=abc.ABCMeta):
    """Estimates the relative pose of an image pair and the geometrically verified correspondences."""

    def __init__(self, use_intrinsics_in_verification: bool, estimation_threshold_px: float) -> None:
        self._use_intrinsics_in_verification = use_intrinsics_in_verification
        self._estimation_threshold_px = estimation_threshold_px
        self._min_matches = (
            NUM_MATCHES_REQ_E_MATRIX if self._use_intrinsics_in_verification else NUM_MATCHES_REQ_F_MATRIX
        )
        # i2Ri1=None, i2Ui1=None, no verified correspondences, inlier_ratio_est_model=0.0 (verifier_base.py:56)
        self._failure_result = (None, None, np.array([], dtype=np.uint64), 0.0)

    @abc.abstractmethod
    def verify(
        self,
        keypoints_i1: Keypoints,
        keypoints_i2: Keypoints,
        match_indices: np.ndarray,
        camera_intrinsics_i1,
        camera_intrinsics_i2,
    ) -> Tuple[Optional[object], Optional[object], np.ndarray, float]:
        """Returns (i2Ri1 or None, i2Ui1 or None, verified (K,2) indices, inlier ratio w.r.t. the model)."""
