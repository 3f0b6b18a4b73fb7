"""Matcher plugin interface (reference: gtsfm/frontend/matcher/matcher_base.py:14-63)."""
import abc
from typing import Tuple

import numpy as np

from gtsfm_amd.common.keypoints import Keypoints


class MatcherBase(metaclass=abc.ABCMeta):
    """Matches the descriptors of one image pair by descriptor distance."""

    @abc.abstractmethod
    def match(
        self,
        keypoints_i1: Keypoints,
        keypoints_i2: Keypoints,
        descriptors_i1: np.ndarray,
        descriptors_i2: np.ndarray,
        im_shape_i1: Tuple[int, int, int],
        im_shape_i2: Tuple[int, int, int],
    ) -> np.ndarray:
        """Returns (N, 2) uint32 match indices (column 0: image i1, column 1: image i2), best first."""
