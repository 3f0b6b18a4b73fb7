"""Detector-descriptor plugin interface (reference: gtsfm/frontend/detector_descriptor/detector_descriptor_base.py)."""
import abc
from typing import Tuple

import numpy as np

from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints


class DetectorDescriptorBase(metaclass=abc.ABCMeta):
    """Joint keypoint detector + descriptor working on one image."""

    def __init__(self, max_keypoints: int = 5000):
        self.max_keypoints = max_keypoints

    @abc.abstractmethod
    def detect_and_describe(self, image: Image) -> Tuple[Keypoints, np.ndarray]:
        """Returns keypoints (N <= max_keypoints) and their (N, D) descriptors."""
