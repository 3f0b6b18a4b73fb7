"""Base class of the global image descriptors (mirrors gtsfm/frontend/global_descriptor/global_descriptor_base.py:13-28)."""
import abc
from typing import List

import numpy as np

from gtsfm_amd.common.image import Image


class GlobalDescriptorBase:
    """Assigns one vector to each input image."""

    @abc.abstractmethod
    def describe(self, image: Image) -> np.ndarray:
        """(D,) global descriptor of one image (global_descriptor_base.py:19-28)."""

    def describe_batch(self, images: List[Image]) -> List[np.ndarray]:
        """One descriptor per image; device implementations batch this (no reference counterpart)."""
        return [self.describe(im) for im in images]
