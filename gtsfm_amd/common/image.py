"""Image container with the fields the front-end uses (reference: gtsfm/common/image.py:19-175)."""
from typing import Any, Dict, Optional, Tuple

import numpy as np

from gtsfm_amd.common.geometry import Cal3Bundler


class Image:
    """value_array (H, W[, C]) uint8, optional EXIF dict and (H, W) mask of valid pixels."""

    def __init__(self, value_array: np.ndarray, exif_data: Optional[Dict[str, Any]] = None,
                 file_name: Optional[str] = None, mask: Optional[np.ndarray] = None):
        self._value_array = value_array
        self._exif_data = exif_data
        self._file_name = file_name
        self._mask = mask

    @property
    def value_array(self) -> np.ndarray:
        return self._value_array

    @property
    def height(self) -> int:
        return self._value_array.shape[0]

    @property
    def width(self) -> int:
        return self._value_array.shape[1]

    @property
    def channels(self) -> int:
        return 1 if self._value_array.ndim == 2 else self._value_array.shape[2]

    @property
    def shape(self) -> Tuple[int, int, int]:
        return (self.height, self.width, self.channels)

    @property
    def mask(self) -> Optional[np.ndarray]:
        return self._mask

    @property
    def exif_data(self) -> Optional[Dict[str, Any]]:
        return self._exif_data

    @property
    def file_name(self) -> Optional[str]:
        return self._file_name

    def get_intrinsics(self, default_focal_length_factor: float = 1.2) -> Cal3Bundler:
        """Default intrinsics when EXIF is absent: f = 1.2 max(W, H), principal point at the centre (image.py:150-168)."""
        f = default_focal_length_factor * max(self.width, self.height)
        return Cal3Bundler(float(f), 0.0, 0.0, float(self.width / 2), float(self.height / 2))
