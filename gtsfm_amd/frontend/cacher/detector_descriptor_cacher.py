"""Detector-descriptor cache (reference gtsfm/frontend/cacher/detector_descriptor_cacher.py:28-95).

`cache/detector_descriptor/{DetectorClassName}_{image hash}.pbz2` holding `{"keypoints": Keypoints,
"descriptors": (N, D) array}`: the reference's key, path and payload, so either implementation reads the other's
entries (gtsfm_amd/utils/io.py writes the Keypoints under the reference's class path).
"""
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

import gtsfm_amd.utils.cache as cache_utils
import gtsfm_amd.utils.io as io_utils
from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.detector_descriptor.detector_descriptor_base import DetectorDescriptorBase

# the reference's repo-root `cache/` folder (detector_descriptor_cacher.py:26), here relative to this package's root
CACHE_ROOT_PATH = Path(__file__).resolve().parent.parent.parent.parent / "cache"


class DetectorDescriptorCacher(DetectorDescriptorBase):
    """Wraps a detector-descriptor; results are keyed on the input image."""

    def __init__(self, detector_descriptor_obj: DetectorDescriptorBase, cache_root: Optional[Path] = None) -> None:
        super().__init__(max_keypoints=detector_descriptor_obj.max_keypoints)
        self._detector_descriptor = detector_descriptor_obj
        self._detector_descriptor_obj_cache_key = type(self._detector_descriptor).__name__
        self._cache_root = Path(cache_root) if cache_root is not None else CACHE_ROOT_PATH

    def __repr__(self) -> str:
        return f"DetectorDescriptorCacher({self._detector_descriptor!r})"

    def _cache_path(self, image: Image) -> Path:
        key = "{}_{}".format(self._detector_descriptor_obj_cache_key, cache_utils.generate_hash_for_image(image))
        return self._cache_root / "detector_descriptor" / f"{key}.pbz2"

    @property
    def wrapped(self) -> DetectorDescriptorBase:
        """The detector-descriptor whose results are cached (the batched generator runs its misses on the device)."""
        return self._detector_descriptor

    def cache_lookup(self, image: Image) -> Optional[Tuple[Keypoints, np.ndarray]]:
        """The cached (keypoints, descriptors) of `image`, or None on a miss (:58-63)."""
        cached = io_utils.read_from_bz2_file(self._cache_path(image))
        if cached is None:
            return None
        return cached["keypoints"], cached["descriptors"]

    def cache_store(self, image: Image, keypoints: Keypoints, descriptors: np.ndarray) -> None:
        """Writes the entry under the reference's key and payload (:65-69)."""
        io_utils.write_to_bz2_file({"keypoints": keypoints, "descriptors": descriptors}, self._cache_path(image))

    def detect_and_describe(self, image: Image) -> Tuple[Keypoints, np.ndarray]:
        """Cached `detect_and_describe` of the wrapped object (:71-95)."""
        cached = self.cache_lookup(image)
        if cached is not None:
            return cached
        keypoints, descriptors = self._detector_descriptor.detect_and_describe(image)
        self.cache_store(image, keypoints, descriptors)
        return keypoints, descriptors
