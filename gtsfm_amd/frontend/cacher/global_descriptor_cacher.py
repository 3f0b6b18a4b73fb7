"""Global descriptor cache (reference gtsfm/frontend/cacher/global_descriptor_cacher.py:28-97).

`cache/global_descriptor/{DescriptorClassName}_{image hash}.pbz2` holding `{"global_descriptor": (D,) array}`: the
reference's key, path and payload.
"""
from pathlib import Path
from typing import Optional

import numpy as np

import gtsfm_amd.utils.cache as cache_utils
import gtsfm_amd.utils.io as io_utils
from gtsfm_amd.common.image import Image
from gtsfm_amd.frontend.global_descriptor.global_descriptor_base import GlobalDescriptorBase

CACHE_ROOT_PATH = Path(__file__).resolve().parent.parent.parent.parent / "cache"


class GlobalDescriptorCacher(GlobalDescriptorBase):
    """Wraps a global descriptor; results are keyed on the input image."""

    def __init__(self, global_descriptor_obj: GlobalDescriptorBase, cache_root: Optional[Path] = None) -> None:
        self._global_descriptor = global_descriptor_obj
        self._global_descriptor_obj_cache_key = type(self._global_descriptor).__name__
        self._cache_root = Path(cache_root) if cache_root is not None else CACHE_ROOT_PATH

    def __repr__(self) -> str:
        return f"GlobalDescriptorCacher({self._global_descriptor!r})"

    @property
    def wrapped(self) -> GlobalDescriptorBase:
        return self._global_descriptor

    def cache_path(self, image: Image) -> Path:
        key = "{}_{}".format(self._global_descriptor_obj_cache_key, cache_utils.generate_hash_for_image(image))
        return self._cache_root / "global_descriptor" / f"{key}.pbz2"

    def cache_lookup(self, image: Image) -> Optional[np.ndarray]:
        cached = io_utils.read_from_bz2_file(self.cache_path(image))
        return None if cached is None else cached["global_descriptor"]

    def cache_store(self, image: Image, global_descriptor: np.ndarray) -> None:
        io_utils.write_to_bz2_file({"global_descriptor": global_descriptor}, self.cache_path(image))

    def describe(self, image: Image) -> np.ndarray:
        """Cached `describe` of the wrapped object (:76-97)."""
        cached = self.cache_lookup(image)
        if cached is not None:
            return cached
        global_descriptor = self._global_descriptor.describe(image)
        self.cache_store(image, global_descriptor)
        return global_descriptor
