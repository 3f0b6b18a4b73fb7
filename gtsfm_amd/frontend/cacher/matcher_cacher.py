"""Matcher cache (reference gtsfm/frontend/cacher/matcher_cacher.py:26-192).

`cache/matcher/{MatcherClassName}_{sha1}.pbz2` holding the (M, 2) match indices. The key hashes, per image, the first
10 keypoint coordinates, responses and scales (when present) and descriptors, then both image shapes (:51-80), so a
key computed here equals the reference's for the same inputs.
"""
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

import gtsfm_amd.utils.cache as cache_utils
import gtsfm_amd.utils.io as io_utils
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.matcher.matcher_base import MatcherBase

CACHE_ROOT_PATH = Path(__file__).resolve().parent.parent.parent.parent / "cache"
NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH = 10


def matcher_cache_key(matcher_name: str, keypoints_i1: Keypoints, keypoints_i2: Keypoints,
                      descriptors_i1: np.ndarray, descriptors_i2: np.ndarray,
                      im_shape_i1: Tuple[int, int, int], im_shape_i2: Tuple[int, int, int]) -> str:
    """`{matcher_name}_{sha1}` exactly as matcher_cacher.py:51-80 (np.concatenate promotes to the widest dtype)."""
    arrays: List[np.ndarray] = []
    for kp, desc in ((keypoints_i1, descriptors_i1), (keypoints_i2, descriptors_i2)):
        arrays.append(kp.coordinates[:NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH].flatten())
        if kp.responses is not None:
            arrays.append(kp.responses[:NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH].flatten())
        if kp.scales is not None:
            arrays.append(kp.scales[:NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH].flatten())
        arrays.append(desc[:NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH].flatten())
    h1, w1, c1 = im_shape_i1
    h2, w2, c2 = im_shape_i2
    arrays.append(np.array([h1, w1, c1, h2, w2, c2]))
    return "{}_{}".format(matcher_name, cache_utils.generate_hash_for_numpy_array(np.concatenate(arrays)))


class MatcherCacher(MatcherBase):
    """Wraps a matcher; results are keyed on a sample of its inputs."""

    def __init__(self, matcher_obj: MatcherBase, cache_root: Optional[Path] = None) -> None:
        super().__init__()
        self._matcher = matcher_obj
        self._matcher_obj_key = type(self._matcher).__name__
        self._cache_root = Path(cache_root) if cache_root is not None else CACHE_ROOT_PATH

    def __repr__(self) -> str:
        return f"MatcherCacher({self._matcher!r})"

    @property
    def wrapped(self) -> MatcherBase:
        """The matcher whose results are cached (the batched generator runs its misses on the device)."""
        return self._matcher

    def cache_path(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, descriptors_i1: np.ndarray,
                   descriptors_i2: np.ndarray, im_shape_i1: Tuple[int, int, int],
                   im_shape_i2: Tuple[int, int, int]) -> Path:
        """`cache/matcher/{key}.pbz2` (:82-84). Only the first 10 descriptor rows of each image enter the key."""
        key = matcher_cache_key(self._matcher_obj_key, keypoints_i1, keypoints_i2, descriptors_i1, descriptors_i2,
                                im_shape_i1, im_shape_i2)
        return self._cache_root / "matcher" / f"{key}.pbz2"

    def match(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, descriptors_i1: np.ndarray,
              descriptors_i2: np.ndarray, im_shape_i1: Tuple[int, int, int],
              im_shape_i2: Tuple[int, int, int]) -> np.ndarray:
        """Cached `match` of the wrapped object (:126-192)."""
        path = self.cache_path(keypoints_i1, keypoints_i2, descriptors_i1, descriptors_i2, im_shape_i1, im_shape_i2)
        cached = io_utils.read_from_bz2_file(path)
        if cached is not None:
            return cached
        match_indices = self._matcher.match(keypoints_i1, keypoints_i2, descriptors_i1, descriptors_i2,
                                            im_shape_i1, im_shape_i2)
        io_utils.write_to_bz2_file(match_indices, path)
        return match_indices
