"""Two-view estimator cache (reference gtsfm/two_view_estimator_cacher.py:36-114).

`cache/two_view_estimator/{sha1}.pbz2` holding the TWO_VIEW_OUTPUT 6-tuple. The key hashes the coordinates of the first
10 putative correspondences in both images (:51-64), as in the reference. The payload's rotation / direction objects
are this package's `Rot3` / `Unit3` (gtsam's when gtsam is importable), so entries written without gtsam are not
readable by the reference and entries holding gtsam objects are refused here unless gtsam is the active backend.
"""
from pathlib import Path
from typing import Any, List, Optional

import numpy as np

import gtsfm_amd.utils.cache as cache_utils
import gtsfm_amd.utils.io as io_utils
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.two_view_estimator import TWO_VIEW_OUTPUT, TwoViewEstimator

NUM_KEYPOINTS_TO_SAMPLE_FOR_HASH = 10
NUM_CORRESPONDENCES_TO_SAMPLE_FOR_HASH = 10
CACHE_ROOT_PATH = Path(__file__).resolve().parent.parent / "cache"


def two_view_cache_key(keypoints_i1: Keypoints, keypoints_i2: Keypoints, putative_corr_idxs: np.ndarray) -> str:
    """sha1 of the sampled correspondences' coordinates (two_view_estimator_cacher.py:51-64)."""
    # reshape: an empty (0,) match array keys like an empty (0, 2) one (the reference would raise on it)
    sampled = np.asarray(putative_corr_idxs).reshape(-1, 2)[:NUM_CORRESPONDENCES_TO_SAMPLE_FOR_HASH].astype(np.int64)
    arrays: List[np.ndarray] = [keypoints_i1.coordinates[sampled[:, 0]].flatten(),
                                keypoints_i2.coordinates[sampled[:, 1]].flatten()]
    return cache_utils.generate_hash_for_numpy_array(np.concatenate(arrays))


class TwoViewEstimatorCacher(TwoViewEstimator):
    """Wraps a TwoViewEstimator; `run_2view` results are keyed on the putative correspondences."""

    def __init__(self, two_view_estimator_obj: TwoViewEstimator, cache_root: Optional[Path] = None) -> None:
        self._two_view_estimator = two_view_estimator_obj
        self._cache_root = Path(cache_root) if cache_root is not None else CACHE_ROOT_PATH

    def __repr__(self) -> str:
        return self._two_view_estimator.__repr__()

    def __getattr__(self, name: str) -> Any:
        # the batched driver reads the wrapped estimator's verifier / processor
        if name.startswith("__") or name in ("_two_view_estimator", "_cache_root"):
            raise AttributeError(name)
        return getattr(self._two_view_estimator, name)

    def _cache_path(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, putative_corr_idxs: np.ndarray) -> Path:
        key = two_view_cache_key(keypoints_i1, keypoints_i2, putative_corr_idxs)
        return self._cache_root / "two_view_estimator" / f"{key}.pbz2"

    def cache_lookup(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints,
                     putative_corr_idxs: np.ndarray) -> Optional[TWO_VIEW_OUTPUT]:
        return io_utils.read_from_bz2_file(self._cache_path(keypoints_i1, keypoints_i2, putative_corr_idxs))

    def cache_store(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, putative_corr_idxs: np.ndarray,
                    result: TWO_VIEW_OUTPUT) -> None:
        io_utils.write_to_bz2_file(result, self._cache_path(keypoints_i1, keypoints_i2, putative_corr_idxs))

    def run_2view(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, putative_corr_idxs: np.ndarray,
                  camera_intrinsics_i1, camera_intrinsics_i2, i2Ti1_prior=None, gt_camera_i1=None,
                  gt_camera_i2=None, gt_scene_mesh=None) -> TWO_VIEW_OUTPUT:
        """Cached `run_2view` of the wrapped estimator (:86-114)."""
        result = self.cache_lookup(keypoints_i1, keypoints_i2, putative_corr_idxs)
        if result is not None:
            return result
        result = self._two_view_estimator.run_2view(keypoints_i1, keypoints_i2, putative_corr_idxs,
                                                    camera_intrinsics_i1, camera_intrinsics_i2, i2Ti1_prior,
                                                    gt_camera_i1, gt_camera_i2, gt_scene_mesh)
        self.cache_store(keypoints_i1, keypoints_i2, putative_corr_idxs, result)
        return result
