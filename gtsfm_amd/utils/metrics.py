"""Ground-truth correspondence metrics of the two-view report (reference gtsfm/utils/metrics.py:38-128 and
gtsfm/utils/verification.py:113-214).

For pinhole ground-truth cameras, every verified correspondence is classified by its squared Sampson distance to
the GT epipolar geometry: i2Ti1 = wTi2^-1 wTi1, E = [t/|t|]x R (gtsam EssentialMatrix(R, Unit3(t))),
F = K2^-T E K1^-1, d^2 = (x2^T F x1)^2 / (|(F x1)_xy|^2 + |(F^T x2)_xy|^2), inlier iff d^2 < threshold^2. The
returned "reprojection error" is that squared distance, as in the reference (metrics.py:121-127). Host-side numpy:
this runs only when GT cameras are supplied (evaluation), never on the benchmark path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from gtsfm_amd.common import geometry
from gtsfm_amd.common.keypoints import Keypoints


def _homogeneous(x: np.ndarray) -> np.ndarray:
    return np.hstack((x, np.ones((x.shape[0], 1))))


def compute_epipolar_distances_sq_sampson(coordinates_i1: np.ndarray, coordinates_i2: np.ndarray,
                                          i2Fi1: np.ndarray) -> Optional[np.ndarray]:
    """verification.py:170-214."""
    if coordinates_i1 is None or coordinates_i1.size == 0 or coordinates_i2 is None or coordinates_i2.size == 0:
        return None
    lines_i2 = _homogeneous(coordinates_i1) @ i2Fi1.T  # F x1
    lines_i1 = _homogeneous(coordinates_i2) @ i2Fi1  # F^T x2
    sq_i1 = np.sum(np.square(lines_i1[:, :2]), axis=1)
    sq_i2 = np.sum(np.square(lines_i2[:, :2]), axis=1)
    numerator = np.square(np.sum(_homogeneous(coordinates_i1) * lines_i1, axis=1))
    return numerator / (sq_i1 + sq_i2)


def essential_to_fundamental_matrix(i2Ei1: np.ndarray, K1: np.ndarray, K2: np.ndarray) -> np.ndarray:
    """verification.py:113-126."""
    return np.linalg.inv(K2.T) @ i2Ei1 @ np.linalg.inv(K1)


def epipolar_inlier_correspondences(keypoints_i1: Keypoints, keypoints_i2: Keypoints, K1: np.ndarray,
                                    K2: np.ndarray, i2Ri1: np.ndarray, i2ti1: np.ndarray,
                                    dist_threshold: float) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
    """metrics.py:99-128."""
    u = i2ti1 / np.linalg.norm(i2ti1)
    E = geometry.skew(u) @ i2Ri1
    F = essential_to_fundamental_matrix(E, K1, K2)
    d2 = compute_epipolar_distances_sq_sampson(keypoints_i1.coordinates, keypoints_i2.coordinates, F)
    return (d2 < dist_threshold ** 2 if d2 is not None else None), d2


def compute_correspondence_metrics(keypoints_i1: Keypoints, keypoints_i2: Keypoints, corr_idxs_i1i2: np.ndarray,
                                   dist_threshold: float, gt_camera_i1=None, gt_camera_i2=None,
                                   gt_scene_mesh=None) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
    """metrics.py:38-96: (inlier mask, squared Sampson distance) of the verified correspondences w.r.t. GT cameras."""
    corr = np.asarray(corr_idxs_i1i2)
    if corr.size == 0:
        return None, None
    if gt_camera_i1 is None or gt_camera_i2 is None:
        return None, None
    if gt_scene_mesh is not None:
        raise NotImplementedError("mesh-based GT correspondence metrics need trimesh ray casting, not in this image")
    corr = corr.reshape(-1, 2).astype(np.int64)
    kp1 = keypoints_i1.extract_indices(corr[:, 0])
    kp2 = keypoints_i2.extract_indices(corr[:, 1])
    (R1, t1), (R2, t2) = geometry.camera_pose(gt_camera_i1), geometry.camera_pose(gt_camera_i2)
    i2Ri1 = R2.T @ R1  # wTi2.between(wTi1)
    i2ti1 = R2.T @ (t1 - t2)
    return epipolar_inlier_correspondences(kp1, kp2, geometry.calibration_matrix(gt_camera_i1),
                                           geometry.calibration_matrix(gt_camera_i2), i2Ri1, i2ti1, dist_threshold)
