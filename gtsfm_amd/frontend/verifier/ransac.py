"""RANSAC essential-matrix verifier on the MI355X.

Drop-in for gtsfm/frontend/verifier/ransac.py:50-111 (Ransac) with the verify() flow of
gtsfm/frontend/verifier/opencv_verifier_base.py:45-109: fewer than 5 (E) / 6 putatives -> failure tuple; putatives
normalised with K; threshold estimation_threshold_px / max(fx1, fx2); inlier mask; inlier ratio = mean(mask);
relative pose from the essential matrix and the verified correspondences (utils/verification.py:52-94).

The estimation runs in libgtsfm_hip.so: gtsfm_ransac_E_batched (5-point RANSAC with deterministic sampling,
iterative local optimisation and the recoverPose cheirality vote, one wavefront per pair) when
use_intrinsics_in_verification=True, gtsfm_ransac_F_batched (7-point RANSAC / LMedS on pixel coordinates, 8-point
refit, E = K2^T F K1, recoverPose; ransac.py:84-111, utils/verification.py:97-110) otherwise.
"""
from enum import Enum, unique
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common import geometry
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.verifier.verifier_base import VerifierBase

RANSAC_SUCCESS_PROB = 0.999999
RANSAC_MAX_ITERS = 1000  # cv2.findEssentialMat default maxIters
RANSAC_MAX_ITERS_F = 1000000  # ransac.py:23, passed to cv2.findFundamentalMat


@unique
class RobustEstimationType(str, Enum):
    """ransac.py:28-48 (cv2 method names). Ransac.estimate_E's default is USAC_ACCURATE (:58)."""

    FM_7POINT: str = "FM_7POINT"
    FM_8POINT: str = "FM_8POINT"
    FM_RANSAC: str = "FM_RANSAC"
    RANSAC: str = "RANSAC"
    LMEDS: str = "LMEDS"
    RHO: str = "RHO"
    USAC_DEFAULT: str = "USAC_DEFAULT"
    USAC_PARALLEL: str = "USAC_PARALLEL"
    USAC_FM_8PTS: str = "USAC_FM_8PTS"
    USAC_FAST: str = "USAC_FAST"
    USAC_ACCURATE: str = "USAC_ACCURATE"
    USAC_PROSAC: str = "USAC_PROSAC"
    USAC_MAGSAC: str = "USAC_MAGSAC"


# E-path model selection per method: the USAC family scores models by MSAC (truncated quadratic); cv2 RANSAC by
# inlier count. LMEDS / RHO / MAGSAC++ / PROSAC sampling are not implemented on the E path.
_E_SCORING = {
    RobustEstimationType.RANSAC: native.GTSFM_RANSAC_SCORING_RANSAC,
    RobustEstimationType.USAC_DEFAULT: native.GTSFM_RANSAC_SCORING_MSAC,
    RobustEstimationType.USAC_PARALLEL: native.GTSFM_RANSAC_SCORING_MSAC,
    RobustEstimationType.USAC_FAST: native.GTSFM_RANSAC_SCORING_MSAC,
    RobustEstimationType.USAC_ACCURATE: native.GTSFM_RANSAC_SCORING_MSAC,
}


def _checked_indices(match_indices: np.ndarray, n1: int, n2: int) -> np.ndarray:
    """(M, 2) int64 keypoint indices, as numpy's fancy indexing in the reference would take them
    (opencv_verifier_base.py:73-74, uv_norm[match_indices[:, k]]): negative indices wrap once, anything outside
    [-n, n) raises IndexError before a device kernel could read out of bounds."""
    m = np.ascontiguousarray(np.asarray(match_indices).reshape(-1, 2), dtype=np.int64)
    for col, n in ((0, n1), (1, n2)):
        c = m[:, col]
        if len(c) and (c.min() < -n or c.max() >= n):
            raise IndexError(f"match index out of bounds for {n} keypoints (column {col})")
        m[:, col] = np.where(c < 0, c + n, c)
    return m


def _calibration(cal) -> np.ndarray:
    if cal is None:  # the reference fails on None intrinsics too (normalize_coordinates calls cal.calibrate)
        raise ValueError("camera intrinsics are required by the verifier")
    return geometry.calibration_params(cal)


class Ransac(VerifierBase):
    """RANSAC verifier computed by HIP kernels: 5-point E path with intrinsics, 7-point F path without."""

    def __init__(self, use_intrinsics_in_verification: bool, estimation_threshold_px: float,
                 seed: int = native.RANSAC_DEFAULT_SEED,
                 robust_estimation_type: RobustEstimationType = RobustEstimationType.USAC_ACCURATE) -> None:
        """robust_estimation_type: the E path's method, estimate_E's argument in the reference (ransac.py:58; verify()
        always passes the default USAC_ACCURATE). RANSAC selects by inlier count, the USAC family by MSAC score."""
        super().__init__(use_intrinsics_in_verification, estimation_threshold_px)
        self._seed = seed
        rt = RobustEstimationType(robust_estimation_type)
        if rt not in _E_SCORING:
            raise ValueError(f"robust_estimation_type {rt.value} is not supported on the essential-matrix path")
        self._scoring = _E_SCORING[rt]

    def verify(
        self,
        keypoints_i1: Keypoints,
        keypoints_i2: Keypoints,
        match_indices: np.ndarray,
        camera_intrinsics_i1,
        camera_intrinsics_i2,
    ) -> Tuple[Optional[object], Optional[object], np.ndarray, float]:
        if match_indices.shape[0] < self._min_matches or match_indices.shape[0] < 6:
            return self._failure_result
        checked = _checked_indices(match_indices, len(keypoints_i1), len(keypoints_i2))
        intr = np.stack([_calibration(camera_intrinsics_i1), _calibration(camera_intrinsics_i2)])
        native.require_gpu()
        M = match_indices.shape[0]
        if not self._use_intrinsics_in_verification:
            return self.verify_batch([keypoints_i1, keypoints_i2], {(0, 1): match_indices},
                                     [camera_intrinsics_i1, camera_intrinsics_i2])[(0, 1)]
        dev = torch.device("cuda")
        c1 = keypoints_i1.coordinates.astype(np.float32)
        c2 = keypoints_i2.coordinates.astype(np.float32)
        kmax = max(len(c1), len(c2))
        kp = np.zeros((2, kmax, 2), np.float32)
        kp[0, : len(c1)] = c1
        kp[1, : len(c2)] = c2
        mi = checked.astype(np.int32).reshape(1, M, 2)
        res = device.ransac_essential(
            torch.from_numpy(kp).to(dev), torch.from_numpy(intr).to(dev),
            torch.tensor([[0, 1]], dtype=torch.int32, device=dev), torch.from_numpy(mi).to(dev),
            torch.tensor([M], dtype=torch.int32, device=dev), self._estimation_threshold_px,
            RANSAC_SUCCESS_PROB, RANSAC_MAX_ITERS, self._seed, scoring=self._scoring)
        status = int(res.status[0].item())
        if status != native.RANSAC_STATUS_OK:
            return self._failure_result
        mask = res.mask[0, :M].cpu().numpy().astype(bool)
        v_corr_idxs = match_indices[np.flatnonzero(mask)]
        inlier_ratio = float(np.mean(mask))
        R = res.R[0].cpu().numpy()
        t = res.t[0].cpu().numpy()
        return geometry.Rot3(R), geometry.Unit3(t), v_corr_idxs, inlier_ratio

    def verify_batch(
        self,
        keypoints_list: Sequence[Keypoints],
        putative_corr_idxs_dict: Dict[Tuple[int, int], np.ndarray],
        camera_intrinsics: Sequence,
        chunk: int = 8192,
    ) -> Dict[Tuple[int, int], Tuple[Optional[object], Optional[object], np.ndarray, float]]:
        """verify() of every pair of the dict through ONE gtsfm_ransac_E_batched launch sequence per chunk.

        Same guards and failure tuple as verify(), and the same sampler stream: every pair is keyed by pair id 0,
        as a one-pair verify() call is, so the batch reproduces verify() pair for pair.
        """
        native.require_gpu()
        dev = torch.device("cuda")
        n = len(keypoints_list)
        kmax = max([len(k) for k in keypoints_list] + [1])
        kp = np.zeros((n, kmax, 2), np.float32)
        for i, k in enumerate(keypoints_list):
            kp[i, : len(k)] = k.coordinates
        kp_d = torch.from_numpy(kp).to(dev)
        used = {i for p in putative_corr_idxs_dict for i in p}
        intr = np.stack([_calibration(c) if i in used else np.zeros(3) for i, c in enumerate(camera_intrinsics)])
        intr_d = torch.from_numpy(intr).to(dev)
        keys = list(putative_corr_idxs_dict.keys())
        out: Dict[Tuple[int, int], Tuple[Optional[object], Optional[object], np.ndarray, float]] = {}
        for s in range(0, len(keys), chunk):
            blk = keys[s: s + chunk]
            run = [p for p in blk if len(putative_corr_idxs_dict[p]) >= max(self._min_matches, 6)]
            for p in blk:
                out[p] = self._failure_result
            if not run:
                continue
            mcap = max(len(putative_corr_idxs_dict[p]) for p in run)
            mi = np.zeros((len(run), mcap, 2), np.int32)
            cnt = np.zeros(len(run), np.int32)
            for j, p in enumerate(run):
                m = _checked_indices(putative_corr_idxs_dict[p], len(keypoints_list[p[0]]), len(keypoints_list[p[1]]))
                mi[j, : len(m)] = m.astype(np.int32)
                cnt[j] = len(m)
            args = (kp_d, intr_d, torch.tensor(run, dtype=torch.int32, device=dev), torch.from_numpy(mi).to(dev),
                    torch.from_numpy(cnt).to(dev), self._estimation_threshold_px, RANSAC_SUCCESS_PROB)
            ids = torch.zeros(len(run), dtype=torch.int32, device=dev)
            if self._use_intrinsics_in_verification:
                res = device.ransac_essential(*args, RANSAC_MAX_ITERS, self._seed, pair_ids=ids, scoring=self._scoring)
            else:
                res = device.ransac_fundamental(*args, RANSAC_MAX_ITERS_F, self._seed, pair_ids=ids)
            status = res.status.cpu().numpy()
            mask = res.mask.cpu().numpy().astype(bool)
            R, t = res.R.cpu().numpy(), res.t.cpu().numpy()
            for j, p in enumerate(run):
                if status[j] != native.RANSAC_STATUS_OK:
                    continue
                m = np.asarray(putative_corr_idxs_dict[p]).reshape(-1, 2)
                mk = mask[j, : len(m)]
                out[p] = (geometry.Rot3(R[j]), geometry.Unit3(t[j]), m[np.flatnonzero(mk)], float(np.mean(mk)))
        return out
