"""Two-view estimation of every putative pair: verify -> report -> inlier-support filter.

Drop-in for gtsfm/two_view_estimator.py: `TwoViewEstimator.run_2view` (:276-351), `generate_two_view_report`
(:354-393), `compute_relative_pose_metrics` (:396-420) and `run_two_view_estimator_as_futures` (:531-587), with
the same TWO_VIEW_OUTPUT 6-tuple (i2Ri1, i2Ui1, v_corr_idxs, pre-BA report, post-BA report, post-ISP report).

`run_two_view_estimator_as_futures` is where the batching happens: instead of one Dask task per pair, every pair
goes through ONE batched RANSAC launch sequence (Ransac.verify_batch), then -- with bundle_adjust_2view=True, as in
every shipped configuration -- ONE batched two-view triangulation + bundle adjustment launch
(gtsfm_ba2_batched: `bundle_adjust`, :136-208, on the pairs with >= min_num_inliers verified rows, :311), and only
the cheap report / ISP logic runs per pair on the host. After BA the report keeps the pre-BA inlier ratio, as the
reference does (:325-327). Relative-pose priors (PosePrior, :165,192) go to the BA kernel per pair: the prior
initialises the second camera and adds a between factor (gtsfm_ba2_batched's d_prior_Rt / d_prior_sigmas).
"""
from __future__ import annotations

import dataclasses
import logging
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
from scipy.spatial.transform import Rotation

import math

from gtsfm_amd.common import geometry
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.common.two_view_estimation_report import TwoViewEstimationReport
from gtsfm_amd.frontend.inlier_support_processor import InlierSupportProcessor
from gtsfm_amd.frontend.verifier.verifier_base import VerifierBase
from gtsfm_amd.utils import metrics as metric_utils

logger = logging.getLogger(__name__)

TWO_VIEW_OUTPUT = Tuple[Optional[Any], Optional[Any], np.ndarray, TwoViewEstimationReport, TwoViewEstimationReport,
                        TwoViewEstimationReport]


def _pose(camera) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """(wRi, wti) of a GT camera: a gtsam camera (.pose()), or a 4x4 / 3x4 wTi matrix."""
    return geometry.camera_pose(camera)


def compute_relative_pose_metrics(i2Ri1, i2Ui1, gt_camera_i1, gt_camera_i2) -> Tuple[Optional[float], Optional[float]]:
    """Rotation angle of i2Ri1^-1 * i2Ri1_gt and angle between i2Ui1 and the GT direction, in degrees
    (two_view_estimator.py:396-420 with geometry_comparisons.py:266-309)."""
    p1, p2 = _pose(gt_camera_i1), _pose(gt_camera_i2)
    if p1 is None or p2 is None:
        return None, None
    (R1, t1), (R2, t2) = p1, p2
    R_gt = R2.T @ R1  # i2Ti1 = wTi2^-1 * wTi1
    t_gt = R2.T @ (t1 - t2)
    R_err = U_err = None
    if i2Ri1 is not None:
        rel = geometry.rotation_matrix(i2Ri1).T @ R_gt
        R_err = float(np.rad2deg(np.linalg.norm(Rotation.from_matrix(rel).as_rotvec())))
    if i2Ui1 is not None:
        u = t_gt / np.linalg.norm(t_gt)
        U_err = float(np.rad2deg(np.arccos(np.clip(np.dot(geometry.unit_vector(i2Ui1), u), -1, 1))))
    return R_err, U_err


def generate_two_view_report(inlier_ratio_est_model: float, v_corr_idxs: np.ndarray, R_error_deg=None,
                             U_error_deg=None, v_corr_idxs_inlier_mask_gt=None,
                             reproj_error_gt_model=None) -> TwoViewEstimationReport:
    if v_corr_idxs_inlier_mask_gt is not None and reproj_error_gt_model is not None:
        num_gt = np.count_nonzero(v_corr_idxs_inlier_mask_gt)
        ratio_gt = num_gt / v_corr_idxs.shape[0] if len(v_corr_idxs) > 0 else 0.0
        inl_err = np.mean(reproj_error_gt_model[v_corr_idxs_inlier_mask_gt])
        out_err = np.nanmean(reproj_error_gt_model[np.logical_not(v_corr_idxs_inlier_mask_gt)])
    else:
        num_gt, ratio_gt, inl_err, out_err = 0, float("nan"), float("nan"), float("nan")
    return TwoViewEstimationReport(
        inlier_ratio_est_model=inlier_ratio_est_model, num_inliers_est_model=v_corr_idxs.shape[0],
        num_inliers_gt_model=num_gt, inlier_ratio_gt_model=ratio_gt,
        v_corr_idxs_inlier_mask_gt=v_corr_idxs_inlier_mask_gt, v_corr_idxs=v_corr_idxs, R_error_deg=R_error_deg,
        U_error_deg=U_error_deg, reproj_error_gt_model=reproj_error_gt_model,
        inlier_avg_reproj_error_gt_model=inl_err, outlier_avg_reproj_error_gt_model=out_err)


BA_PAIR_CHUNK = 8192
GTSAM_LM_DEFAULT_MAX_ITERS = 100  # gtsam.LevenbergMarquardtParams().maxIterations


class TwoViewEstimator:
    def __init__(self, verifier: VerifierBase, inlier_support_processor: InlierSupportProcessor,
                 bundle_adjust_2view: bool, eval_threshold_px: float, triangulation_options: Any = None,
                 bundle_adjust_2view_maxiters: int = 100, ba_reproj_error_thresholds: List[Optional[float]] = [0.5]
                 ) -> None:
        self._verifier = verifier
        self.processor = inlier_support_processor
        self._bundle_adjust_2view = bundle_adjust_2view
        self._corr_metric_dist_threshold = eval_threshold_px
        self._triangulation_options = triangulation_options
        self._ba_reproj_error_thresholds = ba_reproj_error_thresholds
        self._bundle_adjust_2view_maxiters = bundle_adjust_2view_maxiters

    # ---------------------------------------------------------------- two-view bundle adjustment (:101-208)
    def _ba_params(self) -> Tuple[int, int, float, float]:
        """(min verified rows, max LM iterations, post-BA reprojection threshold, triangulation threshold)."""
        opts = self._triangulation_options
        mode = getattr(opts, "mode", "NO_RANSAC")
        if str(getattr(mode, "value", mode)) != "NO_RANSAC":
            raise NotImplementedError("two-view triangulation supports TriangulationSamplingMode.NO_RANSAC only")
        if getattr(opts, "min_triangulation_angle", 0.0):
            raise NotImplementedError("min_triangulation_angle > 0 is not supported on the MI355X BA path")
        tri = getattr(opts, "reproj_error_threshold", math.inf)
        # run_ba repeats the stage from the same initial data for every threshold; the last stage's output is kept
        # (bundle_adjustment.py:396-419)
        thr = self._ba_reproj_error_thresholds[-1] if self._ba_reproj_error_thresholds else None
        min_inl = self.processor._min_num_inliers_est_model if self.processor is not None else 0
        # setMaxIterations only when maxiters is truthy (bundle_adjustment.py:273-274): else GTSAM's default of 100
        max_iters = int(self._bundle_adjust_2view_maxiters or 0) or GTSAM_LM_DEFAULT_MAX_ITERS
        # reproj_error_thresh None: no landmark filter (bundle_adjustment.py:346-355) -> an infinite threshold
        return (min_inl, max_iters, math.inf if thr is None else float(thr),
                1e300 if tri is None or math.isinf(tri) else float(tri))

    def bundle_adjust_batch(self, keypoints_list: Sequence[Keypoints],
                            jobs: Dict[Tuple[int, int], Tuple[Any, Any, np.ndarray]], camera_intrinsics: Sequence,
                            priors: Optional[Dict[Tuple[int, int], Any]] = None
                            ) -> Dict[Tuple[int, int], Tuple[Any, Any, np.ndarray]]:
        """bundle_adjust (:136-208) of every (i1, i2) -> (i2Ri1, i2Ui1, verified_corr_idxs) job in batched
        gtsfm_ba2_batched launches; returns (i2Ri1, i2Ui1, valid_corr_idxs) per job, as the reference returns them:
        the initial pose (the prior's when the job has one) and an empty (0, 2) int32 array when nothing
        triangulates, the verifier's pose and the (empty) valid rows when BA leaves no valid track. priors: optional
        (i1, i2) -> PosePrior (i2Ti1_prior)."""
        import torch

        from gtsfm_amd import device, native

        native.require_gpu()
        _, max_iters, thr, tri = self._ba_params()
        from gtsfm_amd.common.pose_prior import prior_arrays

        priors = {k: v for k, v in (priors or {}).items() if v is not None}
        out: Dict[Tuple[int, int], Tuple[Any, Any, np.ndarray]] = {}
        # the initial pose is the prior's when given, else the verifier's (:165-171); neither: nothing to adjust
        keys = [k for k, (R, U, _) in jobs.items() if (R is not None and U is not None) or k in priors]
        for k in jobs:
            if k not in keys:
                out[k] = (None, None, jobs[k][2])
        if not keys:
            return out
        dev = torch.device("cuda")
        n = len(keypoints_list)
        kmax = max([len(k) for k in keypoints_list] + [1])
        kp = np.zeros((n, kmax, 2), np.float32)
        for i, k in enumerate(keypoints_list):
            kp[i, : len(k)] = k.coordinates
        intr = np.zeros((n, 3))
        used = {i for key in keys for i in key}
        for i in used:
            intr[i] = geometry.calibration_params(camera_intrinsics[i])
        kp_d, intr_d = torch.from_numpy(kp).to(dev), torch.from_numpy(intr).to(dev)

        class _Verified:
            pass

        for s in range(0, len(keys), BA_PAIR_CHUNK):
            blk = keys[s: s + BA_PAIR_CHUNK]
            rows = [np.asarray(jobs[k][2]).reshape(-1, 2) for k in blk]
            mcap = max([len(r) for r in rows] + [1])
            idx = np.zeros((len(blk), mcap, 2), np.int32)
            cnt = np.zeros(len(blk), np.int32)
            mask = np.zeros((len(blk), mcap), np.uint8)
            R0 = np.zeros((len(blk), 3, 3))
            t0 = np.zeros((len(blk), 3))
            pRt = np.zeros((len(blk), 12))
            psg = np.zeros((len(blk), 6))
            for j, (k, r) in enumerate(zip(blk, rows)):
                idx[j, : len(r)] = r.astype(np.int64)
                cnt[j] = len(r)
                mask[j, : len(r)] = 1
                if k in priors:
                    Rp, tp, sp = prior_arrays(priors[k])
                    pRt[j, :9], pRt[j, 9:], psg[j] = Rp.ravel(), tp, sp
                if jobs[k][0] is not None and jobs[k][1] is not None:
                    R0[j] = geometry.rotation_matrix(jobs[k][0])
                    t0[j] = geometry.unit_vector(jobs[k][1])
                else:  # prior only: the kernel initialises from the prior
                    R0[j] = pRt[j, :9].reshape(3, 3)
                    t0[j] = pRt[j, 9:] / np.linalg.norm(pRt[j, 9:])
            v = _Verified()
            v.mask, v.R, v.t = (torch.from_numpy(x).to(dev) for x in (mask, R0, t0))
            v.status = torch.zeros(len(blk), dtype=torch.int32, device=dev)
            has_prior = bool(psg[:, 0].any())
            res = device.bundle_adjust_2view(kp_d, intr_d, torch.tensor(blk, dtype=torch.int32, device=dev),
                                             torch.from_numpy(idx).to(dev), torch.from_numpy(cnt).to(dev), v,
                                             min_inliers=0, max_iters=max_iters, reproj_thresh=thr, tri_thresh=tri,
                                             prior_Rt=torch.from_numpy(pRt).to(dev) if has_prior else None,
                                             prior_sigmas=torch.from_numpy(psg).to(dev) if has_prior else None)
            st = res.ba_status.cpu().numpy()
            R, t, m = res.R.cpu().numpy(), res.t.cpu().numpy(), res.mask.cpu().numpy().astype(bool)
            for j, (k, r) in enumerate(zip(blk, rows)):
                if st[j] == native.BA2_STATUS_NO_TRACKS:  # the initial pose (:186-187): the prior's when given
                    init = (geometry.Rot3(R[j]), geometry.Unit3(t[j])) if k in priors else (jobs[k][0], jobs[k][1])
                    out[k] = (init[0], init[1], np.zeros((0, 2), dtype=np.int32))
                elif st[j] == native.BA2_STATUS_NONE_VALID:
                    out[k] = (jobs[k][0], jobs[k][1], np.asarray(jobs[k][2]).reshape(-1, 2)[:0])
                else:
                    out[k] = (geometry.Rot3(R[j]), geometry.Unit3(t[j]),
                              np.asarray(jobs[k][2]).reshape(-1, 2)[m[j, : len(r)]])
        return out

    def bundle_adjust(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, verified_corr_idxs: np.ndarray,
                      camera_intrinsics_i1, camera_intrinsics_i2, i2Ri1_initial, i2Ui1_initial, i2Ti1_prior=None):
        """Drop-in for TwoViewEstimator.bundle_adjust (:136-208): one pair through the batched kernel."""
        if i2Ti1_prior is None and (i2Ri1_initial is None or i2Ui1_initial is None):
            return None, None, verified_corr_idxs
        return self.bundle_adjust_batch([keypoints_i1, keypoints_i2],
                                        {(0, 1): (i2Ri1_initial, i2Ui1_initial, verified_corr_idxs)},
                                        [camera_intrinsics_i1, camera_intrinsics_i2],
                                        priors={(0, 1): i2Ti1_prior})[(0, 1)]

    def _wants_ba(self, v_corr) -> bool:
        return self._bundle_adjust_2view and len(v_corr) >= self.processor._min_num_inliers_est_model

    def get_corr_metric_dist_threshold(self) -> float:
        return self._corr_metric_dist_threshold

    def _report(self, i2Ri1, i2Ui1, keypoints_i1, keypoints_i2, v_corr, ratio, gt_camera_i1, gt_camera_i2,
                gt_scene_mesh=None) -> TwoViewEstimationReport:
        """__get_2view_report_from_results (:210-270): pose errors w.r.t. GT, and for pinhole GT cameras the
        Sampson-distance classification of the verified correspondences (utils/metrics.py:38-96)."""
        R_err = U_err = mask_gt = err_gt = None
        if gt_camera_i1 is not None and gt_camera_i2 is not None:
            R_err, U_err = compute_relative_pose_metrics(i2Ri1, i2Ui1, gt_camera_i1, gt_camera_i2)
            if geometry.is_pinhole_cal3bundler(gt_camera_i1) and geometry.is_pinhole_cal3bundler(gt_camera_i2):
                mask_gt, err_gt = metric_utils.compute_correspondence_metrics(
                    keypoints_i1, keypoints_i2, v_corr, self._corr_metric_dist_threshold, gt_camera_i1, gt_camera_i2,
                    gt_scene_mesh)
        return generate_two_view_report(ratio, v_corr, R_error_deg=R_err, U_error_deg=U_err,
                                        v_corr_idxs_inlier_mask_gt=mask_gt, reproj_error_gt_model=err_gt)

    def _finish(self, verified, keypoints_i1, keypoints_i2, gt_camera_i1, gt_camera_i2, gt_scene_mesh=None,
                post_ba=None) -> TWO_VIEW_OUTPUT:
        """Reports + inlier-support processor for one verifier result and its BA result, if BA ran (:298-351)."""
        i2Ri1, i2Ui1, v_corr, ratio = verified
        pre_ba_report = self._report(i2Ri1, i2Ui1, keypoints_i1, keypoints_i2, v_corr, ratio, gt_camera_i1,
                                     gt_camera_i2, gt_scene_mesh)
        if post_ba is not None:
            R_b, U_b, v_b = post_ba
            # the reference keeps the pre-BA inlier ratio after BA (:325-327)
            post_ba_report = self._report(R_b, U_b, keypoints_i1, keypoints_i2, v_b, ratio, gt_camera_i1,
                                          gt_camera_i2, gt_scene_mesh)
        else:
            R_b, U_b, v_b = i2Ri1, i2Ui1, v_corr
            post_ba_report = dataclasses.replace(pre_ba_report)
        post_isp = self.processor.run_inlier_support(R_b, U_b, v_b, post_ba_report)
        return post_isp[0], post_isp[1], post_isp[2], pre_ba_report, post_ba_report, post_isp[3]

    def run_2view(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, putative_corr_idxs: np.ndarray,
                  camera_intrinsics_i1, camera_intrinsics_i2, i2Ti1_prior=None, gt_camera_i1=None,
                  gt_camera_i2=None, gt_scene_mesh=None) -> TWO_VIEW_OUTPUT:
        verified = self._verifier.verify(keypoints_i1, keypoints_i2, putative_corr_idxs, camera_intrinsics_i1,
                                         camera_intrinsics_i2)
        post_ba = None
        if self._wants_ba(verified[2]):
            post_ba = self.bundle_adjust(keypoints_i1, keypoints_i2, verified[2], camera_intrinsics_i1,
                                         camera_intrinsics_i2, verified[0], verified[1], i2Ti1_prior)
        return self._finish(verified, keypoints_i1, keypoints_i2, gt_camera_i1, gt_camera_i2, gt_scene_mesh, post_ba)


def run_two_view_estimator_as_futures(
    client,
    two_view_estimator: TwoViewEstimator,
    keypoints_list: Sequence[Keypoints],
    putative_corr_idxs_dict: Dict[Tuple[int, int], np.ndarray],
    camera_intrinsics: Sequence,
    relative_pose_priors: Dict[Tuple[int, int], Any],
    gt_cameras: Sequence[Optional[Any]],
    gt_scene_mesh: Optional[Any],
) -> Dict[Tuple[int, int], TWO_VIEW_OUTPUT]:
    """All pairs of `putative_corr_idxs_dict` -> TWO_VIEW_OUTPUT, one batched verifier launch for all of them.

    `client` is accepted for signature compatibility (two_view_estimator.py:531-540) and unused.
    """
    verifier = two_view_estimator._verifier
    gt = list(gt_cameras) if gt_cameras is not None else [None] * len(keypoints_list)
    # a TwoViewEstimatorCacher answers hits from disk; only the misses go through the batched verifier
    cached = getattr(two_view_estimator, "cache_lookup", None)
    results: Dict[Tuple[int, int], TWO_VIEW_OUTPUT] = {}
    if cached is not None:
        for (i1, i2), m in putative_corr_idxs_dict.items():
            hit = cached(keypoints_list[i1], keypoints_list[i2], m)
            if hit is not None:
                results[(i1, i2)] = hit
    todo = {k: m for k, m in putative_corr_idxs_dict.items() if k not in results}
    if hasattr(verifier, "verify_batch"):
        verified = verifier.verify_batch(keypoints_list, todo, camera_intrinsics)
    else:
        verified = {(i1, i2): verifier.verify(keypoints_list[i1], keypoints_list[i2], m, camera_intrinsics[i1],
                                              camera_intrinsics[i2])
                    for (i1, i2), m in todo.items()}
    post_ba: Dict[Tuple[int, int], Any] = {}
    ba_jobs = {k: verified[k][:3] for k in todo if two_view_estimator._wants_ba(verified[k][2])}
    if ba_jobs:
        post_ba = two_view_estimator.bundle_adjust_batch(keypoints_list, ba_jobs, camera_intrinsics,
                                                         priors={k: (relative_pose_priors or {}).get(k)
                                                                 for k in ba_jobs})
    for (i1, i2), m in todo.items():
        results[(i1, i2)] = two_view_estimator._finish(verified[(i1, i2)], keypoints_list[i1], keypoints_list[i2],
                                                       gt[i1], gt[i2], gt_scene_mesh, post_ba.get((i1, i2)))
        if cached is not None:
            two_view_estimator.cache_store(keypoints_list[i1], keypoints_list[i2], m, results[(i1, i2)])
    return {k: results[k] for k in putative_corr_idxs_dict}
