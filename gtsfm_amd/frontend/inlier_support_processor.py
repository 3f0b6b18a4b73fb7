"""Inlier-support filter on verified pairs (reference: gtsfm/frontend/inlier_support_processor.py:19-95).

Same thresholds and the same failure tuple: a pair fails when its inlier ratio w.r.t. the estimated model is below
`min_inlier_ratio_est_model` (:79), or when it has a model (> 0 inliers) with fewer than
`min_num_inliers_est_model` inliers (:84). The failure report keeps the verified indices but reports 0 inliers.
"""
import dataclasses
from typing import Optional, Tuple

import numpy as np

from gtsfm_amd.common.two_view_estimation_report import TwoViewEstimationReport


class InlierSupportProcessor:
    def __init__(self, min_num_inliers_est_model: int, min_inlier_ratio_est_model: float) -> None:
        self._min_num_inliers_est_model = min_num_inliers_est_model
        self._min_inlier_ratio_est_model = min_inlier_ratio_est_model

    def run_inlier_support(
        self, i2Ri1, i2Ui1, v_corr_idxs: np.ndarray, two_view_report: TwoViewEstimationReport
    ) -> Tuple[Optional[object], Optional[object], np.ndarray, TwoViewEstimationReport]:
        failure_result = (
            None,
            None,
            np.array([], dtype=np.uint64),
            TwoViewEstimationReport(v_corr_idxs=v_corr_idxs, num_inliers_est_model=0),
        )
        report_post_isp = dataclasses.replace(two_view_report)
        insufficient_inliers = two_view_report.num_inliers_est_model < self._min_num_inliers_est_model
        valid_model = two_view_report.num_inliers_est_model > 0
        if two_view_report.inlier_ratio_est_model < self._min_inlier_ratio_est_model:
            return failure_result
        if valid_model and insufficient_inliers:
            return failure_result
        return i2Ri1, i2Ui1, v_corr_idxs, report_post_isp
