"""Per-pair verification report (reference: gtsfm/common/two_view_estimation_report.py:13-53, same fields)."""
from dataclasses import dataclass
from typing import Any, Optional

import numpy as np


@dataclass(frozen=False)
class TwoViewEstimationReport:
    """What the verifier concluded about edge (i1, i2); GT fields stay None without ground-truth cameras."""

    v_corr_idxs: np.ndarray
    num_inliers_est_model: float
    inlier_ratio_est_model: Optional[float] = None
    num_inliers_gt_model: Optional[float] = None
    inlier_ratio_gt_model: Optional[float] = None
    v_corr_idxs_inlier_mask_gt: Optional[np.ndarray] = None
    R_error_deg: Optional[float] = None
    U_error_deg: Optional[float] = None
    i2Ri1: Optional[Any] = None
    i2Ui1: Optional[Any] = None
    reproj_error_gt_model: Optional[np.ndarray] = None
    inlier_avg_reproj_error_gt_model: Optional[float] = None
    outlier_avg_reproj_error_gt_model: Optional[float] = None
