"""Pose prior type (reference gtsfm/common/pose_prior.py): a Pose3 value, its sigmas in GTSAM's tangent order
(rotation, then translation; the reference names the field `covariance` although it holds sigmas) and the
constraint type. Two-view bundle adjustment takes one per pair as i2Ti1_prior (two_view_estimator.py:165,192)."""
from enum import Enum
from typing import Any, NamedTuple

import numpy as np


class PosePriorType(str, Enum):
    HARD_CONSTRAINT = "hard_constraint"
    SOFT_CONSTRAINT = "soft_constraint"


class PosePrior(NamedTuple):
    value: Any           # Pose3 (gtsam's, or gtsfm_amd.common.geometry.Pose3 without gtsam)
    covariance: np.ndarray  # sigmas (6,)
    type: PosePriorType


def prior_arrays(prior: PosePrior):
    """(R (3, 3), t (3,), sigmas (6,)) float64 of a PosePrior, for the device BA."""
    from gtsfm_amd.common import geometry

    R = geometry.rotation_matrix(prior.value.rotation())
    t = np.asarray(prior.value.translation(), dtype=np.float64).reshape(3)
    sig = np.asarray(prior.covariance, dtype=np.float64).reshape(6)
    if not np.all(sig > 0):
        raise ValueError("pose prior sigmas must be positive")
    return R, t, sig
