"""TriangulationOptions of the two-view estimator (reference gtsfm/data_association/point3d_initializer.py:51-99).

Only the fields the two-view bundle adjustment reads are used: `mode` must be NO_RANSAC (the two-view estimator's
configuration, sift_front_end.yaml), `reproj_error_threshold` (default inf, "no filtering unless specified") and
`min_triangulation_angle` (default 0: no rejection). The RANSAC fields are kept for constructor compatibility.
"""
import math
import sys
from enum import Enum
from typing import NamedTuple


class TriangulationSamplingMode(str, Enum):
    NO_RANSAC = "NO_RANSAC"
    RANSAC_SAMPLE_UNIFORM = "RANSAC_SAMPLE_UNIFORM"
    RANSAC_SAMPLE_BIASED_BASELINE = "RANSAC_SAMPLE_BIASED_BASELINE"
    RANSAC_TOPK_BASELINES = "RANSAC_TOPK_BASELINES"


class TriangulationOptions(NamedTuple):
    mode: TriangulationSamplingMode
    reproj_error_threshold: float = math.inf
    min_triangulation_angle: float = 0.0
    min_inlier_ratio: float = 0.1
    confidence: float = 0.9999
    dyn_num_hypotheses_multiplier: float = 3.0
    min_num_hypotheses: int = 0
    max_num_hypotheses: int = sys.maxsize
