"""Plugins survive pickling, as the reference requires for scattering them to Dask workers
(tests/frontend/matcher/test_matcher_base.py:102-107, tests/frontend/verifier/test_verifier_base.py:140-146,
tests/frontend/detector/test_detector_base.py:51-56). CPU only: construction and pickling must not touch the GPU,
and device-side state (packed weights) is dropped from the pickled state and re-created lazily per process.
"""
import pickle

import numpy as np
import pytest

from gtsfm_amd.frontend.cacher.detector_descriptor_cacher import DetectorDescriptorCacher
from gtsfm_amd.frontend.cacher.matcher_cacher import MatcherCacher
from gtsfm_amd.frontend.correspondence_generator.det_desc_correspondence_generator import (
    DetDescCorrespondenceGenerator,
)
from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor
from gtsfm_amd.frontend.detector_descriptor.superpoint import SuperPointDetectorDescriptor
from gtsfm_amd.frontend.inlier_support_processor import InlierSupportProcessor
from gtsfm_amd.frontend.matcher.superglue_matcher import SuperGlueMatcher
from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher
from gtsfm_amd.frontend.verifier.ransac import Ransac
from gtsfm_amd.two_view_estimator import TwoViewEstimator
from gtsfm_amd.two_view_estimator_cacher import TwoViewEstimatorCacher


def _plugins():
    sift = SIFTDetectorDescriptor(max_keypoints=2048)
    matcher = TwoWayMatcher(ratio_test_threshold=0.8)
    verifier = Ransac(use_intrinsics_in_verification=True, estimation_threshold_px=4.0)
    est = TwoViewEstimator(verifier, InlierSupportProcessor(15, 0.1), bundle_adjust_2view=False, eval_threshold_px=4)
    return [
        sift, matcher, verifier, est,
        Ransac(use_intrinsics_in_verification=False, estimation_threshold_px=4.0),
        SuperPointDetectorDescriptor(max_keypoints=4096),
        SuperGlueMatcher(),
        DetDescCorrespondenceGenerator(matcher, sift),
        DetectorDescriptorCacher(sift), MatcherCacher(matcher), TwoViewEstimatorCacher(est),
    ]


@pytest.mark.parametrize("idx", range(11))
def test_plugin_pickles(idx):
    obj = _plugins()[idx]
    clone = pickle.loads(pickle.dumps(obj))
    assert type(clone) is type(obj)
    if hasattr(obj, "max_keypoints"):
        assert clone.max_keypoints == obj.max_keypoints


def test_device_state_not_pickled():
    sp = SuperPointDetectorDescriptor(max_keypoints=4096)
    sp._blob = object()  # stands in for packed device weights
    assert pickle.loads(pickle.dumps(sp))._blob is None
    sg = SuperGlueMatcher()
    sg._blob = object()
    assert pickle.loads(pickle.dumps(sg))._blob is None


def test_empty_inputs_need_no_gpu():
    """Empty descriptor sets return the reference's empty result (twoway_matcher.py:71-72) without a device call."""
    m = TwoWayMatcher(ratio_test_threshold=0.8)
    out = m.match(None, None, np.zeros((0, 128), np.float32), np.zeros((5, 128), np.float32), (4, 4, 3), (4, 4, 3))
    assert out.size == 0


def test_ransac_rejects_out_of_range_indices_and_missing_intrinsics():
    """Index checks happen on the host before any device call (reference: numpy IndexError on fancy indexing)."""
    import pytest

    from gtsfm_amd.common import geometry
    from gtsfm_amd.common.keypoints import Keypoints
    from gtsfm_amd.frontend.verifier.ransac import Ransac, _checked_indices

    kp = Keypoints(coordinates=np.random.default_rng(0).uniform(0, 100, (10, 2)))
    v = Ransac(use_intrinsics_in_verification=True, estimation_threshold_px=4)
    bad = np.stack([np.arange(8), np.arange(8)], 1)
    bad[3, 1] = 10
    with pytest.raises(IndexError):
        v.verify(kp, kp, bad, geometry.Cal3Bundler(), geometry.Cal3Bundler())
    with pytest.raises(ValueError):
        v.verify(kp, kp, bad[:, ::-1] % 10, None, geometry.Cal3Bundler())
    np.testing.assert_array_equal(_checked_indices(np.array([[-1, 2], [3, -10]]), 10, 10), [[9, 2], [3, 0]])
