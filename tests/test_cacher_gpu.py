"""Front-end caches over the HIP plugins: a cache hit returns exactly what the HIP path
computed, and the HIP path is not called again. Reference behaviour: gtsfm/frontend/cacher/*_cacher.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from gtsfm_amd import native

    native.require_gpu()
    native.lib()
    return torch.device("cuda")


class _Counting:
    """Forwards to a plugin and counts the calls that reach it."""

    def __init__(self, inner, method):
        self.inner, self.method, self.calls = inner, method, 0
        self.max_keypoints = getattr(inner, "max_keypoints", None)

    def __getattr__(self, name):
        if name == self.__dict__.get("method"):
            def call(*a, **k):
                self.calls += 1
                return getattr(self.inner, name)(*a, **k)
            return call
        raise AttributeError(name)


def test_sift_and_matcher_cachers_over_hip(dev, oracle_mod, tmp_path):
    from gtsfm_amd import synthetic
    from gtsfm_amd.common.image import Image
    from gtsfm_amd.frontend.cacher.detector_descriptor_cacher import DetectorDescriptorCacher
    from gtsfm_amd.frontend.cacher.matcher_cacher import MatcherCacher
    from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher

    scene = synthetic.render_scene(2, 240, 320, device=dev)
    arr = scene.images.cpu().numpy()
    det = _Counting(SIFTDetectorDescriptor(max_keypoints=400), "detect_and_describe")
    dcache = DetectorDescriptorCacher(det, cache_root=tmp_path)
    images = [Image(arr[i], file_name=f"view_{i}.png") for i in (0, 1)]
    fresh = [dcache.detect_and_describe(im) for im in images]
    cached = [dcache.detect_and_describe(im) for im in images]
    assert det.calls == 2
    for (k0, d0), (k1, d1) in zip(fresh, cached):
        assert k0 == k1 and np.array_equal(d0, d1)

    m = _Counting(TwoWayMatcher(ratio_test_threshold=0.8), "match")
    mcache = MatcherCacher(m, cache_root=tmp_path)
    args = (fresh[0][0], fresh[1][0], fresh[0][1], fresh[1][1], arr[0].shape, arr[1].shape)
    a = mcache.match(*args)
    b = mcache.match(*args)
    assert m.calls == 1
    assert np.array_equal(a, b) and b.dtype == np.uint32
    assert np.array_equal(a.reshape(-1, 2), oracle_mod.twoway_match(fresh[0][1], fresh[1][1], 0.8).reshape(-1, 2))
