"""The reference's shipped front-end wiring through the batched device path.

sift_front_end.yaml:23-33 wraps SIFTDetectorDescriptor(max_keypoints=5000) in DetectorDescriptorCacher and
TwoWayMatcher(ratio_test_threshold=0.8) in MatcherCacher. DetDescCorrespondenceGenerator looks through both cachers:
hits are read from disk under the reference's keys, only the misses go through the batched extraction / matcher
launches, and the misses are written back (reference: frontend/cacher/detector_descriptor_cacher.py:71-95,
matcher_cacher.py:126-192, det_desc_correspondence_generator.py:64-87).

Checked on BASELINE config C1 (the 12 Lund Door images, all 66 pairs):
- cold cache: keypoints, descriptors and putatives bit-identical to the oracle golden (which the unwrapped batched run
  also equals, tests/test_lund_door_c1_gpu.py); 12 + 66 entries written, by ONE batched extraction of 12 images and
  ONE batched match of 66 pairs; the per-call plugin methods are never called;
- the written entries equal what the per-call cachers write for the same image / pair;
- warm cache: every entry read, no device launch, results identical;
- partial cache: only the deleted images / pairs are recomputed (batched), results identical;
- an entry written by the REFERENCE'S own cacher (tests/golden/reference_cache, OpenCV descriptors) mixes with a
  batched miss, and the pair's putatives equal the oracle matcher's on those descriptors.
"""
import json
import os
import shutil
from pathlib import Path

import numpy as np
import pytest

from tests.test_lund_door_c1_gpu import LUND, _images, _sha

pytestmark = pytest.mark.gpu


class _Spy:
    """Wraps a module-level batched function and records the number of items each call got."""

    def __init__(self, fn, arg):
        self.fn, self.arg, self.sizes = fn, arg, []

    def __call__(self, *a, **k):
        self.sizes.append(len(a[self.arg]))
        return self.fn(*a, **k)


@pytest.fixture()
def spies(monkeypatch):
    from gtsfm_amd.frontend.correspondence_generator import det_desc_correspondence_generator as g
    from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher

    def per_call(*a, **k):
        raise AssertionError("the per-call plugin path was used")

    monkeypatch.setattr(SIFTDetectorDescriptor, "detect_and_describe", per_call)
    monkeypatch.setattr(TwoWayMatcher, "match", per_call)
    ex = _Spy(g.extract_sift_batched, 1)
    mt = _Spy(g.match_pairs_batched, 1)
    monkeypatch.setattr(g, "extract_sift_batched", ex)
    monkeypatch.setattr(g, "match_pairs_batched", mt)
    return ex, mt


def _yaml_generator(root: Path):
    """sift_front_end.yaml:20-33's object graph, with the caches under `root`."""
    from gtsfm_amd.frontend.cacher.detector_descriptor_cacher import DetectorDescriptorCacher
    from gtsfm_amd.frontend.cacher.matcher_cacher import MatcherCacher
    from gtsfm_amd.frontend.correspondence_generator.det_desc_correspondence_generator import \
        DetDescCorrespondenceGenerator
    from gtsfm_amd.frontend.detector_descriptor.sift import SIFTDetectorDescriptor
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher

    return DetDescCorrespondenceGenerator(
        matcher=MatcherCacher(TwoWayMatcher(ratio_test_threshold=0.8), cache_root=root),
        detector_descriptor=DetectorDescriptorCacher(SIFTDetectorDescriptor(max_keypoints=5000), cache_root=root))


def _check_golden(kps, corr, z, sh, pairs):
    off = np.concatenate([[0], np.cumsum(z["match_count"])])
    for p, key in enumerate(pairs):
        np.testing.assert_array_equal(corr[key].reshape(-1, 2), z["matches"][off[p]: off[p + 1]].reshape(-1, 2))
        assert corr[key].dtype == np.uint32 or corr[key].size == 0
    np.testing.assert_array_equal([len(k) for k in kps], z["kp_count"])


def test_shipped_cacher_wiring_batched_cold_warm_partial(tmp_path, spies):
    from gtsfm_amd import native
    from gtsfm_amd.common.image import Image
    from gtsfm_amd.frontend.cacher.matcher_cacher import MatcherCacher
    from gtsfm_amd.utils import io as io_utils

    native.require_gpu()
    ex, mt = spies
    gt, arrs = _images()
    imgs = [Image(a) for a in arrs]
    z = np.load(os.path.join(LUND, "oracle_c1.npz"))
    sh = json.load(open(os.path.join(LUND, "oracle_c1_features.json")))
    pairs = [tuple(map(int, p)) for p in z["pairs"]]

    # cold: everything computed by one batched extraction and one batched match, everything written
    gen = _yaml_generator(tmp_path)
    kps, corr = gen.generate_correspondences(None, imgs, pairs)
    assert ex.sizes == [12] and mt.sizes == [66]
    _check_golden(kps, corr, z, sh, pairs)
    det_files = sorted((tmp_path / "detector_descriptor").glob("*.pbz2"))
    match_files = sorted((tmp_path / "matcher").glob("*.pbz2"))
    assert len(det_files) == 12 and len(match_files) == 66
    # each detector entry is the per-call plugin's output: the oracle's features (sha of xy f32 + descriptors)
    dc = gen._detector_descriptor
    for i, im in enumerate(imgs):
        kp, desc = dc.cache_lookup(im)
        assert desc.dtype == np.float32 and kp.coordinates.dtype == np.float64
        assert _sha(kp.coordinates.astype(np.float32), desc) == sh["sha256_xy_desc"][i], i
    # each matcher entry sits under the key the per-call MatcherCacher computes from the per-call outputs
    mc: MatcherCacher = gen._matcher
    for (i1, i2) in pairs[::11]:
        k1, d1 = dc.cache_lookup(imgs[i1])
        k2, d2 = dc.cache_lookup(imgs[i2])
        p = mc.cache_path(k1, k2, d1, d2, imgs[i1].shape, imgs[i2].shape)
        np.testing.assert_array_equal(io_utils.read_from_bz2_file(p), corr[(i1, i2)])

    # warm: every entry read, no launch
    ex.sizes.clear(), mt.sizes.clear()
    kps_w, corr_w = _yaml_generator(tmp_path).generate_correspondences(None, imgs, pairs)
    assert ex.sizes == [] and mt.sizes == []
    for a, b in zip(kps, kps_w):
        assert a == b
    for key in pairs:
        np.testing.assert_array_equal(corr[key], corr_w[key])

    # partial: two images and five pairs deleted -> only those recomputed, batched, results unchanged
    for i in (3, 7):
        os.remove(dc._cache_path(imgs[i]))
    gone = pairs[5:10]
    for (i1, i2) in gone:
        os.remove(mc.cache_path(kps[i1], kps[i2], _head(gen, i1), _head(gen, i2), imgs[i1].shape, imgs[i2].shape))
    ex.sizes.clear(), mt.sizes.clear()
    gen_p = _yaml_generator(tmp_path)
    kps_p, corr_p = gen_p.generate_correspondences(None, imgs, pairs)
    assert ex.sizes == [2] and mt.sizes == [5]
    _check_golden(kps_p, corr_p, z, sh, pairs)
    feats = gen_p.device_features
    cnt = feats.count.cpu().numpy()
    xy, desc = feats.xy.cpu().numpy(), feats.desc.cpu().numpy()
    for i in range(12):  # hits uploaded from disk and batched misses scattered into one block
        assert _sha(xy[i, : cnt[i]], desc[i, : cnt[i]]) == sh["sha256_xy_desc"][i], i
    assert len(list((tmp_path / "detector_descriptor").glob("*.pbz2"))) == 12
    assert len(list((tmp_path / "matcher").glob("*.pbz2"))) == 66


def _head(gen, i):
    f = gen.device_features
    n = int(f.count[i].item())
    return f.desc[i, : min(10, n)].cpu().numpy()


def test_reference_written_entry_mixes_with_batched_miss(tmp_path, spies, oracle_mod):
    """Image 0 is answered by the detector entry the reference's own DetectorDescriptorCacher wrote (OpenCV SIFT
    descriptors of DSC_0001, keyed by a crop); Lund image 1 misses and is extracted on the device. The pair's putatives equal the oracle
    matcher on (reference descriptors, HIP descriptors)."""
    from gtsfm_amd import native
    from gtsfm_amd.common.image import Image

    native.require_gpu()
    ex, mt = spies
    ref = Path(__file__).resolve().parent / "golden" / "reference_cache"
    shutil.copytree(ref / "detector_descriptor", tmp_path / "detector_descriptor")
    inp = np.load(ref / "inputs.npz")
    _, arrs = _images()
    # image 0's key is the crop; its payload is the reference fixture's 300 OpenCV features of the whole DSC_0001
    imgs = [Image(inp["crop"], file_name="DSC_0001.JPG"), Image(arrs[1])]
    gen = _yaml_generator(tmp_path)
    kps, corr = gen.generate_correspondences(None, imgs, [(0, 1)])
    assert ex.sizes == [1] and mt.sizes == [1]
    np.testing.assert_array_equal(kps[0].coordinates, inp["coords0"])
    d1 = gen._detector_descriptor.cache_lookup(imgs[1])[1]
    want = oracle_mod.twoway_match(inp["d0"], d1, 0.8)
    np.testing.assert_array_equal(corr[(0, 1)].reshape(-1, 2), want.reshape(-1, 2))
    assert len(want) > 0
