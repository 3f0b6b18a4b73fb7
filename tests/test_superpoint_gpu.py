"""HIP SuperPoint (gtsfm_superpoint_batched) against the reference module's own outputs.

Golden: tests/golden/superpoint_random_w0.npz, written by tests/golden/make_superpoint_golden.py, which runs
thirdparty/SuperGluePretrainedNetwork/models/superpoint.py (torch fp32, CPU) with the seeded random weights of
tests/superpoint_weights.py (the pretrained weights are not available offline). The HIP convolutions are exact fp32
MFMA products/sums in a different order than torch's, so scores agree to ~1e-6 relative; keypoints are compared as
sets (>= 99.5 % identical; a differing keypoint needs two NMS-window scores within that rounding), scores within
rtol 1e-4, descriptors within 2e-4 per entry.
"""
import os

import numpy as np
import pytest
import torch

from superpoint_weights import superpoint_state_dict

pytestmark = pytest.mark.gpu
CASES = ["synthetic_240x320", "lund_250x333", "lund_480x640"]


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "superpoint_random_w0.npz"))


@pytest.fixture(scope="module")
def det():
    from gtsfm_amd import native
    from gtsfm_amd.frontend.detector_descriptor.superpoint import SuperPointDetectorDescriptor

    native.require_gpu()
    return SuperPointDetectorDescriptor(max_keypoints=16384, state_dict=superpoint_state_dict(0))


def _keyset(xy):
    return {(int(round(x)), int(round(y))) for x, y in xy}


@pytest.mark.parametrize("case", CASES)
def test_matches_reference_module(det, golden, case):
    img = golden[f"{case}__image"]
    ref_kp, ref_sc = golden[f"{case}__keypoints"], golden[f"{case}__scores"]
    res = det.extract_batch([img])
    n = int(res.count[0])
    assert int(res.n_detected[0]) == n  # max_keypoints above the detection count: everything, raster order
    xy = res.xy[0, :n].cpu().numpy()
    sc = res.scores[0, :n].cpu().numpy()
    desc = res.desc[0, :n].cpu().numpy()
    assert np.array_equal(xy, np.round(xy))
    a, b = _keyset(xy), _keyset(ref_kp)
    common = a & b
    assert len(common) >= 0.995 * max(len(a), len(b)), (len(a), len(b), len(common))
    pos = {k: i for i, k in enumerate(map(tuple, np.round(xy).astype(int)))}
    # raster order (row-major on (y, x)), as torch.nonzero returns it
    order = np.lexsort((xy[:, 0], xy[:, 1]))
    assert np.array_equal(order, np.arange(n))
    ref_pos = [pos.get((int(x), int(y)), -1) for x, y in ref_kp]
    m = np.array([p >= 0 for p in ref_pos])
    np.testing.assert_allclose(sc[np.array(ref_pos)[m]], ref_sc[m], rtol=1e-4)
    rows = golden[f"{case}__desc_rows"]
    rdesc = golden[f"{case}__desc"]
    for r, d in zip(rows, rdesc):
        p = ref_pos[r]
        if p >= 0:
            np.testing.assert_allclose(desc[p], d, atol=2e-4)
    np.testing.assert_allclose(np.linalg.norm(desc, axis=1), 1.0, atol=1e-5)


def test_top_k_and_batch(det, golden):
    """Same-size batch == single calls; top-k keeps the k highest scores (raster order within)."""
    img = golden["synthetic_240x320__image"]
    full = det.extract_batch([img])
    n = int(full.count[0])
    k = n // 3
    sub = det.extract_batch([img, img[::-1].copy()], max_kpts=k)
    assert int(sub.count[0]) == k and int(sub.n_detected[0]) == n
    sc_all = full.scores[0, :n].cpu().numpy()
    thr = np.sort(sc_all)[::-1][k - 1]
    got = sub.scores[0, :k].cpu().numpy()
    assert (got >= thr).all() and np.isclose(np.sort(got)[::-1], np.sort(sc_all)[::-1][:k]).all()
    xy = sub.xy[0, :k].cpu().numpy()
    assert np.array_equal(np.lexsort((xy[:, 0], xy[:, 1])), np.arange(k))
    single_flip = det.extract_batch([img[::-1].copy()], max_kpts=k)
    m = int(single_flip.count[0])
    assert m == int(sub.count[1])
    assert torch.equal(single_flip.xy[0, :m], sub.xy[1, :m])
    assert torch.equal(single_flip.desc[0, :m], sub.desc[1, :m])


def test_plugin_api(det, golden):
    from gtsfm_amd.common.image import Image

    img = golden["lund_250x333__image"]
    rgb = np.repeat(img[:, :, None], 3, axis=2)
    d = type(det)(max_keypoints=500, state_dict=superpoint_state_dict(0))
    kp, desc = d.detect_and_describe(Image(rgb))
    assert len(kp) == 500 and desc.shape == (500, 256) and desc.dtype == np.float32
    assert kp.scales is None and kp.responses.shape == (500,) and kp.coordinates.dtype == np.float32


def test_c3_1080p_top_4096(det, golden, golden_dir):
    """BASELINE config C3's extraction: a 1920 x 1080 image, max_keypoints 4096 (the drop-in's get_top_k(4096) over
    the reference module's detections). The kept set is the reference's 4096 highest scores (ties at the boundary
    aside), emitted in raster order; scores rtol 1e-4 and descriptors 2e-4 as above."""
    from PIL import Image as PILImage

    gray = np.asarray(PILImage.open(os.path.join(golden_dir, "lund_door_DSC_0001_gray.png")))
    img = np.ascontiguousarray(gray[8:1928, 108:1188])  # make_superpoint_golden.LUND_1080P_CROP
    ref_kp, ref_sc = golden["lund_1920x1080__keypoints"], golden["lund_1920x1080__scores"]
    res = det.extract_batch([img], max_kpts=4096)
    n = int(res.count[0])
    assert n == 4096 and abs(int(res.n_detected[0]) - len(ref_kp)) <= 0.005 * len(ref_kp)
    xy = res.xy[0, :n].cpu().numpy()
    sc = res.scores[0, :n].cpu().numpy()
    desc = res.desc[0, :n].cpu().numpy()
    assert np.array_equal(np.lexsort((xy[:, 0], xy[:, 1])), np.arange(n))
    top = np.argsort(-ref_sc, kind="stable")[:4096]
    a, b = _keyset(xy), _keyset(ref_kp[top])
    assert len(a & b) >= 0.995 * 4096, len(a & b)
    pos = {k: i for i, k in enumerate(map(tuple, np.round(xy).astype(int)))}
    ref_pos = np.array([pos.get((int(x), int(y)), -1) for x, y in ref_kp])
    m = ref_pos >= 0
    np.testing.assert_allclose(sc[ref_pos[m]], ref_sc[m], rtol=1e-4)
    for r, d in zip(golden["lund_1920x1080__desc_rows"], golden["lund_1920x1080__desc"]):
        if ref_pos[r] >= 0:
            np.testing.assert_allclose(desc[ref_pos[r]], d, atol=2e-4)


def _c3_mask(H, W):
    """A mask with a hole, a margin and stray values 2 (filter_by_mask keeps only == 1)."""
    rng = np.random.default_rng(11)
    m = np.ones((H, W), np.uint8)
    m[H // 4: H // 2, W // 3: 2 * W // 3] = 0
    m[:, : W // 10] = 0
    m[rng.random((H, W)) < 0.05] = 2
    return m


def test_c3_1080p_mask_top_4096(det, golden_dir):
    """Row a16 with image.mask (reference superpoint.py:68-72: filter_by_mask, then get_top_k(4096)): the masked
    device run equals, bit for bit, the unmasked device run's detections filtered by mask == 1 and cut to the 4096
    highest scores (raster order within, ties by raster order); and keeps >= 99.5 % of the oracle's masked set."""
    from PIL import Image as PILImage

    gray = np.asarray(PILImage.open(os.path.join(golden_dir, "lund_door_DSC_0001_gray.png")))
    img = np.ascontiguousarray(gray[8:1928, 108:1188])
    H, W = img.shape
    mask = _c3_mask(H, W)
    full = det.extract_batch([img], max_kpts=1 << 17)
    n = int(full.count[0])
    assert n == int(full.n_detected[0]) and n > 8192
    xy = full.xy[0, :n].cpu().numpy()
    sc = full.scores[0, :n].cpu().numpy()
    desc = full.desc[0, :n].cpu().numpy()
    keep = np.flatnonzero(mask[xy[:, 1].astype(int), xy[:, 0].astype(int)] == 1)
    assert 0 < len(keep) < n
    top = keep[np.sort(np.argsort(-sc[keep], kind="stable")[:4096])]
    res = det.extract_batch([img], max_kpts=4096, masks=[mask])
    m = int(res.count[0])
    assert m == min(4096, len(keep)) and int(res.n_detected[0]) == len(keep)
    assert np.array_equal(res.xy[0, :m].cpu().numpy(), xy[top])
    assert np.array_equal(res.scores[0, :m].cpu().numpy(), sc[top])
    assert np.array_equal(res.desc[0, :m].cpu().numpy(), desc[top])
    # the oracle (reference module restated on the host) with the same mask
    from oracle import deep

    o_xy, o_sc, _ = deep.superpoint(img, superpoint_state_dict(0), max_keypoints=4096, mask=mask)
    a, b = _keyset(res.xy[0, :m].cpu().numpy()), _keyset(o_xy)
    assert len(a & b) >= 0.995 * max(len(a), len(b)), (len(a), len(b), len(a & b))


def test_plugin_mask_equals_batched(det, golden):
    """The drop-in's detect_and_describe(Image(value, mask)) and the batched generator's extraction agree, and a mask
    of all ones changes nothing."""
    from gtsfm_amd.common.image import Image
    from gtsfm_amd.frontend.correspondence_generator.det_desc_correspondence_generator import \
        extract_superpoint_batched

    img = golden["lund_480x640__image"]
    mask = _c3_mask(*img.shape)
    d = type(det)(max_keypoints=700, state_dict=superpoint_state_dict(0))
    kp, desc = d.detect_and_describe(Image(img, mask=mask))
    assert len(kp) <= 700 and (mask[kp.coordinates[:, 1].astype(int), kp.coordinates[:, 0].astype(int)] == 1).all()
    feats = extract_superpoint_batched(d, [Image(img, mask=mask), Image(img)])
    n0 = int(feats.count[0])
    assert n0 == len(kp)
    assert np.array_equal(feats.xy[0, :n0].cpu().numpy(), kp.coordinates)
    assert np.array_equal(feats.desc[0, :n0].cpu().numpy(), desc)
    kp1, desc1 = d.detect_and_describe(Image(img, mask=np.ones(img.shape, np.uint8)))
    kp2, desc2 = d.detect_and_describe(Image(img))
    assert np.array_equal(kp1.coordinates, kp2.coordinates) and np.array_equal(desc1, desc2)
