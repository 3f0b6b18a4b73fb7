"""GPU verifier (gtsfm_ransac_E_batched via the Ransac drop-in) against the reference's known answers and the oracle.

Known answers (reference tests, committed as data): two-plane scene (all 8 verified, R/t < 2 deg), Argoverse
hand-labelled pair (Euler +-1 deg, t +-0.01), the M<6 failure path, empty matches.
Oracle parity: same sampling, same solver, same fp32 inlier test, same LO, the same fp64 operations (no FMA
contraction, the same explicit fma()s, the LO normal-matrix sums in the wave reduction's order) => per pair the same
number of hypotheses, the same inlier count and mask, and bit-identical R and t.
"""
import json
import os

import numpy as np
import pytest
import torch
from scipy.spatial.transform import Rotation

from tests import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from gtsfm_amd import native

    native.require_gpu()
    native.lib()
    return torch.device("cuda")


def _kp(xy):
    from gtsfm_amd.common.keypoints import Keypoints

    return Keypoints(coordinates=np.asarray(xy, dtype=np.float64))


def test_two_plane_scene(dev):
    from gtsfm_amd.common import geometry
    from gtsfm_amd.frontend.verifier.ransac import Ransac

    uv1, uv2, R, t = scenes.two_planes_scene(4, 4)
    match = np.vstack((np.arange(8), np.arange(8))).T
    v = Ransac(use_intrinsics_in_verification=True, estimation_threshold_px=0.5)
    Rc, Uc, idx, ratio = v.verify(_kp(uv1), _kp(uv2), match, geometry.Cal3Bundler(), geometry.Cal3Bundler())
    np.testing.assert_array_equal(idx, match)
    assert ratio == 1.0
    assert scenes.rotation_angle_deg(R, geometry.rotation_matrix(Rc)) < 2
    assert scenes.direction_angle_deg(t, geometry.unit_vector(Uc)) < 2


def test_argoverse_known_answer(dev, golden_dir):
    from gtsfm_amd.common import geometry
    from gtsfm_amd.frontend.verifier.ransac import Ransac

    a = json.load(open(os.path.join(golden_dir, "argoverse_known_answer.json")))
    kp1 = _kp(np.stack([a["x1"], a["y1"]], 1).astype(np.float32))
    kp2 = _kp(np.stack([a["x2"], a["y2"]], 1).astype(np.float32))
    cal = geometry.Cal3Bundler(a["fx"], 0.0, 0.0, a["px"], a["py"])
    match = np.vstack([np.arange(20), np.arange(20)]).T
    v = Ransac(use_intrinsics_in_verification=True, estimation_threshold_px=a["estimation_threshold_px"])
    Rc, Uc, _, _ = v.verify(kp1, kp2, match, cal, cal)
    R = geometry.rotation_matrix(Rc)
    t = geometry.unit_vector(Uc)
    euler = Rotation.from_matrix(R.T).as_euler("zyx", degrees=True)
    np.testing.assert_allclose(euler, a["expected_euler_zyx_deg_i1Ri2"], atol=a["euler_tol_deg"])
    np.testing.assert_allclose(-R.T @ t, a["expected_i1ti2"], atol=a["translation_tol"])
    # 5 correspondences: the reference's failure path (opencv_verifier_base.py:77-78)
    r = v.verify(kp1, kp2, match[:5], cal, cal)
    assert r[0] is None and r[1] is None and r[2].size == 0 and r[3] == 0.0


def test_empty_matches(dev):
    from gtsfm_amd.common import geometry
    from gtsfm_amd.frontend.verifier.ransac import Ransac

    v = Ransac(use_intrinsics_in_verification=True, estimation_threshold_px=4)
    r = v.verify(_kp(np.zeros((10, 2))), _kp(np.zeros((10, 2))), np.zeros((0, 2), np.uint32),
                 geometry.Cal3Bundler(), geometry.Cal3Bundler())
    assert r[0] is None and r[2].dtype == np.uint64 and r[3] == 0.0


def test_batched_parity_with_oracle(dev, oracle_mod):
    """40 synthetic pairs with 30-70% inliers and 20..1500 putatives in one batched call vs the oracle."""
    from gtsfm_amd import device, native

    rng = np.random.default_rng(12)
    n_pairs = 40
    kps, Ks, gts, Ms = [], [], [], []
    for p in range(n_pairs):
        n_in = int(rng.integers(10, 700))
        n_out = int(n_in * rng.uniform(0.4, 1.5)) if p % 7 else 0
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, n_in, n_out)
        kps.append((kp1, kp2))
        Ks.append(K)
        gts.append((R, t))
        Ms.append(len(kp1))
    kmax = max(Ms)
    n_img = 2 * n_pairs
    kp = np.zeros((n_img, kmax, 2), np.float32)
    intr = np.zeros((n_img, 3))
    pairs = np.zeros((n_pairs, 2), np.int32)
    mi = np.zeros((n_pairs, kmax, 2), np.int32)
    for p, ((a, b), K) in enumerate(zip(kps, Ks)):
        kp[2 * p, : len(a)] = a
        kp[2 * p + 1, : len(b)] = b
        intr[2 * p] = intr[2 * p + 1] = (K[0, 0], K[0, 2], K[1, 2])
        pairs[p] = (2 * p, 2 * p + 1)
        mi[p, : Ms[p]] = np.arange(Ms[p])[:, None]
    res = device.ransac_essential(torch.from_numpy(kp).to(dev), torch.from_numpy(intr).to(dev),
                                  torch.from_numpy(pairs).to(dev), torch.from_numpy(mi).to(dev),
                                  torch.tensor(Ms, dtype=torch.int32, device=dev), 4.0)
    status = res.status.cpu().numpy()
    n_inl = res.n_inliers.cpu().numpy()
    R_all = res.R.cpu().numpy()
    t_all = res.t.cpu().numpy()
    mask = res.mask.cpu().numpy()
    n_hyp = res.n_hyp.cpu().numpy()
    for p in range(n_pairs):
        K = Ks[p]
        a, b = kps[p]
        x1 = (a.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        x2 = (b.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        ref = oracle_mod.ransac_E(x1, x2, 4.0 / K[0, 0], pair_id=p)
        assert status[p] == native.RANSAC_STATUS_OK, p
        _, rmask, rR, rt, rn, rh = ref
        # hypotheses evaluated: chunks of 64 with the bound re-evaluated per chunk, whatever chunks a launch covers
        assert int(n_hyp[p]) == rh, (p, n_hyp[p], rh)
        assert int(n_inl[p]) == rn, (p, n_inl[p], rn)
        np.testing.assert_array_equal(mask[p, : Ms[p]], rmask.astype(mask.dtype))
        np.testing.assert_array_equal(R_all[p], rR)
        np.testing.assert_array_equal(t_all[p], rt)
        if rn >= 50:  # estimator accuracy vs ground truth (only meaningful with enough support)
            assert scenes.rotation_angle_deg(R_all[p], gts[p][0]) < 2.0, p


def test_too_few_and_degenerate_in_batch(dev):
    from gtsfm_amd import device, native

    kp = np.zeros((2, 16, 2), np.float32)
    kp[0, :, 0] = np.arange(16)
    kp[1, :, 0] = np.arange(16)
    intr = np.array([[500.0, 0, 0], [500.0, 0, 0]])
    mi = np.zeros((2, 16, 2), np.int32)
    mi[:, :, 0] = mi[:, :, 1] = np.arange(16)
    res = device.ransac_essential(torch.from_numpy(kp).to(dev), torch.from_numpy(intr).to(dev),
                                  torch.tensor([[0, 1], [0, 1]], dtype=torch.int32, device=dev),
                                  torch.from_numpy(mi).to(dev), torch.tensor([5, 16], dtype=torch.int32, device=dev),
                                  4.0)
    st = res.status.cpu().numpy()
    assert st[0] == native.RANSAC_STATUS_TOO_FEW
    assert st[1] in (native.RANSAC_STATUS_OK, native.RANSAC_STATUS_NO_MODEL)  # collinear points: degenerate


@pytest.mark.gpu
def test_putatives_beyond_lds_staging(dev, oracle_mod):
    """A pair with more putatives than the score kernel stages in LDS (> 8704: points read from global memory), and a
    small pair in the same launch, against the oracle (same bar as the batched parity test)."""
    from gtsfm_amd import device, native

    rng = np.random.default_rng(31)
    kps, Ks, Ms = [], [], []
    for n_in, n_out in ((6000, 3500), (300, 200)):
        kp1, kp2, K, _, _, _ = scenes.random_two_view(rng, n_in, n_out)
        kps.append((kp1, kp2))
        Ks.append(K)
        Ms.append(len(kp1))
    kmax = max(Ms)
    assert kmax * 16 > 136 * 1024
    kp = np.zeros((4, kmax, 2), np.float32)
    intr = np.zeros((4, 3))
    mi = np.zeros((2, kmax, 2), np.int32)
    for p, ((a, b), K) in enumerate(zip(kps, Ks)):
        kp[2 * p, : len(a)] = a
        kp[2 * p + 1, : len(b)] = b
        intr[2 * p] = intr[2 * p + 1] = (K[0, 0], K[0, 2], K[1, 2])
        mi[p, : Ms[p]] = np.arange(Ms[p])[:, None]
    res = device.ransac_essential(torch.from_numpy(kp).to(dev), torch.from_numpy(intr).to(dev),
                                  torch.tensor([[0, 1], [2, 3]], dtype=torch.int32, device=dev),
                                  torch.from_numpy(mi).to(dev), torch.tensor(Ms, dtype=torch.int32, device=dev), 4.0)
    for p in range(2):
        K = Ks[p]
        a, b = kps[p]
        x1 = (a.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        x2 = (b.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        _, rmask, rR, rt, rn, rh = oracle_mod.ransac_E(x1, x2, 4.0 / K[0, 0], pair_id=p)
        assert int(res.status[p]) == native.RANSAC_STATUS_OK
        assert int(res.n_hyp[p]) == rh, (p, int(res.n_hyp[p]), rh)
        assert int(res.n_inliers[p]) == rn, (p, int(res.n_inliers[p]), rn)
        np.testing.assert_array_equal(res.mask[p, : Ms[p]].cpu().numpy(), rmask.astype(np.uint8))
        np.testing.assert_array_equal(res.R[p].cpu().numpy(), rR)
        np.testing.assert_array_equal(res.t[p].cpu().numpy(), rt)
