"""The verifier oracle (oracle/ransac.c) against the reference's known-answer verifier tests.

- two-plane scene (tests/frontend/verifier/test_verifier_base.py:81-100, simulate_two_planes_scene): all 8 putatives
  verified, rotation and direction within 2 degrees (:24-25);
- Argoverse hand-labelled pair (tests/frontend/verifier/test_verifier_argoverse.py:73-118): Euler zyx of i1Ri2 within
  1 degree of [-0.37, 32.47, -0.42], i1ti2 within 0.01 of [0.21, -0.0024, 0.976];
- recoverPose on the 10+10 two-plane scene (tests/utils/test_verification_utils.py:17-29): equal within 1e-3.
"""
import json
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from tests import scenes


def _argoverse(golden_dir):
    a = json.load(open(os.path.join(golden_dir, "argoverse_known_answer.json")))
    kp1 = np.stack([a["x1"], a["y1"]], 1).astype(np.float32).astype(np.float64)
    kp2 = np.stack([a["x2"], a["y2"]], 1).astype(np.float32).astype(np.float64)
    pp = np.array([a["px"], a["py"]])
    return a, (kp1 - pp) / a["fx"], (kp2 - pp) / a["fx"]


@pytest.mark.parametrize("scoring", [0, 1])
def test_two_plane_scene(oracle_mod, scoring):
    uv1, uv2, R, t = scenes.two_planes_scene(4, 4)
    E, mask, Re, te, n, _ = oracle_mod.ransac_E(uv1, uv2, 0.5, scoring=scoring)
    assert n == 8 and mask.all()
    assert scenes.rotation_angle_deg(R, Re) < 2 and scenes.direction_angle_deg(t, te) < 2


@pytest.mark.parametrize("scoring", [0, 1])
def test_argoverse_known_answer(oracle_mod, golden_dir, scoring):
    a, x1, x2 = _argoverse(golden_dir)
    E, mask, R, t, n, _ = oracle_mod.ransac_E(x1, x2, a["estimation_threshold_px"] / a["fx"], scoring=scoring)
    euler = Rotation.from_matrix(R.T).as_euler("zyx", degrees=True)
    np.testing.assert_allclose(euler, a["expected_euler_zyx_deg_i1Ri2"], atol=a["euler_tol_deg"])
    np.testing.assert_allclose(-R.T @ t, a["expected_i1ti2"], atol=a["translation_tol"])


def test_recover_pose_two_plane_10_10(oracle_mod):
    uv1, uv2, R, t = scenes.two_planes_scene(10, 10)
    E = scenes.skew(t) @ R
    Re, te, _ = oracle_mod.recover_pose(E, uv1, uv2)
    np.testing.assert_allclose(Re, R, atol=1e-3)
    np.testing.assert_allclose(te, t, atol=1e-3)


def test_five_point_solutions_satisfy_constraints(oracle_mod):
    rng = np.random.default_rng(1)
    for _ in range(20):
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 5, 0, noise_px=0.0)
        x1 = (kp1 - K[:2, 2]) / K[0, 0]
        x2 = (kp2 - K[:2, 2]) / K[0, 0]
        Es = oracle_mod.five_point(x1, x2)
        assert len(Es) >= 1
        Egt = scenes.skew(t) @ R
        Egt /= np.linalg.norm(Egt)
        h1 = np.c_[x1, np.ones(5)]
        h2 = np.c_[x2, np.ones(5)]
        best = min(min(np.linalg.norm(E - Egt), np.linalg.norm(E + Egt)) for E in Es)
        assert best < 1e-6
        for E in Es:
            assert np.abs(np.sum(h2 * (h1 @ E.T), 1)).max() < 1e-9
            assert abs(np.linalg.det(E)) < 1e-6


@pytest.mark.parametrize("scoring", [0, 1])
def test_synthetic_scenes_pose_accuracy(oracle_mod, scoring):
    rng = np.random.default_rng(0)
    for _ in range(8):
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 300, 300)
        x1 = (kp1 - K[:2, 2]) / K[0, 0]
        x2 = (kp2 - K[:2, 2]) / K[0, 0]
        E, mask, Re, te, n, nh = oracle_mod.ransac_E(x1, x2, 4.0 / K[0, 0], scoring=scoring)
        assert scenes.rotation_angle_deg(R, Re) < 1.5
        assert scenes.direction_angle_deg(t, te) < 8
        assert (mask.astype(bool) & inl).sum() >= 0.95 * inl.sum()


def test_too_few_correspondences(oracle_mod):
    assert oracle_mod.ransac_E(np.zeros((5, 2)), np.zeros((5, 2)), 0.01) is None


# ---------------------------------------------------------------- fundamental-matrix path (oracle/fundamental.c)
def test_F_two_plane_scene(oracle_mod):
    """tests/frontend/verifier/test_ransac.py:22-30 (TestRansacForFundamentalMatrix) on the same two-plane scene:
    8 putatives -> the LMedS branch; all verified, R and t within 2 deg."""
    uv1, uv2, R, t = scenes.two_planes_scene(4, 4)
    Re, te, mask, n = oracle_mod.verify_F(uv1, uv2, np.eye(3), np.eye(3), 0.5)
    assert n == 8 and mask.all()
    assert scenes.rotation_angle_deg(R, Re) < 2 and scenes.direction_angle_deg(t, te) < 2


def test_F_seven_point_solutions(oracle_mod):
    rng = np.random.default_rng(3)
    for _ in range(20):
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 7, 0, noise_px=0.0)
        Fs = oracle_mod.seven_point(kp1, kp2)
        assert 1 <= len(Fs) <= 3
        Kinv = np.linalg.inv(K)
        Fgt = Kinv.T @ scenes.skew(t) @ R @ Kinv
        Fgt /= Fgt[2, 2]
        h1, h2 = np.c_[kp1, np.ones(7)], np.c_[kp2, np.ones(7)]
        for F in Fs:
            assert F[2, 2] == 1.0
            assert np.abs(oracle_mod.f_errors(F, kp1, kp2)).max() < 1e-6
            assert abs(np.linalg.det(F / np.linalg.norm(F))) < 1e-9
        # the true F is one of the roots
        assert min(np.linalg.norm(F - Fgt) / np.linalg.norm(Fgt) for F in Fs) < 1e-5


def test_F_synthetic_scenes_pose_accuracy(oracle_mod):
    rng = np.random.default_rng(5)
    for _ in range(6):
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 300, 200)
        r = oracle_mod.verify_F(kp1, kp2, K, K, 4.0, max_iters=100000)
        assert r is not None
        Re, te, mask, n = r
        assert (mask.astype(bool) & inl).sum() >= 0.9 * inl.sum()
        assert scenes.rotation_angle_deg(R, Re) < 3.0
        assert scenes.direction_angle_deg(t, te) < 10.0


def test_F_lmeds_branch_and_guards(oracle_mod):
    rng = np.random.default_rng(9)
    kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 12, 0, noise_px=0.0)
    F, mask, n, nh = oracle_mod.ransac_F(kp1, kp2, 1.0)
    assert n == 12 and mask.all() and nh >= 64  # M < 15: LMedS with its fixed iteration count
    assert oracle_mod.ransac_F(kp1[:7], kp2[:7], 1.0) is None  # M < 8


def _msac_score_np(E, x1, x2, thr):
    """numpy restatement of the oracle's quantised MSAC score (float32 terms, fma emulated in float64 then rounded)."""
    f = np.float32
    Ef = E.astype(f).ravel()
    p = [x1[:, 0].astype(f), x1[:, 1].astype(f), x2[:, 0].astype(f), x2[:, 1].astype(f)]

    def fma(a, b, c):
        return (a.astype(np.float64) * b + c).astype(f)

    a0 = fma(Ef[1], p[1], fma(Ef[0], p[0], np.full_like(p[0], Ef[2])))
    a1 = fma(Ef[4], p[1], fma(Ef[3], p[0], np.full_like(p[0], Ef[5])))
    a2 = fma(Ef[7], p[1], fma(Ef[6], p[0], np.full_like(p[0], Ef[8])))
    b0 = fma(Ef[3], p[3], fma(Ef[0], p[2], np.full_like(p[0], Ef[6])))
    b1 = fma(Ef[4], p[3], fma(Ef[1], p[2], np.full_like(p[0], Ef[7])))
    num = fma(p[3], a1, fma(p[2], a0, a2))
    den = fma(b1, b1, fma(b0, b0, fma(a1, a1, a0 * a0)))
    thr2 = f(thr * thr)
    nn = num * num
    inl = nn <= thr2 * den
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(den > 0, nn / den, f(0))
    q = r * (f(65536) / thr2)
    cost = np.where(inl, np.where(q < 65535, np.floor(q), 65535), 65536).astype(np.int64)
    return int(cost.sum()), inl


def test_msac_selects_lower_truncated_cost(oracle_mod):
    """MSAC's final model scores no worse than RANSAC's under the MSAC objective, and its mask is that model's inlier
    set; both modes agree on clean data."""
    rng = np.random.default_rng(5)
    wins = 0
    for _ in range(6):
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, 200, 200, noise_px=1.5)
        x1 = (kp1 - K[:2, 2]) / K[0, 0]
        x2 = (kp2 - K[:2, 2]) / K[0, 0]
        thr = 4.0 / K[0, 0]
        Em, mm, *_ = oracle_mod.ransac_E(x1, x2, thr, scoring=1)
        Er, mr, *_ = oracle_mod.ransac_E(x1, x2, thr, scoring=0)
        sm, im = _msac_score_np(Em, x1, x2, thr)
        sr, _ = _msac_score_np(Er, x1, x2, thr)
        assert np.array_equal(im, mm.astype(bool))
        wins += sm <= sr
    assert wins >= 5


def test_oracle_pinned_to_round2_oracle_on_lund_c1(oracle_mod):
    """The E-path oracle vs its round-2 version (tests/golden/make_prev_oracle_c1.py: Gauss-Jordan null space, Jacobi
    LO, compiler-placed FMAs), which nothing of the kernel shaped: on all 66 C1 pairs the stored results agree (equal
    inlier counts and masks, R and t within 2e-3 deg), and the current oracle recomputes three of them from its own
    SIFT + matcher."""
    from tests.test_lund_door_c1_gpu import LUND, _images

    cur = np.load(os.path.join(LUND, "oracle_c1.npz"))
    prev = np.load(os.path.join(LUND, "oracle_c1_prev.npz"))
    np.testing.assert_array_equal(prev["pairs"], cur["pairs"])
    np.testing.assert_array_equal(prev["match_count"], cur["match_count"])
    np.testing.assert_array_equal(prev["status"], cur["status"])
    np.testing.assert_array_equal(prev["n_inliers"], cur["n_inliers"])
    masks = np.unpackbits(prev["masks"])[: len(cur["masks"])]
    np.testing.assert_array_equal(masks, cur["masks"])

    def close(R, t, p):
        dR = np.rad2deg(np.linalg.norm(Rotation.from_matrix(R @ prev["R"][p].T).as_rotvec()))
        dt = scenes.direction_angle_deg(t, prev["t"][p])
        assert dR < 2e-3 and dt < 2e-3, (p, dR, dt)

    for p in range(len(cur["pairs"])):
        close(cur["R"][p], cur["t"][p], p)
    gt, imgs = _images()
    f, u0, v0 = gt["fx_u0_v0"]
    kps = [oracle_mod.sift(oracle_mod.rgb_to_gray(imgs[i]), 5000)[:2] for i in range(3)]
    off = np.concatenate([[0], np.cumsum(cur["match_count"])])
    pairs = [tuple(map(int, q)) for q in cur["pairs"]]
    for i1, i2 in ((0, 1), (0, 2), (1, 2)):
        p = pairs.index((i1, i2))
        m = oracle_mod.twoway_match(kps[i1][1], kps[i2][1], 0.8).reshape(-1, 2).astype(np.int64)
        np.testing.assert_array_equal(m, cur["matches"][off[p]: off[p + 1]])
        x1 = (kps[i1][0][m[:, 0], :2].astype(np.float64) - [u0, v0]) / f
        x2 = (kps[i2][0][m[:, 1], :2].astype(np.float64) - [u0, v0]) / f
        _, mask, R, t, n, _ = oracle_mod.ransac_E(x1, x2, 4.0 / f, pair_id=0)
        assert n == prev["n_inliers"][p]
        np.testing.assert_array_equal(mask, masks[off[p]: off[p + 1]])
        close(R, t, p)


def _gc_energy(q, key, lab, lam):
    """2 * E(L) * den of the graph-cut LO (oracle/ransac.c gc_label) by its definition, summed over pairs."""
    Q = 65536
    num, den = lam
    U = sum(2 * qi if li else 2 * (Q - qi) for qi, li in zip(q, lab))
    P = 0
    for i in range(len(q)):
        for j in range(i + 1, len(q)):
            if key[i] != key[j]:
                continue
            if lab[i] and lab[j]:
                P += q[i] + q[j]
            elif not lab[i] and not lab[j]:
                P += 2 * Q - q[i] - q[j]
            else:
                P += 2 * Q
    return (den - num) * U + num * P


@pytest.mark.parametrize("lam", [(39, 40), (1, 2), (7, 50), (0, 1)])
def test_gc_label_is_the_exact_min_cut(oracle_mod, lam):
    """The per-cell closed form of the graph-cut labelling equals the exhaustive minimum of its energy over every
    labelling of small random cells (the minimal inlier set on ties), so any exact min-cut agrees with it."""
    import itertools

    rng = np.random.default_rng(int(lam[0]) * 7 + 1)
    for trial in range(40):
        k = int(rng.integers(1, 9))
        q = rng.choice([0, 1, 500, 20000, 32768, 40000, 65535, 65536], size=k).astype(np.int64)
        q = np.where(rng.random(k) < 0.5, rng.integers(0, 65537, size=k), q)
        key = rng.integers(0, 3, size=k)
        got = oracle_mod.gc_label_q(q, key, lam)
        best = min(_gc_energy(q, key, lab, lam) for lab in itertools.product([0, 1], repeat=k))
        assert _gc_energy(q, key, got, lam) == best, (trial, q, key, got)
        # minimal: no optimal labelling has fewer inliers in any cell
        for c in np.unique(key):
            cells = [lab for lab in itertools.product([0, 1], repeat=k) if _gc_energy(q, key, lab, lam) == best]
            assert min(sum(l for l, kk in zip(lab, key) if kk == c) for lab in cells) == got[key == c].sum()


def test_gc_lo_stage_on_known_answers(oracle_mod):
    """The graph-cut LO stage (GC-RANSAC's local optimisation, after or instead of the iterative LO) keeps the
    two-plane scene's known answer: every putative verified, R and t within 2 degrees."""
    uv1, uv2, R, t = scenes.two_planes_scene(4, 4)
    for gc_iters in (10, -10):
        E, mask, Re, te, n, _ = oracle_mod.ransac_E_gc(uv1, uv2, 0.5, gc_iters, 0.2)
        assert n == len(uv1)
        assert scenes.rotation_angle_deg(Re, R) < 2.0
        assert scenes.direction_angle_deg(te, t) < 2.0
