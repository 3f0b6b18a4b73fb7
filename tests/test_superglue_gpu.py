"""HIP SuperGlue (gtsfm_superglue_batched) against the reference module's own outputs.

Golden: tests/golden/superglue_random_w0.npz from tests/golden/make_superglue_golden.py (the reference's
thirdparty/.../superglue.py run in torch fp32 with seeded random weights, 20 Sinkhorn iterations). The HIP network
is exact-fp32 MFMA arithmetic in a different summation order (and an online softmax), so the log-assignment
matrix agrees within 2e-3 absolute after 18 layers + 20 Sinkhorn iterations, and the matches agree except where
two candidates are within that margin (>= 98 % of the reference's matches, no extra matches beyond 2 %).
"""
import os

import numpy as np
import pytest
import torch

from superpoint_weights import superglue_state_dict

pytestmark = pytest.mark.gpu
CASES = ["small_150x170", "mid_700x650", "c5_2048x2048"]


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "superglue_random_w0.npz"))


@pytest.fixture(scope="module")
def matcher():
    from gtsfm_amd import native
    from gtsfm_amd.frontend.matcher.superglue_matcher import SuperGlueMatcher

    native.require_gpu()
    return SuperGlueMatcher(state_dict=superglue_state_dict(0))


def _case(golden, name):
    from gtsfm_amd.common.keypoints import Keypoints

    g = lambda k: golden[f"{name}__{k}"]  # noqa: E731
    H, W = (int(x) for x in g("hw"))
    kp0 = Keypoints(g("kp0"), responses=g("s0"))
    kp1 = Keypoints(g("kp1"), responses=g("s1"))
    return kp0, kp1, g("d0"), g("d1"), (H, W, 1), g("matches0")


@pytest.mark.parametrize("name", CASES)
def test_matches_reference_module(matcher, golden, name):
    kp0, kp1, d0, d1, shape, m0 = _case(golden, name)
    got = matcher.match(kp0, kp1, d0, d1, shape, shape)
    ref = np.stack([np.flatnonzero(m0 >= 0), m0[m0 >= 0]], 1).astype(np.uint32)
    assert got.dtype == np.uint32 and got.ndim == 2 and got.shape[1] == 2
    assert np.all(np.diff(got[:, 0].astype(np.int64)) > 0)  # ascending i, one match per i
    a, b = set(map(tuple, got.tolist())), set(map(tuple, ref.tolist()))
    assert len(a & b) >= 0.98 * len(b) and len(a - b) <= 0.02 * max(len(b), 1), (len(a), len(b), len(a & b))


def test_batch_and_empty(matcher, golden):
    from gtsfm_amd.common.keypoints import Keypoints

    kp0, kp1, d0, d1, shape, _ = _case(golden, "small_150x170")
    kq0, kq1, e0, e1, shape2, _ = _case(golden, "mid_700x650")
    empty = Keypoints(np.zeros((0, 2), np.float32), responses=np.zeros(0, np.float32))
    out = matcher.match_batch([kp0, kp1, kq0, kq1, empty], [d0, d1, e0, e1, np.zeros((0, 256), np.float32)],
                              [shape, shape, shape2, shape2, shape], [(0, 1), (2, 3), (0, 4)])
    assert np.array_equal(out[(0, 1)], matcher.match(kp0, kp1, d0, d1, shape, shape))
    assert np.array_equal(out[(2, 3)], matcher.match(kq0, kq1, e0, e1, shape2, shape2))
    assert out[(0, 4)].shape == (0, 2) and out[(0, 4)].dtype == np.uint32
    with pytest.raises(ValueError):
        matcher.match(Keypoints(kp0.coordinates), kp1, d0, d1, shape, shape)


@pytest.mark.parametrize("name", CASES)
def test_matching_scores_close(matcher, golden, name):
    """matching_scores0 (exp of the mutual row maxima of the final log-assignment) within 2e-3 absolute."""
    from gtsfm_amd import device

    kp0, kp1, d0, d1, shape, m0 = _case(golden, name)
    n0, n1 = len(kp0), len(kp1)
    kmax = (max(n0, n1) + 63) // 64 * 64
    kp = np.zeros((2, kmax, 2), np.float32)
    sc = np.zeros((2, kmax), np.float32)
    de = np.zeros((2, kmax, 256), np.float32)
    kp[0, :n0], kp[1, :n1] = kp0.coordinates, kp1.coordinates
    sc[0, :n0], sc[1, :n1] = kp0.responses, kp1.responses
    de[0, :n0], de[1, :n1] = d0, d1
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    _, _, ms = device.superglue_match(t(kp), t(sc), t(de), t(np.array([n0, n1], np.int32)),
                                      t(np.array([shape[:2], shape[:2]], np.int32)), t(np.array([[0, 1]], np.int32)),
                                      matcher.weights())
    ref = golden[f"{name}__mscores0"]
    np.testing.assert_allclose(ms[0, :n0].cpu().numpy(), ref, atol=2e-3)


@pytest.mark.parametrize("name", ["small_150x170", "c5_2048x2048"])
def test_log_assignment_matrix(matcher, golden, name):
    """The final log-assignment matrix (log_optimal_transport's output, dustbins included) against the reference
    module's: the full (m+1) x (n+1) matrix for the small case, every 32nd row + the dustbin row at 2048 x 2048
    (BASELINE config C5's keypoint count). atol 2e-3 on entries above -20 (exp(-20) ~ 2e-9 of probability mass)."""
    from gtsfm_amd import device

    kp0, kp1, d0, d1, shape, _ = _case(golden, name)
    n0, n1 = len(kp0), len(kp1)
    kmax = (max(n0, n1) + 63) // 64 * 64
    kp = np.zeros((2, kmax, 2), np.float32)
    sc = np.zeros((2, kmax), np.float32)
    de = np.zeros((2, kmax, 256), np.float32)
    kp[0, :n0], kp[1, :n1] = kp0.coordinates, kp1.coordinates
    sc[0, :n0], sc[1, :n1] = kp0.responses, kp1.responses
    de[0, :n0], de[1, :n1] = d0, d1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    from gtsfm_amd import native

    ws = torch.empty(native.lib().gtsfm_superglue_workspace_bytes(1, kmax), dtype=torch.uint8, device="cuda")
    device.superglue_match(t(kp), t(sc), t(de), t(np.array([n0, n1], np.int32)),
                           t(np.array([shape[:2], shape[:2]], np.int32)), t(np.array([[0, 1]], np.int32)),
                           matcher.weights(), workspace=ws)
    Z = device.superglue_log_assignment(ws, 1, kmax, 0).cpu().numpy()[: n0 + 1, : n1 + 1]
    if f"{name}__Z" in golden.files:
        rows, ref = np.arange(n0 + 1), golden[f"{name}__Z"]
    else:
        rows, ref = golden[f"{name}__Z_rows"], golden[f"{name}__Z_sub"]
    got = Z[rows]
    assert ref.shape == got.shape and np.isfinite(got).all()
    live = ref > -20
    np.testing.assert_allclose(got[live], ref[live], atol=2e-3)
    assert (got[~live] < -15).all()


@pytest.mark.parametrize("name", CASES)
def test_matches_exact_up_to_near_ties(matcher, golden, name):
    """Every keypoint whose HIP match differs from the reference module's sits at a near-tie of the decision
    SuperGlue takes (superglue.py:270-283: row argmax, column argmax for the mutual check, exp(max) > threshold):
    measured on the HIP log-assignment itself, its row's top two, the involved columns' top two or its score against
    match_threshold are within 4e-3 (twice the log-assignment tolerance above). Everything else agrees exactly."""
    from gtsfm_amd import device, native

    kp0, kp1, d0, d1, shape, m0 = _case(golden, name)
    n0, n1 = len(kp0), len(kp1)
    kmax = (max(n0, n1) + 63) // 64 * 64
    kp = np.zeros((2, kmax, 2), np.float32)
    sc = np.zeros((2, kmax), np.float32)
    de = np.zeros((2, kmax, 256), np.float32)
    kp[0, :n0], kp[1, :n1] = kp0.coordinates, kp1.coordinates
    sc[0, :n0], sc[1, :n1] = kp0.responses, kp1.responses
    de[0, :n0], de[1, :n1] = d0, d1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ws = torch.empty(native.lib().gtsfm_superglue_workspace_bytes(1, kmax), dtype=torch.uint8, device="cuda")
    idx, cnt, _ = device.superglue_match(t(kp), t(sc), t(de), t(np.array([n0, n1], np.int32)),
                                         t(np.array([shape[:2], shape[:2]], np.int32)),
                                         t(np.array([[0, 1]], np.int32)), matcher.weights(), workspace=ws)
    Z = device.superglue_log_assignment(ws, 1, kmax, 0).cpu().numpy()[:n0, :n1].astype(np.float64)
    got = np.full(n0, -1, np.int64)
    pairs = idx[0, : int(cnt[0])].cpu().numpy().astype(np.int64)
    got[pairs[:, 0]] = pairs[:, 1]
    from gtsfm_amd.frontend.matcher.superglue_matcher import MATCH_THRESHOLD

    thr = float(MATCH_THRESHOLD)
    top2 = lambda v: np.sort(v)[-2:] if len(v) > 1 else np.array([-np.inf, v.max()])  # noqa: E731
    diff = np.flatnonzero(got != m0)
    assert len(diff) <= max(2, 0.02 * max(int((m0 >= 0).sum()), 1)), (len(diff), int((m0 >= 0).sum()))
    for i in diff:
        r2 = top2(Z[i])
        margins = [r2[1] - r2[0]]
        for j in {int(got[i]), int(m0[i]), int(np.argmax(Z[i]))} - {-1}:
            c2 = top2(Z[:, j])
            margins += [c2[1] - c2[0], abs(np.exp(Z[i, j]) - thr)]
        assert min(margins) < 4e-3, (name, int(i), int(got[i]), int(m0[i]), margins)


def test_fused_sinkhorn_equals_two_pass(matcher, golden, monkeypatch):
    """The one-pass Sinkhorn (sk_pass_kernel: row log-sum-exps and the columns' partials from one read of Z per
    iteration, merged by sk_vmerge_kernel) against the two-pass form (GTSFM_SG_SINKHORN_TWO_PASS=1): the column sums
    run in another order, so the log-assignment matrices agree to fp32 rounding (1e-4 absolute above -20 after 20
    iterations) and the matches are identical, at C5's 2048 x 2048 and on a batch with ragged counts."""
    from gtsfm_amd import device, native

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("GTSFM_SG_SINKHORN_TWO_PASS", mode)
        out = []
        for names in (["c5_2048x2048"], ["small_150x170", "mid_700x650"]):
            cs = [_case(golden, nm) for nm in names]
            kmax = (max(max(len(c[0]), len(c[1])) for c in cs) + 63) // 64 * 64
            P = len(cs)
            kp = np.zeros((2 * P, kmax, 2), np.float32)
            sc = np.zeros((2 * P, kmax), np.float32)
            de = np.zeros((2 * P, kmax, 256), np.float32)
            cnt, hw = [], []
            for q, (kp0, kp1, d0, d1, shape, _) in enumerate(cs):
                for s_, (k_, d_) in enumerate(((kp0, d0), (kp1, d1))):
                    n = len(k_)
                    kp[2 * q + s_, :n], sc[2 * q + s_, :n], de[2 * q + s_, :n] = k_.coordinates, k_.responses, d_
                    cnt.append(n)
                    hw.append(shape[:2])
            ws = torch.empty(native.lib().gtsfm_superglue_workspace_bytes(P, kmax), dtype=torch.uint8, device="cuda")
            idx, mc, _ = device.superglue_match(t(kp), t(sc), t(de), t(np.array(cnt, np.int32)),
                                                t(np.array(hw, np.int32)),
                                                t(np.array([[2 * q, 2 * q + 1] for q in range(P)], np.int32)),
                                                matcher.weights(), workspace=ws)
            for q in range(P):
                Z = device.superglue_log_assignment(ws, P, kmax, q).cpu().numpy()[: cnt[2 * q] + 1, : cnt[2 * q + 1] + 1]
                out.append((Z, idx[q, : int(mc[q])].cpu().numpy()))
        res[mode] = out
    for (za, ma), (zb, mb) in zip(res["0"], res["1"]):
        live = zb > -20
        np.testing.assert_allclose(za[live], zb[live], atol=1e-4)
        np.testing.assert_array_equal(ma, mb)


@pytest.mark.parametrize("mode", ["2", "3", "4"])
def test_dma_staged_gemm_bit_identical(matcher, golden, monkeypatch, mode):
    """The weight GEMMs staged by LDS-DMA (sg_gemm3d_kernel: 128-row tiles with 2 or 3 chunks in flight, or 256-row
    tiles; GTSFM_SG_GEMM_DMA) split A on
    the fragment read with the staged kernel's split3x8 and run the same MFMA sequence, so the whole network's output
    (log-assignment, matches, scores) is identical bit for bit to the register-staged kernel (GTSFM_SG_GEMM_DMA=0), on
    C5's 2048 x 2048 and on a ragged pair."""
    from gtsfm_amd import device, native

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    res = {}
    for m in ("0", mode):
        monkeypatch.setenv("GTSFM_SG_GEMM_DMA", m)
        out = []
        for name in ("c5_2048x2048", "mid_700x650"):
            kp0, kp1, d0, d1, shape, _ = _case(golden, name)
            n0, n1 = len(kp0), len(kp1)
            kmax = (max(n0, n1) + 63) // 64 * 64
            kp = np.zeros((2, kmax, 2), np.float32)
            sc = np.zeros((2, kmax), np.float32)
            de = np.zeros((2, kmax, 256), np.float32)
            kp[0, :n0], kp[1, :n1] = kp0.coordinates, kp1.coordinates
            sc[0, :n0], sc[1, :n1] = kp0.responses, kp1.responses
            de[0, :n0], de[1, :n1] = d0, d1
            ws = torch.empty(native.lib().gtsfm_superglue_workspace_bytes(1, kmax), dtype=torch.uint8, device="cuda")
            idx, cnt, ms = device.superglue_match(t(kp), t(sc), t(de), t(np.array([n0, n1], np.int32)),
                                                  t(np.array([shape[:2], shape[:2]], np.int32)),
                                                  t(np.array([[0, 1]], np.int32)), matcher.weights(), workspace=ws)
            Z = device.superglue_log_assignment(ws, 1, kmax, 0).cpu().numpy()[: n0 + 1, : n1 + 1]
            out.append((Z, idx[0, : int(cnt[0])].cpu().numpy(), ms[0, :n0].cpu().numpy()))
        res[m] = out
    for a, b in zip(res["0"], res[mode]):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
