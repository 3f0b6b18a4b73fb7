"""GPU parity of the HIP matcher (libgtsfm_hip.so via the C ABI) against the oracle and the reference's answers.

Bar: bit-exact match indices and order. Cases mirror the reference's matcher tests
(tests/frontend/matcher/test_matcher_base.py: empty input, index validity, one-to-one; the two known-answer tests)
plus ragged batches, NaN rows, ties, partial tiles and the 5000-keypoint Lund-door fixture.
"""
import json
import os

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


def _sift_like(rng, n, dim=128):
    """Integer descriptors with L2 norm ~512 (OpenCV SIFT normalisation), as uint8-valued float32."""
    x = rng.gamma(0.6, 1.0, size=(n, dim))
    x = x / np.linalg.norm(x, axis=1, keepdims=True) * 512.0
    return np.clip(np.round(x), 0, 255).astype(np.float32)


def _planted_pair(rng, n1, n2, frac=0.3, noise=8, dim=128):
    a = _sift_like(rng, n1, dim)
    b = _sift_like(rng, n2, dim)
    k = int(frac * min(n1, n2))
    src = rng.permutation(n1)[:k]
    dst = rng.permutation(n2)[:k]
    b[dst] = np.clip(a[src] + rng.integers(-noise, noise + 1, size=(k, dim)), 0, 255)
    return a, b


def test_known_answers(dev, golden_dir):
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher

    ka = json.load(open(os.path.join(golden_dir, "twoway_known_answers.json")))
    d1 = np.array(ka["descriptors_i1"], np.float32).reshape(-1, 1)
    d2 = np.array(ka["descriptors_i2"], np.float32).reshape(-1, 1)
    r = TwoWayMatcher(ratio_test_threshold=0.8).match(None, None, d1, d2, (300, 100), (300, 100))
    np.testing.assert_array_equal(r, np.array(ka["expected_ratio_0.8"]))
    assert r.dtype == np.uint32
    r = TwoWayMatcher().match(None, None, d1, d2, (300, 100), (300, 100))
    np.testing.assert_array_equal(r, np.array(ka["expected_no_ratio"]))


@pytest.mark.parametrize("ratio", [0.8, None])
def test_lund_door_full_int_path_bit_exact(dev, golden_dir, ratio):
    from gtsfm_amd import native
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher, select_match_mode

    z = np.load(os.path.join(golden_dir, "lund_door_descriptors.npz"))
    g = np.load(os.path.join(golden_dir, "lund_door_matches_oracle.npz"))
    d0 = z["d0"].astype(np.float32)
    d1 = z["d1"].astype(np.float32)
    assert select_match_mode(d0, d1) == native.GTSFM_MATCH_INT_F16
    r = TwoWayMatcher(ratio_test_threshold=ratio).match(None, None, d0, d1, None, None)
    np.testing.assert_array_equal(r, g["full_ratio_0_8" if ratio else "full_no_ratio"])


def test_exact_path_float_descriptors_vs_oracle(dev, oracle_mod):
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(7)
    a = rng.normal(size=(700, 32)).astype(np.float32)
    b = np.concatenate([a[:300] + 0.05 * rng.normal(size=(300, 32)), rng.normal(size=(500, 32))]).astype(np.float32)
    for ratio in (0.8, None):
        np.testing.assert_array_equal(match_descriptor_pair(a, b, ratio), oracle_mod.twoway_match(a, b, ratio))


@pytest.mark.parametrize("n1,n2", [(2048, 2048), (1999, 2048), (37, 1500), (2048, 33), (257, 255), (1, 5)])
def test_int_path_shapes_vs_oracle(dev, oracle_mod, n1, n2):
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(n1 * 7 + n2)
    a, b = _planted_pair(rng, n1, n2)
    np.testing.assert_array_equal(match_descriptor_pair(a, b, 0.8), oracle_mod.twoway_match(a, b, 0.8))


def test_ties_take_lowest_index(dev, oracle_mod):
    """Duplicated train descriptors: OpenCV keeps the lowest train index first (strict '<' scan)."""
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(11)
    a = _sift_like(rng, 300)
    b = np.concatenate([a[:100], a[:100], _sift_like(rng, 100)])
    for ratio in (None, 0.8):
        np.testing.assert_array_equal(match_descriptor_pair(a, b, ratio), oracle_mod.twoway_match(a, b, ratio))


def test_ties_on_both_sides(dev, oracle_mod):
    """Duplicates in both images (zero distances, tied minima on the query and the train side): the kernel keeps
    value-only top-2s for image i2, so tied i2 keypoints go through the exact recomputation in finalize."""
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(13)
    base = _sift_like(rng, 150)
    a = np.concatenate([base[:60], base[:60], _sift_like(rng, 200), base[60:90]])
    b = np.concatenate([base[:90], base[30:60], _sift_like(rng, 90), base[:20]])
    for ratio in (None, 0.8, 1.0):
        np.testing.assert_array_equal(match_descriptor_pair(a, b, ratio), oracle_mod.twoway_match(a, b, ratio))
        np.testing.assert_array_equal(match_descriptor_pair(b, a, ratio), oracle_mod.twoway_match(b, a, ratio))


def test_nan_rows_and_empty(dev, oracle_mod):
    from gtsfm_amd.frontend.matcher.twoway_matcher import TwoWayMatcher

    rng = np.random.default_rng(5)
    a, b = _planted_pair(rng, 400, 380)
    a[[3, 50, 399]] = np.nan
    m = TwoWayMatcher(ratio_test_threshold=0.8)
    r = m.match(None, None, a, b, None, None)
    keep = np.array([i for i in range(400) if i not in (3, 50, 399)])
    ref = oracle_mod.twoway_match(a[keep], b, 0.8)
    ref[:, 0] = keep[ref[:, 0]]
    np.testing.assert_array_equal(r, ref)
    assert m.match(None, None, np.zeros((0, 128), np.float32), b, None, None).size == 0


def test_batched_ragged_pairs_vs_oracle(dev, oracle_mod):
    """All pairs of 6 images with ragged keypoint counts in one batched call."""
    from gtsfm_amd import device, native

    rng = np.random.default_rng(21)
    counts = [2048, 1700, 513, 2048, 64, 1999]
    kmax = max(counts)
    descs = [_sift_like(rng, n) for n in counts]
    for i in range(1, len(counts)):  # plant shared structure
        k = min(counts[i], counts[0]) // 3
        descs[i][:k] = np.clip(descs[0][:k] + rng.integers(-6, 7, size=(k, 128)), 0, 255)
    host = np.zeros((len(counts), kmax, 128), np.float32)
    for i, d in enumerate(descs):
        host[i, : len(d)] = d
    pairs = [(i, j) for i in range(len(counts)) for j in range(i + 1, len(counts))]
    idx, cnt = device.match_pairs(torch.from_numpy(host).to(dev), torch.tensor(counts, dtype=torch.int32, device=dev),
                                  torch.tensor(pairs, dtype=torch.int32, device=dev), 0.8, native.GTSFM_MATCH_INT_F16)
    idx = idx.cpu().numpy().view(np.uint32)
    cnt = cnt.cpu().numpy()
    for p, (i, j) in enumerate(pairs):
        ref = oracle_mod.twoway_match(descs[i], descs[j], 0.8)
        np.testing.assert_array_equal(idx[p, : cnt[p]], ref, err_msg=f"pair {(i, j)}")


def test_mfma_distance_is_exact_integer(dev, oracle_mod):
    """Intermediate check: the MFMA row top-2 distances equal the oracle's exact distances."""
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(2)
    a = np.zeros((64, 128), np.float32)
    a[np.arange(64), np.arange(64)] = 255.0  # asymmetric, exact integer operands
    b = a[::-1].copy()
    b[:, 100] = np.arange(64, dtype=np.float32)
    np.testing.assert_array_equal(match_descriptor_pair(a, b, None), oracle_mod.twoway_match(a, b, None))


def _batch(dev, descs):
    counts = [len(d) for d in descs]
    kmax = max(counts)
    host = np.zeros((len(descs), kmax, descs[0].shape[1]), np.float32)
    for i, d in enumerate(descs):
        host[i, : len(d)] = d
    return torch.from_numpy(host).to(dev), torch.tensor(counts, dtype=torch.int32, device=dev)


def test_grouped_workgroups_vs_oracle(dev, oracle_mod):
    """The distance GEMM with several pairs per workgroup (gtsfm_match_batched_grouped): block-tiled groups from
    pair_groups, and hand-made groups whose pairs do NOT share image i1 (the A-fragment reload path), both equal the
    oracle pair for pair; so does a group list in reverse order with empty slots."""
    from gtsfm_amd import device, native

    rng = np.random.default_rng(31)
    counts = [2048, 1300, 2048, 700, 1999, 2048, 513, 1024, 1]
    descs = [_sift_like(rng, n) for n in counts]
    for i in range(1, len(counts)):
        k = min(counts[i], counts[0]) // 3
        descs[i][:k] = np.clip(descs[0][:k] + rng.integers(-6, 7, size=(k, 128)), 0, 255)
    d, c = _batch(dev, descs)
    pairs = np.array([(i, j) for i in range(len(counts)) for j in range(i + 1, len(counts))], np.int32)
    G = device.match_group_size(max(counts), 128)
    assert G >= 2
    tiled = device.pair_groups(pairs, G)
    mixed = np.full((-(-len(pairs) // G), G), -1, np.int32)
    mixed.flat[: len(pairs)] = np.arange(len(pairs))[::-1]
    pt = torch.from_numpy(pairs).to(dev)
    refs = [oracle_mod.twoway_match(descs[i], descs[j], 0.8) for i, j in pairs]
    for groups in (tiled, mixed):
        idx, cnt = device.match_pairs(d, c, pt, 0.8, native.GTSFM_MATCH_INT_F16,
                                      groups=torch.from_numpy(groups).to(dev))
        idx = idx.cpu().numpy().view(np.uint32)
        cnt = cnt.cpu().numpy()
        for p in range(len(pairs)):
            np.testing.assert_array_equal(idx[p, : cnt[p]], refs[p], err_msg=f"pair {tuple(pairs[p])}")


@pytest.mark.parametrize("split", ["1", "2", "4"])
def test_pass_split_vs_oracle(dev, oracle_mod, monkeypatch, split):
    """A group's 512-row passes cut over 1, 2 or 4 workgroups (the split the library picks when a launch has too few
    groups to fill the CUs, forced here through GTSFM_MATCH_PASS_SPLIT): rows per pass, columns folded into colres
    by global atomics. Ragged counts leave some splits with no rows of a pair; every pair equals the oracle."""
    from gtsfm_amd import device, native

    monkeypatch.setenv("GTSFM_MATCH_PASS_SPLIT", split)
    rng = np.random.default_rng(47)
    counts = [2048, 1300, 2048, 700, 1999, 513, 1537, 1]
    descs = [_sift_like(rng, n) for n in counts]
    for i in range(1, len(counts)):
        k = min(counts[i], counts[0]) // 3
        descs[i][:k] = np.clip(descs[0][:k] + rng.integers(-6, 7, size=(k, 128)), 0, 255)
    d, c = _batch(dev, descs)
    pairs = np.array([(i, j) for i in range(len(counts)) for j in range(len(counts)) if i != j], np.int32)
    pt = torch.from_numpy(pairs).to(dev)
    refs = [oracle_mod.twoway_match(descs[i], descs[j], 0.8) for i, j in pairs]
    G = device.match_group_size(max(counts), 128)
    for groups in (None, torch.from_numpy(device.pair_groups(pairs, G)).to(dev)):
        idx, cnt = device.match_pairs(d, c, pt, 0.8, native.GTSFM_MATCH_INT_F16, groups=groups)
        idx = idx.cpu().numpy().view(np.uint32)
        cnt = cnt.cpu().numpy()
        for p in range(len(pairs)):
            np.testing.assert_array_equal(idx[p, : cnt[p]], refs[p], err_msg=f"pair {tuple(pairs[p])}")


def test_contract_edge_norms_exact(dev, oracle_mod):
    """Descriptors at the INT_F16 contract's edge (values up to 1023, squared norms just under 2^19): the folded
    accumulator d2 + code/16 stays exact, so the matches equal the oracle's."""
    from gtsfm_amd.frontend.matcher.twoway_matcher import match_descriptor_pair

    rng = np.random.default_rng(41)
    n, dim = 600, 128
    a = np.zeros((n, dim), np.float32)
    a[:, 0] = 724.0                                   # 724^2 = 524176 < 2^19
    a[:, 1:4] = rng.integers(0, 6, size=(n, 3))       # small spread keeps |a|^2 < 2^19
    b = np.zeros((n, dim), np.float32)
    b[:, 1] = 724.0                                   # orthogonal to a: d2 ~ 2^20 - small
    b[:, 2:5] = rng.integers(0, 6, size=(n, 3))
    b[:200] = a[:200] + rng.integers(0, 2, size=(200, dim)) * (np.arange(dim) > 100)
    assert (np.sum(a.astype(np.float64) ** 2, 1) < 2 ** 19).all() and (np.sum(b.astype(np.float64) ** 2, 1) < 2 ** 19).all()
    for ratio in (0.8, None):
        np.testing.assert_array_equal(match_descriptor_pair(a, b, ratio), oracle_mod.twoway_match(a, b, ratio))
        np.testing.assert_array_equal(match_descriptor_pair(b, a, ratio), oracle_mod.twoway_match(b, a, ratio))
