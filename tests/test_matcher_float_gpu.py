"""GTSFM_MATCH_F16_RERANK (fp16 MFMA shortlist + certified exact fp32 re-rank) for float descriptors.

Bar: the matches (indices and their order) are identical to GTSFM_MATCH_EXACT_F32 and to the oracle's TwoWayMatcher
restatement (oracle/twoway.c) on the same inputs, whatever the descriptors: SuperPoint-like unit vectors with planted
matches, dims that are not multiples of 16, exact ties and duplicate rows, keypoint counts below the shortlist size,
values outside the fp16 range (exact rescan), and near-equidistant clusters (certificate fails -> exact rescan).
"""
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


def _unit(rng, n, dim):
    x = rng.normal(size=(n, dim))
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def _planted(rng, n1, n2, dim=256, frac=0.3, noise=0.15):
    a, b = _unit(rng, n1, dim), _unit(rng, n2, dim)
    k = int(frac * min(n1, n2))
    src, dst = rng.permutation(n1)[:k], rng.permutation(n2)[:k]
    y = a[src] + noise * rng.normal(size=(k, dim)) / np.sqrt(dim)
    b[dst] = (y / np.linalg.norm(y, axis=1, keepdims=True)).astype(np.float32)
    return a, b


def _run(dev, descs, pairs, ratio, mode):
    from gtsfm_amd import device

    kmax = max(len(d) for d in descs)
    dim = descs[0].shape[1]
    arr = np.zeros((len(descs), kmax, dim), np.float32)
    for i, d in enumerate(descs):
        arr[i, : len(d)] = d
    cnt = torch.tensor([len(d) for d in descs], dtype=torch.int32, device=dev)
    idx, m = device.match_pairs(torch.from_numpy(arr).to(dev), cnt,
                                torch.tensor(pairs, dtype=torch.int32, device=dev), ratio, mode)
    m = m.cpu().numpy()
    idx = idx.cpu().numpy().view(np.uint32)
    return [idx[p, : m[p]].copy() for p in range(len(pairs))]


def _check(dev, oracle_mod, descs, pairs, ratio, n_oracle=2):
    from gtsfm_amd import native

    fast = _run(dev, descs, pairs, ratio, native.GTSFM_MATCH_F16_RERANK)
    exact = _run(dev, descs, pairs, ratio, native.GTSFM_MATCH_EXACT_F32)
    for p, (f, e) in enumerate(zip(fast, exact)):
        np.testing.assert_array_equal(f, e, err_msg=f"pair {pairs[p]}")
    for p in range(min(n_oracle, len(pairs))):
        i1, i2 = pairs[p]
        ref = oracle_mod.twoway_match(descs[i1], descs[i2], ratio).reshape(-1, 2)
        np.testing.assert_array_equal(fast[p].reshape(-1, 2), ref, err_msg=f"oracle pair {pairs[p]}")
    return fast


@pytest.mark.parametrize("ratio", [0.8, None])
def test_superpoint_like_batch(dev, oracle_mod, ratio):
    rng = np.random.default_rng(31)
    sizes = [1000, 1200, 777, 1024, 64, 3]
    base = _unit(rng, 1200, 256)
    descs = []
    for s in sizes:  # views share a latent set: planted matches between every pair
        d = _unit(rng, s, 256)
        k = s // 3
        y = base[rng.permutation(1200)[:k]] + 0.15 * rng.normal(size=(k, 256)) / 16
        d[rng.permutation(s)[:k]] = y / np.linalg.norm(y, axis=1, keepdims=True)
        descs.append(d)
    pairs = [(i, j) for i in range(len(sizes)) for j in range(i + 1, len(sizes))]
    out = _check(dev, oracle_mod, descs, pairs, ratio, n_oracle=3)
    assert len(out[0]) > 100  # the planted matches are found


@pytest.mark.parametrize("dim", [16, 64, 100, 128, 200, 256, 300])
def test_dims(dev, oracle_mod, dim):
    rng = np.random.default_rng(dim)
    a, b = _planted(rng, 500, 600, dim)
    _check(dev, oracle_mod, [a, b], [(0, 1), (1, 0)], 0.8)


def test_ties_and_duplicate_rows(dev, oracle_mod):
    rng = np.random.default_rng(3)
    a, b = _planted(rng, 400, 400, 256)
    b[10:20] = a[50:60]  # exact copies
    b[20:30] = a[50:60]  # ... twice: tied nearest neighbours
    a[100:105] = a[0]  # duplicate query rows
    b[200] = b[201]
    for ratio in (0.8, None):
        _check(dev, oracle_mod, [a, b], [(0, 1), (1, 0)], ratio)


def test_counts_below_shortlist(dev, oracle_mod):
    rng = np.random.default_rng(4)
    big = _unit(rng, 300, 256)
    for n in (1, 2, 3, 4, 5, 8, 9):  # shortlist of 8: complete up to 8, certified from 9
        small = big[rng.permutation(300)[:n]] + 0.01 * _unit(rng, n, 256)
        _check(dev, oracle_mod, [small, big], [(0, 1), (1, 0)], None)
        _check(dev, oracle_mod, [small, big], [(0, 1), (1, 0)], 0.8)


def test_values_outside_fp16_range(dev, oracle_mod):
    rng = np.random.default_rng(5)
    a, b = _planted(rng, 300, 350, 128)
    _check(dev, oracle_mod, [a * 1e6, b * 1e6], [(0, 1)], 0.8)
    _check(dev, oracle_mod, [a, b * 3e5], [(0, 1)], None)


def test_near_equidistant_clusters(dev, oracle_mod):
    """Every row a tiny perturbation of one of a few centres: distances agree to ~1e-4, far below the fp16 error
    bound, so most shortlists cannot be certified and are rescanned exactly."""
    rng = np.random.default_rng(6)
    centres = _unit(rng, 3, 256)
    a = (centres[rng.integers(0, 3, 500)] + 1e-4 * rng.normal(size=(500, 256))).astype(np.float32)
    b = (centres[rng.integers(0, 3, 450)] + 1e-4 * rng.normal(size=(450, 256))).astype(np.float32)
    _check(dev, oracle_mod, [a, b], [(0, 1)], 0.8)
    _check(dev, oracle_mod, [a, b], [(0, 1)], None)


def test_twoway_matcher_selects_rerank(dev):
    from gtsfm_amd import native
    from gtsfm_amd.frontend.matcher.twoway_matcher import select_match_mode

    rng = np.random.default_rng(8)
    assert select_match_mode(_unit(rng, 5, 256), _unit(rng, 6, 256)) == native.GTSFM_MATCH_F16_RERANK
    assert select_match_mode(_unit(rng, 5, 300), _unit(rng, 6, 300)) == native.GTSFM_MATCH_EXACT_F32


def test_c3_size_4096_by_4096_256d(dev, oracle_mod):
    """BASELINE config C3's matcher shape: 4096 x 4096 x 256-D SuperPoint-like descriptors (planted matches, ratio
    0.8), a batch of image pairs: identical to EXACT_F32 on every pair and to the oracle on two of them."""
    rng = np.random.default_rng(4096)
    base = _unit(rng, 4096, 256)
    descs = []
    for _ in range(4):
        d = _unit(rng, 4096, 256)
        k = int(0.3 * 4096)
        y = base[rng.permutation(4096)[:k]] + 0.15 * rng.normal(size=(k, 256)) / 16
        d[rng.permutation(4096)[:k]] = y / np.linalg.norm(y, axis=1, keepdims=True)
        descs.append(d.astype(np.float32))
    pairs = [(0, 1), (2, 3), (0, 3), (1, 2)]
    fast = _check(dev, oracle_mod, descs, pairs, 0.8, n_oracle=2)
    assert min(len(f) for f in fast) > 200  # ~0.3 x 0.3 x 4096 planted matches per pair


@pytest.mark.parametrize("dim", [200, 256])
def test_clustered_pairs_use_exact_tiles(dev, oracle_mod, dim):
    """A batch mixing clustered pairs (most shortlists uncertified: the whole (pair, side) goes to the tiled exact
    kernel, fl_exact_tile_kernel) with planted pairs (few uncertified: per-keypoint rescans), ragged counts and a dim
    that is not a multiple of the tile's K chunk: identical to EXACT_F32 and to the oracle."""
    rng = np.random.default_rng(60 + dim)
    centres = _unit(rng, 4, dim)

    def clustered(n):
        return (centres[rng.integers(0, 4, n)] + 3e-3 * rng.normal(size=(n, dim)) / np.sqrt(dim)).astype(np.float32)

    a, b = clustered(700), clustered(1000)
    c, d = _planted(rng, 900, 650, dim)
    descs = [a, b, c, d, clustered(65)]
    pairs = [(0, 1), (2, 3), (1, 0), (0, 3), (4, 1), (3, 4)]
    for ratio in (0.8, None):
        _check(dev, oracle_mod, descs, pairs, ratio, n_oracle=3)


def test_rerank_certificate_stats(dev):
    """gtsfm_match_rerank_stats (the C3 bench line's uncertified / rescan fractions): clustered pairs go whole to the
    exact tiles, planted ones certify nearly everything; the per-side counts add up to the total."""
    from gtsfm_amd import device, native

    rng = np.random.default_rng(77)
    centres = _unit(rng, 4, 256)
    clustered = [(centres[rng.integers(0, 4, n)] + 3e-3 * rng.normal(size=(n, 256)) / 16).astype(np.float32)
                 for n in (700, 1000)]
    c, d = _planted(rng, 900, 650, 256)
    descs = clustered + [c, d]
    kmax = max(len(x) for x in descs)
    arr = np.zeros((len(descs), kmax, 256), np.float32)
    for i, x in enumerate(descs):
        arr[i, : len(x)] = x
    cnt = torch.tensor([len(x) for x in descs], dtype=torch.int32, device=dev)
    desc_t = torch.from_numpy(arr).to(dev)
    for pairs, clustered_sides in (([(2, 3)], 0), ([(0, 1), (2, 3)], 1700)):
        st = {}
        device.match_pairs(desc_t, cnt, torch.tensor(pairs, dtype=torch.int32, device=dev), 0.8,
                           native.GTSFM_MATCH_F16_RERANK, stats=st)
        sides = sum(len(descs[i]) + len(descs[j]) for i, j in pairs)
        assert st["keypoint_sides"] == sides
        assert 0 <= st["rescan_frac"] <= st["uncertified_frac"] <= 1 and 0 <= st["tiled_frac"] <= 1
        assert abs(st["tiled_frac"] - clustered_sides / sides) < 1e-9
        if clustered_sides == 0:
            assert st["uncertified_frac"] < 0.05
    st = {}
    device.match_pairs(desc_t, cnt, torch.tensor([(2, 3)], dtype=torch.int32, device=dev), 0.8,
                       native.GTSFM_MATCH_EXACT_F32, stats=st)
    assert st == {}
