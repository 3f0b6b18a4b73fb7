"""GPU retrieval (gtsfm_retrieval_similarity / gtsfm_retrieval_pairs through NetVLADRetriever) against the oracle.

Similarity: fp32 MFMA accumulation vs the oracle's fp64-accumulated fp32 result, |diff| <= 8 sqrt(D) 2^-24
sum_k |a_k b_k| (8 sigma of the random-walk rounding error of a D-term fp32 sum in any order -- torch's own einsum
sits inside the same band); entries below the block diagonal are exactly 0. Selection: bit-exact pair lists vs the oracle on the SAME score matrix (integer/index work). Parity vs the
reference module is unpinned (gtsam absent); see tests/test_retriever.py for the pinning on the reference tests'
expected pair lists.
"""
import numpy as np
import pytest
import torch

from test_retriever import DOOR_EXPECTED, door_like_descriptors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from gtsfm_amd import native

    native.require_gpu()
    native.lib()
    return torch.device("cuda")


def _sim_gpu(d: np.ndarray, bs: int) -> np.ndarray:
    from gtsfm_amd import device as gdev

    return gdev.retrieval_similarity(torch.from_numpy(d).cuda(), bs).cpu().numpy()


@pytest.mark.parametrize("n,dim,bs", [(1, 4, 50), (12, 3, 50), (50, 64, 50), (51, 100, 50), (130, 256, 7),
                                      (300, 4096, 50), (257, 33, 1000), (64, 31, 64)])
def test_similarity_vs_oracle(dev, oracle_mod, n, dim, bs):
    rng = np.random.default_rng(n * 7 + dim)
    d = rng.standard_normal((n, dim)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    got = _sim_gpu(d, bs)
    ref = oracle_mod.retrieval_similarity(d, bs)
    blk = np.arange(n) // bs
    upper = blk[None, :] >= blk[:, None]
    assert np.all(got[~upper] == 0)
    bound = 8 * np.sqrt(dim) * 2.0 ** -24 * (np.abs(d.astype(np.float64)) @ np.abs(d.astype(np.float64)).T) + 1e-30
    assert np.all(np.abs(got - ref)[upper] <= bound[upper])


def test_similarity_empty(dev):
    from gtsfm_amd import device as gdev

    assert gdev.retrieval_similarity(torch.zeros((0, 8), device="cuda"), 50).shape == (0, 0)


@pytest.mark.parametrize("seed", range(8))
def test_pairs_vs_oracle_same_scores(dev, oracle_mod, seed):
    from gtsfm_amd.retriever.netvlad_retriever import pairs_from_score_matrix

    rng = np.random.default_rng(100 + seed)
    n1 = int(rng.integers(1, 700))
    n2 = n1 if seed % 2 == 0 else int(rng.integers(1, 700))
    scores = rng.standard_normal((n1, n2)).astype(np.float32)
    if seed % 3 == 0:
        scores = np.round(scores * 4) / 4  # many ties
    if seed == 5:
        scores[rng.random((n1, n2)) < 0.01] = np.nan
    invalid = rng.random((n1, n2)) < 0.2
    k = min(int(rng.integers(1, 40)), n2, n1)
    min_score = None if seed % 4 == 1 else 0.3
    got = pairs_from_score_matrix(torch.from_numpy(scores).cuda(), invalid, k, min_score)
    assert got == oracle_mod.retrieval_pairs(scores, k, min_score, invalid)


@pytest.mark.parametrize("n,k", [(1, 2), (2, 2), (12, 2), (100, 5), (1000, 10), (3000, 64), (500, 600)])
def test_retriever_vs_oracle(dev, oracle_mod, n, k):
    from gtsfm_amd.retriever.netvlad_retriever import NetVLADRetriever

    rng = np.random.default_rng(n + k)
    d = rng.standard_normal((n, 128)).astype(np.float32) + 0.5
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = NetVLADRetriever(num_matched=k, min_score=0.1)
    sim = r.compute_similarity_matrix(list(d))
    pairs = r.compute_pairs_from_similarity_matrix(sim, [f"{i}.jpg" for i in range(n)])
    assert pairs == oracle_mod.retrieval_pairs(sim.cpu().numpy(), k, 0.1)
    assert all(i < j for i, j in pairs)


def test_retriever_door_like(dev, tmp_path):
    from gtsfm_amd.retriever.joint_netvlad_sequential_retriever import JointNetVLADSequentialRetriever
    from gtsfm_amd.retriever.netvlad_retriever import NetVLADRetriever

    d = door_like_descriptors()
    names = [f"DSC_{i:04d}.JPG" for i in range(12)]
    pairs = NetVLADRetriever(num_matched=2).get_image_pairs(list(d), names, plots_output_dir=tmp_path)
    assert pairs == DOOR_EXPECTED
    assert (tmp_path / "netvlad_named_pairs.txt").read_text().count("\n") == len(DOOR_EXPECTED)
    assert NetVLADRetriever(num_matched=2).get_image_pairs(list(d[:2]), names[:2]) == [(0, 1)]
    joint = JointNetVLADSequentialRetriever(num_matched=2, min_score=0.1, max_frame_lookahead=1)
    assert joint.get_image_pairs(list(d), names) == sorted(set(DOOR_EXPECTED) | {(i, i + 1) for i in range(11)})
    with pytest.raises(ValueError):
        NetVLADRetriever(num_matched=2).get_image_pairs(None, names)


def test_retriever_max_scale(dev, oracle_mod):
    """MAX_NUM_IMAGES x 4096-D (NetVLAD's PCA-whitened size): size-independent properties on the full matrix, exact
    oracle comparison of the selection on sampled rows, and the similarity on sampled rows vs fp64."""
    from gtsfm_amd import device as gdev
    from gtsfm_amd.retriever.netvlad_retriever import MAX_NUM_IMAGES, NetVLADRetriever

    n, dim, k = MAX_NUM_IMAGES, 4096, 10
    g = torch.Generator(device="cuda").manual_seed(0)
    d = torch.randn((n, dim), device="cuda", generator=g) + 0.05
    d /= d.norm(dim=1, keepdim=True)
    r = NetVLADRetriever(num_matched=k, min_score=0.1)
    sim = r.compute_similarity_matrix(d)
    rows = np.random.default_rng(1).choice(n, 24, replace=False)
    dh = d.cpu().numpy().astype(np.float64)
    ref = dh[rows] @ dh.T
    blk = np.arange(n) // 50
    got = sim[torch.from_numpy(rows).cuda()].cpu().numpy()
    for a, i in enumerate(rows):
        up = blk >= blk[i]
        assert np.all(got[a][~up] == 0)
        assert np.max(np.abs(got[a][up] - ref[a][up])) < 8 * np.sqrt(dim) * 2.0 ** -24  # sum |a_k b_k| <= 1
    out, cnt = gdev.retrieval_pairs(sim, k, 0.1)
    out_h, cnt_h = out.cpu().numpy(), cnt.cpu().numpy()
    sim_rows = sim[torch.from_numpy(rows).cuda()].cpu().numpy()
    for a, i in enumerate(rows):
        bad = np.arange(n) <= i  # the retriever's strict upper triangle
        exp = oracle_mod.retrieval_select_row(sim_rows[a], bad, k, 0.1)
        assert out_h[i, :cnt_h[i], 1].tolist() == exp and np.all(out_h[i, :cnt_h[i], 0] == i)
    assert cnt_h[-1] == 0 and np.all(cnt_h <= k)

