"""Retrievers on the CPU: the numpy retrieval oracle and the host-only pair generators.

Parity of the NetVLAD path is unpinned against the reference module itself (netvlad_retriever.py imports gtsam, absent
here, and the NetVLAD weights are not available offline). It is pinned instead on the reference tests' expected pair
lists (tests/retriever/test_netvlad_retriever.py:24-82), reproduced by descriptors whose similarities have the
structure those tests assert ("closest image is most similar", with the door test's (7, 10) exception), and on
torch.topk itself (importable here) for the selection semantics.
"""
import numpy as np
import pytest
import torch

from gtsfm_amd.retriever.sequential_retriever import ExhaustiveRetriever, SequentialRetriever, sequential_pairs

# reference tests/retriever/test_netvlad_retriever.py:59-81 (num_matched=2 over the 12 Lund door images)
DOOR_EXPECTED = [(0, 1), (0, 2), (1, 2), (1, 3), (2, 3), (2, 4), (3, 4), (3, 5), (4, 5), (4, 6), (5, 6), (5, 7),
                 (6, 7), (6, 8), (7, 8), (7, 10), (8, 9), (8, 10), (9, 10), (9, 11), (10, 11)]


def door_like_descriptors(dim: int = 64) -> np.ndarray:
    """12 unit descriptors whose Gram matrix is exp(-|i - j| / 2) except sim(7, 10) = 0.45 > sim(7, 9)."""
    n = 12
    i = np.arange(n)
    S = np.exp(-np.abs(i[:, None] - i[None, :]) / 2.0)
    S[7, 10] = S[10, 7] = 0.45
    L = np.linalg.cholesky(S)  # positive definite: a valid Gram matrix
    Q, _ = np.linalg.qr(np.random.default_rng(0).standard_normal((dim, n)))
    return (L @ Q.T).astype(np.float32)  # rows: unit vectors with <d_i, d_j> = S_ij


def torch_pairs_from_score_matrix(scores: np.ndarray, invalid: np.ndarray, num_select: int, min_score):
    """The reference's selection (netvlad_retriever.py:213-228) run with torch.topk on the CPU."""
    s = torch.from_numpy(scores.copy())
    inv = torch.from_numpy(invalid.copy())
    k = min(num_select, s.shape[0])
    if min_score is not None:
        inv |= s < min_score
    s.masked_fill_(inv, float("-inf"))
    top = torch.topk(s, k=k, dim=1)
    idx, valid = top.indices.numpy(), top.values.isfinite().numpy()
    return [(int(i), int(idx[i, j])) for i, j in zip(*np.where(valid))]


def test_oracle_door_like_pairs(oracle_mod):
    d = door_like_descriptors()
    sim = oracle_mod.retrieval_similarity(d, 50)
    assert oracle_mod.retrieval_pairs(sim, 2, 0.1) == DOOR_EXPECTED


def test_oracle_two_frames(oracle_mod):
    # test_netvlad_retriever.py:24-42: only (0, 1) is possible between two frames
    d = door_like_descriptors()[:2]
    assert oracle_mod.retrieval_pairs(oracle_mod.retrieval_similarity(d, 50), 2, 0.1) == [(0, 1)]


@pytest.mark.parametrize("n,dim,bs", [(1, 4, 50), (7, 3, 2), (51, 16, 50), (130, 32, 64)])
def test_oracle_similarity_blocks(oracle_mod, n, dim, bs):
    d = np.random.default_rng(n).standard_normal((n, dim)).astype(np.float32)
    sim = oracle_mod.retrieval_similarity(d, bs)
    full = d.astype(np.float64) @ d.astype(np.float64).T
    blk = np.arange(n) // bs
    upper = blk[None, :] >= blk[:, None]
    assert np.all(sim[~upper] == 0)
    np.testing.assert_allclose(sim[upper], full[upper], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_selection_matches_torch_topk(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    n1, n2 = int(rng.integers(1, 40)), int(rng.integers(1, 40))
    scores = rng.standard_normal((n1, n2)).astype(np.float32)
    invalid = rng.random((n1, n2)) < 0.3
    k = int(rng.integers(1, n2 + 1))
    k = min(k, n1) if min(k, n1) <= n2 else n2
    min_score = None if seed % 2 else -0.5
    assert oracle_mod.retrieval_pairs(scores, k, min_score, invalid) == \
        torch_pairs_from_score_matrix(scores, invalid, k, min_score)
    # square case with the retriever's own mask
    sq = rng.standard_normal((n1, n1)).astype(np.float32)
    inv = ~np.triu(np.ones((n1, n1), bool), 1)
    assert oracle_mod.retrieval_pairs(sq, k, min_score) == torch_pairs_from_score_matrix(sq, inv, k, min_score)


def test_oracle_selection_edges(oracle_mod):
    inv = ~np.triu(np.ones((5, 5), bool), 1)
    s = np.full((5, 5), 0.5, np.float32)  # all ties: ascending columns
    assert oracle_mod.retrieval_pairs(s, 2, 0.1) == [(0, 1), (0, 2), (1, 2), (1, 3), (2, 3), (2, 4), (3, 4)]
    assert oracle_mod.retrieval_pairs(s, 2, 0.6) == []  # every score below min_score
    assert oracle_mod.retrieval_pairs(s, 99, None) == [(i, j) for i in range(5) for j in range(i + 1, 5)]  # k -> N
    s2 = s.copy()
    s2[0, 3] = np.nan  # NaN takes the first top-k slot and is not emitted
    assert oracle_mod.retrieval_pairs(s2, 2, 0.1)[:1] == [(0, 1)]
    s3 = np.random.default_rng(9).random((5, 5)).astype(np.float32)  # distinct values: torch's order is defined
    s3[0, 3] = s3[1, 2] = np.nan
    assert oracle_mod.retrieval_pairs(s3, 2, 0.1) == torch_pairs_from_score_matrix(s3, inv, 2, 0.1)
    assert oracle_mod.retrieval_pairs(np.zeros((0, 0), np.float32), 2, 0.1) == []


@pytest.mark.parametrize("n,look", [(0, 3), (1, 3), (10, 1), (10, 3), (12, 20)])
def test_sequential_pairs(n, look):
    # sequential_retriever.py:49-56
    ref = [(i1, i2) for i1 in range(n) for i2 in range(i1 + 1, min(i1 + look + 1, n))]
    assert SequentialRetriever(look).get_image_pairs(None, [f"{i}.jpg" for i in range(n)]) == ref
    assert [tuple(p) for p in sequential_pairs(n, look).tolist()] == ref


def test_exhaustive_pairs():
    names = [f"{i}.jpg" for i in range(7)]
    r = ExhaustiveRetriever()
    assert r.get_image_pairs(None, names) == [(i, j) for i in range(7) for j in range(i + 1, 7)]
    assert r.evaluate(7, r.get_image_pairs(None, names)) == {
        "retriever_metrics": {"num_input_images": 7, "num_retrieved_image_pairs": 21}}
