"""BASELINE config C4's workload on one GPU: AllPairsFrontEnd over 1000 rendered 1920x1080 images, all 499,500 pairs,
2048 SIFT keypoints, at the default 131,072-pair match / verify chunks (four chunked launch sequences per step), the
same path bench.py --config c4 times.

Checked on the whole step's host results:
- per-pair records are consistent: status 1 exactly when fewer than 6 putatives (opencv_verifier_base.py:69-78),
  verified rows == inlier count for status 0 and none otherwise, the inlier-support verdict == (status 0, >= 15
  inliers, inlier ratio >= 0.1) (inlier_support_processor.py:39-95), keypoint indices inside each image's count;
and on 48 sampled pairs (24 that pass the inlier-support filter, 24 seeded-random) against the oracle, on the GPU's
own SIFT features (bit-exact vs the oracle elsewhere: tests/test_sift_gpu.py):
- putatives: the oracle TwoWayMatcher's count equals the chunked launch's, and the verified rows are an in-order
  subsequence of the oracle's putatives (bit-exact indices);
- verifier: the oracle's RANSAC on those putatives with the pair's global sampler key -> same status, the same inlier
  count, bit-identical R / t and the same verified rows (tests/test_verifier_gpu.py's bar).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from tests import scenes

pytestmark = pytest.mark.gpu

N_IMG, H, W, KPTS = 1000, 1080, 1920, 2048


@pytest.mark.timeout(900)
def test_c4_one_gpu_all_pairs_consistent_and_sampled_vs_oracle(oracle_mod):
    from gtsfm_amd import native, synthetic
    from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig

    native.require_gpu()
    dev = torch.device("cuda")
    scene = synthetic.render_scene(N_IMG, H, W, device="cuda")
    host = scene.images.cpu().pin_memory()
    del scene.images
    torch.cuda.empty_cache()
    cfg = FrontEndConfig(kpts=KPTS)
    assert cfg.pair_chunk == 131072
    fe = AllPairsFrontEnd(host, scene.intrinsics, N_IMG, 0, 1, dev, cfg)
    assert len(fe.pchunks) == 4 and fe.total_pairs == N_IMG * (N_IMG - 1) // 2
    res = fe.step()
    torch.cuda.synchronize()
    P = len(res.pairs)
    assert P == fe.total_pairs
    st, n_inl, n_m, isp = res.status, res.n_inliers, res.n_matches, res.isp_ok
    assert set(np.unique(st)) <= {0, 1, 2}
    np.testing.assert_array_equal(st == 1, n_m < 6)
    assert np.all(np.diff(res.offsets) >= 0) and res.offsets[0] == 0 and res.offsets[-1] == len(res.v_corr)
    rows = np.diff(res.offsets)
    np.testing.assert_array_equal(rows, np.where(st == 0, n_inl, 0))
    ratio = np.where(n_m > 0, n_inl / np.maximum(n_m, 1), 0.0)
    np.testing.assert_array_equal(isp, (st == 0) & (n_inl >= 15) & (ratio >= 0.1))
    kc = res.kp_count
    pair_of_row = np.repeat(np.arange(P), rows)
    assert np.all(res.v_corr[:, 0] < kc[res.pairs[pair_of_row, 0]])
    assert np.all(res.v_corr[:, 1] < kc[res.pairs[pair_of_row, 1]])
    assert isp.sum() > 1000  # neighbouring views on the orbit verify

    # sampled pairs against the oracle
    rng = np.random.default_rng(4)
    ok_pairs = np.flatnonzero(isp)
    sample = np.unique(np.concatenate([rng.choice(ok_pairs, 24, replace=False), rng.choice(P, 24, replace=False)]))
    imgs = np.unique(res.pairs[sample])
    desc = {int(i): fe.feats.desc[int(i), : kc[i]].cpu().numpy() for i in imgs}
    xy = res.kp_xy
    K = scene.intrinsics

    def check(p):
        i1, i2 = (int(v) for v in res.pairs[p])
        m = oracle_mod.twoway_match(desc[i1], desc[i2], cfg.ratio).reshape(-1, 2)
        out = {"p": p, "n_put": len(m)}
        v = res.verified(p)
        # in-order subsequence of the oracle's putatives
        pos = {(int(a), int(b)): k for k, (a, b) in enumerate(m)}
        idx = [pos.get((int(a), int(b)), -1) for a, b in v]
        out["subseq"] = all(k >= 0 for k in idx) and all(b > a for a, b in zip(idx, idx[1:]))
        if len(m) >= 6:
            f1, f2 = K[i1], K[i2]
            x1 = (xy[i1, m[:, 0]].astype(np.float64) - f1[1:3]) / f1[0]
            x2 = (xy[i2, m[:, 1]].astype(np.float64) - f2[1:3]) / f2[0]
            out["ref"] = oracle_mod.ransac_E(x1, x2, cfg.thresh_px / max(f1[0], f2[0]), pair_id=int(fe.pair_ids[p]))
            out["m"] = m
        return out

    with ThreadPoolExecutor(16) as pool:
        checks = list(pool.map(check, sample))
    for c in checks:
        p = c["p"]
        assert c["n_put"] == n_m[p], (p, c["n_put"], n_m[p])
        assert c["subseq"], p
        if c["n_put"] < 6:
            assert st[p] == 1, p
            continue
        ref = c["ref"]
        if ref is None:  # the oracle found no model
            assert st[p] == 2, (p, st[p])
            continue
        assert st[p] == 0, (p, st[p])
        _, rmask, rR, rt, rn, _ = ref
        assert int(n_inl[p]) == rn, (p, n_inl[p], rn)
        np.testing.assert_array_equal(res.R[p], rR)
        np.testing.assert_array_equal(res.t[p], rt)
        o_rows = [(int(a), int(b)) for a, b in c["m"][rmask.astype(bool)]]
        assert [(int(a), int(b)) for a, b in res.verified(p)] == o_rows, p
