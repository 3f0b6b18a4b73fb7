"""oracle/deep.py (the CPU restatement of SuperPoint / SuperGlue used as checker and CPU baseline) against the reference
modules' own outputs on seeded random weights (tests/golden/superpoint_random_w0.npz, superglue_random_w0.npz, written
in this container by tests/golden/make_superpoint_golden.py / make_superglue_golden.py from
/root/reference/thirdparty/SuperGluePretrainedNetwork/models/*.py)."""
import os

import numpy as np
import pytest

from superpoint_weights import superglue_state_dict, superpoint_state_dict
from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def sp_golden():
    return np.load(os.path.join(GOLDEN, "superpoint_random_w0.npz"))


@pytest.mark.parametrize("case", ["lund_250x333", "synthetic_240x320", "lund_480x640"])
def test_superpoint_restatement_matches_reference(sp_golden, case):
    from oracle import deep

    g = sp_golden
    kp, sc, desc = deep.superpoint(g[f"{case}__image"], superpoint_state_dict(0))
    np.testing.assert_array_equal(kp, g[f"{case}__keypoints"])
    np.testing.assert_allclose(sc, g[f"{case}__scores"], rtol=1e-5, atol=1e-7)
    rows = g[f"{case}__desc_rows"]
    np.testing.assert_allclose(desc[rows], g[f"{case}__desc"], atol=2e-6)


def test_superpoint_mask_follows_reference_filter(sp_golden):
    """The oracle's mask = the reference module's keypoints (golden) through gtsfm's Keypoints.filter_by_mask
    (keypoints.py:124-125: mask[round(y), round(x)] == 1) and then get_top_k's highest-score set (superpoint.py:68-72)."""
    from oracle import deep

    g = sp_golden
    img = g["lund_480x640__image"]
    rng = np.random.default_rng(5)
    mask = (rng.random(img.shape) < 0.7).astype(np.uint8)
    mask[rng.random(img.shape) < 0.1] = 2  # filter_by_mask keeps only == 1
    ref = g["lund_480x640__keypoints"]
    r = np.round(ref).astype(int)
    kept = ref[mask[r[:, 1], r[:, 0]] == 1]
    kp, _, _ = deep.superpoint(img, superpoint_state_dict(0), mask=mask)
    np.testing.assert_array_equal(kp, kept)
    k = len(kept) // 2
    kp_k, sc_k, _ = deep.superpoint(img, superpoint_state_dict(0), max_keypoints=k, mask=mask)
    sc_all = g["lund_480x640__scores"][mask[r[:, 1], r[:, 0]] == 1]
    assert len(kp_k) == k and np.isclose(np.sort(sc_k), np.sort(sc_all)[-k:], rtol=1e-5).all()


@pytest.mark.parametrize("case", ["small_150x170", "mid_700x650"])
def test_superglue_restatement_matches_reference(case):
    from oracle import deep

    g = np.load(os.path.join(GOLDEN, "superglue_random_w0.npz"))
    k = lambda n: g[f"{case}__{n}"]  # noqa: E731
    hw = tuple(int(v) for v in k("hw"))
    m0, ms0 = deep.superglue(k("kp0"), k("kp1"), k("d0"), k("d1"), k("s0"), k("s1"), hw, hw, superglue_state_dict(0))
    ref = k("matches0")
    assert (m0 >= 0).sum() > 10
    # float32 on both sides, different accumulation order inside the einsums: allow the rare near-threshold flip
    assert (m0 != ref).sum() <= max(1, 0.005 * len(ref)), ((m0 != ref).sum(), len(ref))
    both = (m0 >= 0) & (ref >= 0)
    np.testing.assert_allclose(ms0[both], k("mscores0")[both], atol=1e-4)


def test_oracle_netvlad_vs_reference_golden():
    """oracle.deep.netvlad against the reference's NetVLAD.forward / NetVLADLayer (tests/golden/make_netvlad_golden.py,
    seeded random weights; the VGG16 layer list itself is parity-unpinned: torchvision is absent). Only summation
    order differs (the residual sums are formed as sum s x - c sum s instead of the reference's explicit residuals)."""
    from netvlad_weights import netvlad_cases as cases, netvlad_state_dict
    from oracle import deep

    sd = netvlad_state_dict(0)
    with np.load(os.path.join(GOLDEN, "netvlad_random_w0.npz")) as z:
        gold = {k: z[k] for k in z.files}
    for name, imgs in cases().items():
        for i, im in enumerate(imgs):
            desc, vlad = deep.netvlad(im, sd)
            np.testing.assert_allclose(vlad, gold[f"{name}/vlad"][i], atol=2e-6)
            np.testing.assert_allclose(desc, gold[f"{name}/desc"][i], atol=2e-6)
