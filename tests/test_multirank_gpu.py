"""The multi-rank engine with the real HIP kernels on a one-GPU box: two ranks (both on cuda:0, process group gloo,
the packed feature blocks gathered through the host -- RCCL refuses two ranks on one device) extract their images,
exchange, and match / verify their pair shares; the union of their results equals one rank's run of the whole job
bit for bit (keypoints, putatives, verified rows, R, t). What RCCL would carry is the same packed block."""
import os
import sys

import numpy as np
import pytest
import torch

from gtsfm_amd import launch
from tests.conftest import REPO

pytestmark = pytest.mark.gpu
RANK_SCRIPT = os.path.join(REPO, "tests", "frontend_rank.py")


def _load(path):
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("world,n_img", [(2, 5)])
def test_two_ranks_on_one_gpu_equal_one_rank(tmp_path, world, n_img):
    from gtsfm_amd import native
    from gtsfm_amd.frontend import sharding

    native.require_gpu()
    rc = launch.spawn_ranks(world, RANK_SCRIPT, ["gpushared", str(tmp_path), str(n_img)])
    assert rc == 0
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import frontend_rank  # noqa: E402

    _, ref = frontend_rank.run_frontend_gpu(n_img, 0, 1)
    parts = [_load(tmp_path / f"gpu_{world}_{r}.npz") for r in range(world)]
    # rank r holds the pairs sharding.rank_pairs(.., r) (round-robin): back to pair order
    owner = np.concatenate([sharding.rank_pairs(ref.pairs, world, r) for r in range(world)])
    order = np.argsort(owner)
    assert np.array_equal(np.concatenate([p["pairs"] for p in parts])[order], ref.pairs)
    for key in ("status", "n_inliers", "n_matches", "isp_ok"):
        assert np.array_equal(np.concatenate([p[key] for p in parts])[order], getattr(ref, key)), key
    np.testing.assert_array_equal(np.concatenate([p["R"] for p in parts])[order], ref.R)
    np.testing.assert_array_equal(np.concatenate([p["t"] for p in parts])[order], ref.t)
    k = 0
    for part in parts:
        for p in range(len(part["pairs"])):
            q = int(owner[k])
            assert np.array_equal(part["v_corr"][part["offsets"][p]: part["offsets"][p + 1]], ref.verified(q)), q
            k += 1
    for r, part in enumerate(parts):
        for j, i in enumerate(sharding.local_images(n_img, world, r)):
            n = part["kp_count"][j]
            assert n == ref.kp_count[i] and np.array_equal(part["kp_xy"][j, :n], ref.kp_xy[i, :n])
    assert (ref.status == 0).sum() >= 3


def test_rccl_exchange_world1_equals_plain_step(tmp_path):
    """the `nccl` (RCCL) process group forms on cuda:0 (world size 1, before any other GPU call
    in that process), the packed feature exchange runs through all_gather_into_tensor on device buffers and comes back
    byte for byte, and one engine step through the collective equals the plain step (which skips the exchange at
    world 1) in every result field."""
    import json

    from gtsfm_amd import native

    native.require_gpu()
    rc = launch.spawn_ranks(1, RANK_SCRIPT, ["rccl1", str(tmp_path), "4"])
    assert rc == 0
    checks = json.load(open(tmp_path / "rccl_checks.json"))
    assert checks and all(checks.values()), checks
    a, b = _load(tmp_path / "rccl_collective.npz"), _load(tmp_path / "rccl_plain.npz")
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (a["status"] == 0).sum() >= 2
