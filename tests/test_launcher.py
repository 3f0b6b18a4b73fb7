"""Multi-rank launch path on CPU (gloo): gtsfm_amd/launch.py and the AllPairsFrontEnd host logic at world sizes 2 and 3.

- spawn_ranks starts fresh ranks that each see WORLD_SIZE 2 and join one process group (the path `bench.py --gpus N`
  takes before anything touches a GPU); bench.py's own launch is probed the same way;
- a failing rank ends the job with its status instead of leaving its peer blocked;
- AllPairsFrontEnd, sharded over 2 and 3 gloo ranks (7 images over 3: a ragged split) with the oracle standing in
  for the HIP kernels, reproduces the single-rank run pair for pair (R, t, inlier counts, ISP verdicts, verified rows, keypoints): the all-gather is the
  only exchange and every pair keeps its global RANSAC key.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from gtsfm_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK_SCRIPT = os.path.join(REPO, "tests", "frontend_rank.py")


def test_spawn_ranks_reports_world_2(tmp_path):
    rc = launch.spawn_ranks(2, RANK_SCRIPT, ["probe", str(tmp_path)])
    assert rc == 0
    for r in range(2):
        d = json.loads((tmp_path / f"rank_{r}.json").read_text())
        assert d == {"rank": r, "world": 2, "local_rank": r, "dist_world": 2, "device": "cpu"}


def test_bench_launcher_spawns_ranks_before_gpu_use():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-probe"],
                         capture_output=True, text=True, timeout=300, cwd=REPO)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["dist_world"] == 2 for d in lines)


def test_spawn_ranks_propagates_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(3)\n"
                      "time.sleep(120)\n")
    rc = launch.spawn_ranks(2, str(script), [])
    assert rc == 3


def _load(path):
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("world,n_img", [(2, 5), (3, 7)])  # 7 over 3 ranks: ragged (3, 2, 2 images)
def test_frontend_gloo_sharded_equals_single_rank(tmp_path, world, n_img):
    rc = launch.spawn_ranks(world, RANK_SCRIPT, ["frontend", str(tmp_path), str(n_img)])
    assert rc == 0
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import frontend_rank  # noqa: E402

    from gtsfm_amd.frontend import sharding

    torch.set_num_threads(1)
    _, ref = frontend_rank.run_frontend(n_img, launch.RankInfo(0, 1, 0, torch.device("cpu")))
    parts = [_load(tmp_path / f"results_{world}_{r}.npz") for r in range(world)]
    # rank r holds the pairs sharding.rank_pairs(.., r) (round-robin): back to pair order
    owner = np.concatenate([sharding.rank_pairs(ref.pairs, world, r) for r in range(world)])
    order = np.argsort(owner)
    got_pairs = np.concatenate([p["pairs"] for p in parts])[order]
    assert np.array_equal(got_pairs, ref.pairs) and len(ref.pairs) == n_img * (n_img - 1) // 2
    for key in ("status", "n_inliers", "n_matches", "isp_ok"):
        assert np.array_equal(np.concatenate([p[key] for p in parts])[order], getattr(ref, key)), key
    np.testing.assert_array_equal(np.concatenate([p["R"] for p in parts])[order], ref.R)
    np.testing.assert_array_equal(np.concatenate([p["t"] for p in parts])[order], ref.t)
    k = 0
    for part in parts:
        for p in range(len(part["pairs"])):
            rows = part["v_corr"][part["offsets"][p]: part["offsets"][p + 1]]
            assert np.array_equal(rows, ref.verified(int(owner[k]))), int(owner[k])
            k += 1
    # keypoints: each rank holds its own images, identical to the single-rank extraction of the same image
    for r, part in enumerate(parts):
        for j, i in enumerate(sharding.local_images(n_img, world, r)):
            n = part["kp_count"][j]
            assert n == ref.kp_count[i]
            assert np.array_equal(part["kp_xy"][j, :n], ref.kp_xy[i, :n])
    # the engine's results are the oracle's own per-pair results
    assert (ref.status == 0).sum() >= 1 and ref.n_inliers.max() >= 6
    for p in range(len(ref.pairs)):
        v = ref.verified(p)
        assert len(v) == (ref.n_inliers[p] if ref.status[p] == 0 else 0)
