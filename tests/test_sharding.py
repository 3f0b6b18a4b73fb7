"""Multi-rank layout of the front-end (gtsfm_amd/frontend/sharding.py) under gloo, world_size 2 and 3, on CPU.

Checks that every pair is owned by exactly one rank, that the all-gathered feature blocks put image i at
global_slots[i] on every rank, and that a sharded run of the matcher oracle over a small scene reproduces the
single-process result pair for pair (the exchange is the only collective on the data path).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gtsfm_amd.frontend import sharding


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _features(i: int, k: int = 40, d: int = 16):
    rng = np.random.default_rng(100 + i)
    n = k - (i % 3) * 5  # ragged counts
    desc = np.zeros((k, d), np.float32)
    desc[:n] = rng.integers(0, 60, size=(n, d))
    xy = np.zeros((k, 2), np.float32)
    xy[:n] = rng.uniform(0, 100, size=(n, 2))
    return xy, desc, n


def _worker(rank: int, world: int, port: int, n_img: int, out_dir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = sharding.local_images(n_img, world, rank)
        feats = [_features(int(i)) for i in mine]
        xy = torch.from_numpy(np.stack([f[0] for f in feats]))
        desc = torch.from_numpy(np.stack([f[1] for f in feats]))
        cnt = torch.tensor([f[2] for f in feats], dtype=torch.int32)
        n_per = sharding.images_per_rank(n_img, world)
        xy_all, desc_all, cnt_all = sharding.allgather_features((xy, desc, cnt), n_per, wire=(None, torch.uint8, None))
        slot = sharding.global_slots(n_img, world)
        for i in range(n_img):
            exy, edesc, en = _features(i)
            assert int(cnt_all[slot[i]]) == en
            assert np.array_equal(desc_all[slot[i]].numpy(), edesc)
            assert np.array_equal(xy_all[slot[i]].numpy(), exy)
        # pair work of this rank: the matcher oracle stands in for the device kernel (host logic only)
        from oracle import oracle

        pairs = sharding.all_pairs(n_img)
        block = sharding.rank_pairs(pairs, world, rank)
        counts = []
        for p in block:
            i1, i2 = pairs[p]
            s1, s2 = slot[i1], slot[i2]
            m = oracle.twoway_match(desc_all[s1, : cnt_all[s1]].numpy(), desc_all[s2, : cnt_all[s2]].numpy(), 0.8)
            counts.append(len(m))
        local = torch.tensor(counts, dtype=torch.int64)
        full = sharding.gather_pair_results(local, pairs)
        np.save(os.path.join(out_dir, f"counts_{world}_{rank}.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


def test_pair_blocks_partition_all_pairs():
    for n_img in (1, 2, 7, 100):
        pairs = sharding.all_pairs(n_img)
        for world in (1, 2, 3, 8):
            owned = np.concatenate([sharding.rank_pairs(pairs, world, r) for r in range(world)])
            assert np.array_equal(np.sort(owned), np.arange(len(pairs)))  # a partition
            sizes = [len(sharding.rank_pairs(pairs, world, r)) for r in range(world)]
            assert max(sizes) - min(sizes) <= sharding.PAIR_BLOCK  # runs of <= 4 pairs, each to the least-loaded rank
            for r in range(world):  # a rank's pairs stay in list order and keep whole (i1, i2 // 4) runs
                own = sharding.rank_pairs(pairs, world, r)
                assert np.all(np.diff(own) > 0)
                run = sharding.pair_runs(pairs)
                assert set(np.flatnonzero(np.isin(run, run[own])).tolist()) == set(own.tolist())


def test_global_slots_are_rank_major():
    for n_img, world in ((10, 3), (8, 8), (5, 1), (3, 4)):
        slot = sharding.global_slots(n_img, world)
        n_per = sharding.images_per_rank(n_img, world)
        assert len(set(slot.tolist())) == n_img and slot.max() < world * n_per
        for r in range(world):
            loc = sharding.local_images(n_img, world, r)
            assert np.array_equal(slot[loc], r * n_per + np.arange(len(loc)))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_front_end_matches_single_process(world, tmp_path, oracle_mod):
    n_img = 7
    mp.start_processes(_worker, args=(world, _free_port(), n_img, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    # single-process reference of the same host logic
    from oracle import oracle

    pairs = sharding.all_pairs(n_img)
    ref = []
    for i1, i2 in pairs:
        (_, d1, n1), (_, d2, n2) = _features(int(i1)), _features(int(i2))
        ref.append(len(oracle.twoway_match(d1[:n1], d2[:n2], 0.8)))
    for r in range(world):
        got = np.load(tmp_path / f"counts_{world}_{r}.npy")
        assert np.array_equal(got, np.array(ref))


def test_match_plan_fills_the_gpu():
    """C2 (4950 pairs) keeps full groups of 4. The rank shares keep them too (whole runs are dealt): at 2 and 4 ranks
    (nearly) every group of 4 is full and the plan keeps full groups of 2 or 4 (single-pair round-robin dealing left
    them half / a quarter full, so the plan fell back to groups of 1); at 8 ranks (~620 pairs, ~160 groups for 256 CUs)
    the plan trades group size for pass-split workgroups: 10 instead of 12 pair-passes."""
    from gtsfm_amd import device, native
    from gtsfm_amd.frontend import sharding

    native.lib()
    pairs = sharding.all_pairs(100)
    g = device.match_plan(pairs, 2048, 128, n_cu=256)
    assert g.shape[1] == 4
    for world in (2, 4):
        share = pairs[sharding.rank_pairs(pairs, world, 0)]
        gw = device.match_plan(share, 2048, 128, n_cu=256)
        assert (device.pair_groups(share, 4) >= 0).mean() > 0.95
        assert gw.shape[1] >= 2 and (gw >= 0).mean() > 0.95, (world, gw.shape, (gw >= 0).mean())
    share = pairs[sharding.rank_pairs(pairs, 8, 0)]
    g8 = device.match_plan(share, 2048, 128, n_cu=256)
    assert (device.pair_groups(share, 4) >= 0).mean() > 0.95
    assert device._split_cost(len(g8), g8.shape[1], 2048, 256) <= 10
    assert sorted(g8[g8 >= 0].tolist()) == list(range(len(share)))


def test_emulated_allgather_equals_rank_major_gather():
    """One process emulating rank r of a 3-rank job (bench.py --emulate-world): the other ranks' packed blocks plus
    this rank's fresh block unpack to exactly the tensors the real all-gather produces (rank-major, padded to n_per,
    u8 wire for the descriptors)."""
    from gtsfm_amd.frontend import sharding

    n_img, world = 7, 3
    n_per = sharding.images_per_rank(n_img, world)
    g = torch.Generator().manual_seed(3)
    full_xy = torch.rand((n_img, 5, 2), generator=g)
    full_desc = torch.randint(0, 256, (n_img, 5, 8), generator=g).float()
    full_cnt = torch.randint(1, 6, (n_img,), generator=g, dtype=torch.int32)
    wire = [None, torch.uint8, None]

    def local(r):
        i = torch.from_numpy(sharding.local_images(n_img, world, r))
        return [full_xy[i], full_desc[i], full_cnt[i]]

    blocks = [sharding.pack_features(local(r), n_per, wire)[0] for r in range(world)]
    for rank in range(world):
        others = torch.stack(blocks)
        others[rank].zero_()
        got = sharding.allgather_features(local(rank), n_per, wire=wire,
                                          exchange=sharding.EmulatedAllGather(others, rank))
        slot = sharding.global_slots(n_img, world)
        for t, ref in zip(got, (full_xy, full_desc, full_cnt)):
            assert t.shape[0] == world * n_per and t.dtype == ref.dtype
            assert torch.equal(t[torch.from_numpy(slot)], ref)
