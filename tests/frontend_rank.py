"""Child-process body for tests/test_launcher.py: one rank of a gloo job started by gtsfm_amd.launch.spawn_ranks.

    python tests/frontend_rank.py probe OUT_DIR            -> writes rank_<r>.json with what init_rank saw
    python tests/frontend_rank.py frontend OUT_DIR N_IMG   -> runs AllPairsFrontEnd (oracle kernels) and saves
                                                              results_<world>_<rank>.npz
    python tests/frontend_rank.py gpushared OUT_DIR N_IMG  -> every rank on cuda:0 with the HIP kernels (a one-GPU box
                                                              rehearsal of the multi-rank engine); the exchange is the
                                                              engine's packing with the blocks gathered over gloo on
                                                              the host (RCCL refuses two ranks on one GPU)
    python tests/frontend_rank.py rccl1 OUT_DIR N_IMG      -> an RCCL ("nccl") process group of world size 1 on cuda:0,
                                                              formed before any other GPU call; the exchange forced
                                                              through all_gather_into_tensor on device buffers
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gtsfm_amd import launch  # noqa: E402

H, W, KPTS = 240, 320, 400
ORBIT = 24  # cameras on the scene's orbit (15 degrees apart); the job uses the first n_img of them


def run_frontend(n_img: int, info: launch.RankInfo):
    from gtsfm_amd import synthetic
    from gtsfm_amd.frontend import sharding
    from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig
    from oracle_kernels import OracleKernels

    mine = sharding.local_images(n_img, info.world, info.rank)
    scene = synthetic.render_scene(ORBIT, H, W, device="cpu", tex_size=512, indices=mine)
    cfg = FrontEndConfig(kpts=KPTS, extract_chunk=2, pair_chunk=3)
    fe = AllPairsFrontEnd(scene.images, scene.intrinsics[:n_img], n_img, info.rank, info.world, info.device, cfg,
                          kernels=OracleKernels())
    return fe, fe.step()


GPU_H, GPU_W, GPU_KPTS = 480, 640, 1000


class HostGlooAllGather:
    """The all-gather of the packed feature blocks, staged through host memory and gloo (test rehearsal only)."""

    def __call__(self, block):
        world = dist.get_world_size()
        g = torch.empty(world * block.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(g, block.cpu())
        return g.view(world, block.numel()).to(block.device)


def run_frontend_gpu(n_img: int, rank: int, world: int, exchange=None):
    from gtsfm_amd import synthetic
    from gtsfm_amd.frontend import sharding
    from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig

    dev = torch.device("cuda", 0)
    mine = sharding.local_images(n_img, world, rank)
    scene = synthetic.render_scene(ORBIT, GPU_H, GPU_W, device=str(dev), tex_size=1024, indices=mine)
    cfg = FrontEndConfig(kpts=GPU_KPTS, pair_chunk=4)
    fe = AllPairsFrontEnd(scene.images.cpu(), scene.intrinsics[:n_img], n_img, rank, world, dev, cfg,
                          exchange=exchange if exchange is not None else HostGlooAllGather() if world > 1 else None)
    return fe, fe.step()


def run_rccl1(out_dir: str, n_img: int):
    """World-size-1 RCCL group: the packed exchange through the collective (pack -> all_gather_into_tensor ->
    unpack on device buffers), checked byte for byte here, then one engine step through it and one plain step."""
    from gtsfm_amd.frontend import sharding

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)  # before any other GPU call
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        gen = torch.Generator().manual_seed(0)
        xy = (torch.rand((3, 50, 2), generator=gen) * 1000).to(dev)
        desc = torch.randint(0, 256, (3, 50, 128), generator=gen).float().to(dev)
        cnt = torch.tensor([50, 7, 0], dtype=torch.int32, device=dev)
        checks = {}
        for n_per in (3, 5):  # exact and padded rank blocks
            got = sharding.allgather_features([xy, desc, cnt], n_per, wire=[None, torch.uint8, None],
                                              exchange=sharding.CollectiveAllGather())
            for name, a, b in zip(("xy", "desc", "cnt"), (xy, desc, cnt), got):
                assert b.device == dev and b.dtype == a.dtype and b.shape[0] == n_per, (name, b.shape)
                checks[f"{name}_{n_per}"] = bool(torch.equal(b[:3], a)) and bool((b[3:] == 0).all())
        torch.cuda.synchronize()
        _, r_c = run_frontend_gpu(n_img, 0, 1, exchange=sharding.CollectiveAllGather())
        save(os.path.join(out_dir, "rccl_collective.npz"), r_c)
        _, r_p = run_frontend_gpu(n_img, 0, 1)
        save(os.path.join(out_dir, "rccl_plain.npz"), r_p)
        with open(os.path.join(out_dir, "rccl_checks.json"), "w") as f:
            json.dump(checks, f)
    finally:
        dist.destroy_process_group()


def save(path, r):
    np.savez(path, pairs=r.pairs, R=r.R, t=r.t, status=r.status, n_inliers=r.n_inliers, n_matches=r.n_matches,
             isp_ok=r.isp_ok, offsets=r.offsets, v_corr=r.v_corr, kp_xy=r.kp_xy, kp_count=r.kp_count)


def main():
    mode, out_dir = sys.argv[1], sys.argv[2]
    if mode == "rccl1":
        run_rccl1(out_dir, int(sys.argv[3]))
        return
    if mode == "gpushared":
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        dist.init_process_group("gloo")
        try:
            _, r = run_frontend_gpu(int(sys.argv[3]), rank, world)
            save(os.path.join(out_dir, f"gpu_{world}_{rank}.npz"), r)
        finally:
            dist.destroy_process_group()
        return
    info = launch.init_rank("gloo")
    try:
        if mode == "probe":
            with open(os.path.join(out_dir, f"rank_{info.rank}.json"), "w") as f:
                json.dump({"rank": info.rank, "world": info.world, "local_rank": info.local_rank,
                           "dist_world": dist.get_world_size() if dist.is_initialized() else 1,
                           "device": str(info.device)}, f)
        else:
            fe, r = run_frontend(int(sys.argv[3]), info)
            save(os.path.join(out_dir, f"results_{info.world}_{info.rank}.npz"), r)
    finally:
        launch.finish_rank(info)


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
