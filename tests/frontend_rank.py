"""Child-process body for tests/test_launcher.py: one rank of a gloo job started by gtsfm_amd.launch.spawn_ranks.

    python tests/frontend_rank.py probe OUT_DIR            -> writes rank_<r>.json with what init_rank saw
    python tests/frontend_rank.py frontend OUT_DIR N_IMG   -> runs AllPairsFrontEnd (oracle kernels) and saves
                                                              results_<world>_<rank>.npz
    python tests/frontend_rank.py gpushared OUT_DIR N_IMG  -> every rank on cuda:0 with the HIP kernels (a one-GPU box
                                                              rehearsal of the multi-rank engine); the exchange is the
                                                              engine's packing with the blocks gathered over gloo on
                                                              the host (RCCL refuses two ranks on one GPU)
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


def run_frontend_gpu(n_img: int, rank: int, world: int):
    from gtsfm_amd import synthetic
    from gtsfm_amd.frontend import sharding
    from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig

    dev = torch.device("cuda", 0)
    mine = sharding.local_images(n_img, world, rank)
    scene = synthetic.render_scene(ORBIT, GPU_H, GPU_W, device=str(dev), tex_size=1024, indices=mine)
    cfg = FrontEndConfig(kpts=GPU_KPTS, pair_chunk=4)
    fe = AllPairsFrontEnd(scene.images.cpu(), scene.intrinsics[:n_img], n_img, rank, world, dev, cfg,
                          exchange=HostGlooAllGather() if world > 1 else None)
    return fe, fe.step()


def save(path, r):
    np.savez(path, pairs=r.pairs, R=r.R, t=r.t, status=r.status, n_inliers=r.n_inliers, n_matches=r.n_matches,
             isp_ok=r.isp_ok, offsets=r.offsets, v_corr=r.v_corr, kp_xy=r.kp_xy, kp_count=r.kp_count)


def main():
    mode, out_dir = sys.argv[1], sys.argv[2]
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
