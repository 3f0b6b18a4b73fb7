"""Child-process body for tests/test_launcher.py: one rank of a gloo job started by gtsfm_amd.launch.spawn_ranks.

    python tests/frontend_rank.py probe OUT_DIR            -> writes rank_<r>.json with what init_rank saw
    python tests/frontend_rank.py frontend OUT_DIR N_IMG   -> runs AllPairsFrontEnd (oracle kernels) and saves
                                                              results_<world>_<rank>.npz
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


def main():
    mode, out_dir = sys.argv[1], sys.argv[2]
    info = launch.init_rank("gloo")
    try:
        if mode == "probe":
            with open(os.path.join(out_dir, f"rank_{info.rank}.json"), "w") as f:
                json.dump({"rank": info.rank, "world": info.world, "local_rank": info.local_rank,
                           "dist_world": dist.get_world_size() if dist.is_initialized() else 1,
                           "device": str(info.device)}, f)
        else:
            fe, r = run_frontend(int(sys.argv[3]), info)
            np.savez(os.path.join(out_dir, f"results_{info.world}_{info.rank}.npz"), pairs=r.pairs, R=r.R, t=r.t,
                     status=r.status, n_inliers=r.n_inliers, n_matches=r.n_matches, isp_ok=r.isp_ok,
                     offsets=r.offsets, v_corr=r.v_corr, kp_xy=r.kp_xy, kp_count=r.kp_count)
    finally:
        launch.finish_rank(info)


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
