#!/usr/bin/env python
"""bench.py — verified image-pairs/sec of the all-pairs two-view front-end on MI355X (BASELINE.json `metric`).

One step = the whole front-end over one synthetic scene already resident in HBM:
    SIFT (2048 kpts/img) on this rank's images -> [N>1: one all-gather of keypoints+descriptors over RCCL]
    -> mutual-NN + ratio matching of this rank's pairs (fp16 MFMA distance GEMM) -> 5-point RANSAC + LO +
    recoverPose of the same pairs -> inlier-support filter (>= 15 inliers, ratio >= 0.1), all on device.
value = all pairs pushed through match + verify (every rank) / max-over-ranks step time.

Workload (configs[1] of BASELINE.json): 100 rendered 1920x1080 images, all 4950 pairs, at N=1. For N GPUs the scene
grows to the smallest n with n(n-1)/2 >= 4950*N images (per-GPU pair work constant: "scaling": "weak"); pairs are
cut into one contiguous block per rank, images dealt round-robin for extraction.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--images n] [--kpts 2048] [--no-cpu-baseline]

--config c3-match: configs[2]'s matcher on SURVEY.md §8(d)'s synthetic descriptors -- 200 images x 4096 SuperPoint-like
256-D unit vectors (30 % of each image's rows planted from a shared latent set), all 19900 pairs through the fp16 MFMA
shortlist + certified exact re-rank (GTSFM_MATCH_F16_RERANK) with the ratio test; value = matched image-pairs/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from gtsfm_amd import device as hip  # noqa: E402
from gtsfm_amd import native, synthetic  # noqa: E402
from gtsfm_amd.frontend import sharding  # noqa: E402

MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
RATIO = 0.8
THRESH_PX = 4.0
MIN_INLIERS = 15
MIN_INLIER_RATIO = 0.1


def images_for(n_gpus: int, base: int = 100) -> int:
    target = base * (base - 1) // 2 * n_gpus
    n = base
    while n * (n - 1) // 2 < target:
        n += 1
    return n


class FrontEnd:
    """Device-resident all-pairs front-end for one rank."""

    def __init__(self, scene_images: torch.Tensor, intrinsics: np.ndarray, n_img: int, kpts: int, rank: int,
                 world: int):
        self.rank, self.world, self.kpts, self.n_img = rank, world, kpts, n_img
        self.dev = scene_images.device
        self.n_per = sharding.images_per_rank(n_img, world)
        self.local_images = scene_images  # (n_local, H, W, 3): images rank, rank + world, ...
        slot = sharding.global_slots(n_img, world)  # rank-major rows after the all-gather
        pairs = sharding.all_pairs(n_img)
        self.total_pairs = len(pairs)
        block = sharding.rank_pairs(pairs, world, rank)
        self.pair_id_base = int(block[0]) if len(block) else 0  # global pair index keys the RANSAC sampler
        mine = pairs[block]
        self.my_pairs_orig = mine
        self.pairs = torch.from_numpy(slot[mine].astype(np.int32)).to(self.dev)
        intr = np.zeros((world * self.n_per, 3))
        intr[slot] = intrinsics
        self.intr = torch.from_numpy(intr).to(self.dev)
        self.sift_ws = None

    def step(self, events=None):
        ev = events or {}
        if "t0" in ev:
            ev["t0"].record()
        feats = hip.sift_extract(self.local_images, self.kpts)
        if "t1" in ev:
            ev["t1"].record()
        # the one exchange step (N > 1): padded feature blocks, rank-major
        xy_all, desc_all, cnt_all = sharding.allgather_features((feats.xy, feats.desc, feats.count), self.n_per)
        if "t2" in ev:
            ev["t2"].record()
        idx, mcnt = hip.match_pairs(desc_all, cnt_all, self.pairs, RATIO, native.GTSFM_MATCH_INT_F16)
        if "t3" in ev:
            ev["t3"].record()
        res = hip.ransac_essential(xy_all, self.intr, self.pairs, idx, mcnt, THRESH_PX,
                                   pair_id_base=self.pair_id_base)
        if "t4" in ev:
            ev["t4"].record()
        # inlier-support processor (frontend/inlier_support_processor.py:73-87), on device
        m = mcnt.clamp(min=1).to(torch.float64)
        ratio = res.n_inliers.to(torch.float64) / m
        ok = (res.status == native.RANSAC_STATUS_OK) & (ratio >= MIN_INLIER_RATIO) & (res.n_inliers >= MIN_INLIERS)
        n_ok = ok.sum()
        return n_ok, (feats, idx, mcnt, res)


def pmc_traffic():
    """HBM bytes per mnn_mfma_kernel launch from the committed rocprofv3 --pmc summary of this bench's command
    (profiles/*_mnn_pmc.json, written by tools/pmc_summary.py --json): FETCH_SIZE doubled per MI355X_MICROARCH.md
    (gfx950 tallies 128-B reads at 64 B) + WRITE_SIZE, in bytes. None when no summary is committed."""
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_mnn_pmc.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return float(d["hbm_bytes_per_launch"]), os.path.relpath(files[-1], REPO)


def cpu_baseline(scene, kpts: int, threads: int = 16, n_sift: int = 16, n_pairs: int = 64) -> dict:
    """Oracle restatement (oracle/*.c through ctypes, which drops the GIL) timed on `threads` host threads -- the
    box's CPU share for one GPU -- over a bounded sample: SIFT of n_sift images, then match + verify of n_pairs pairs
    among them, each stage wall-clocked across the thread pool and scaled to the full workload."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle

    n_sift = min(n_sift, scene.images.shape[0])
    imgs = scene.images[:n_sift].cpu().numpy()
    K = scene.K
    rng = np.random.default_rng(0)
    oracle.ransac_E(rng.normal(size=(8, 2)), rng.normal(size=(8, 2)), 1e-3)  # one-time solver tables, untimed
    pairs = [(i1, i2) for i1 in range(n_sift) for i2 in range(i1 + 1, n_sift)][:n_pairs]

    def sift_one(im):
        return oracle.sift(oracle.rgb_to_gray(im), kpts)

    def pair_one(p):
        f1, f2 = feats[p[0]], feats[p[1]]
        m = oracle.twoway_match(f1[1], f2[1], RATIO)
        if len(m) >= 6:
            x1 = ((f1[0][m[:, 0], :2] - K[:2, 2]) / K[0, 0]).astype(np.float64)
            x2 = ((f2[0][m[:, 1], :2] - K[:2, 2]) / K[0, 0]).astype(np.float64)
            oracle.ransac_E(x1, x2, THRESH_PX / K[0, 0])

    with ThreadPoolExecutor(threads) as pool:
        t0 = time.time()
        feats = list(pool.map(sift_one, imgs))
        t_sift = (time.time() - t0) / n_sift
        t0 = time.time()
        list(pool.map(pair_one, pairs))
        t_pair = (time.time() - t0) / len(pairs)
    n_img = scene.images.shape[0]
    P = n_img * (n_img - 1) // 2
    total = n_img * t_sift + P * t_pair
    return {"value": P / total, "unit": "verified image-pairs/sec", "cores": threads, "kind": "port",
            "sample": f"oracle (oracle/*.c, {threads} threads): SIFT of {n_sift} of the {n_img} images "
                      f"({t_sift * 1e3:.0f} ms/img wall) + match+verify of {len(pairs)} pairs among them "
                      f"({t_pair * 1e3:.0f} ms/pair wall), scaled to {n_img} images / {P} pairs"}


def c3_descriptors(n_img: int, k: int, d: int, dev) -> torch.Tensor:
    """SuperPoint-like unit descriptors with planted matches (seeded; SURVEY.md 8(d) matcher microbench)."""
    g = torch.Generator(device=dev).manual_seed(3)
    latent = torch.nn.functional.normalize(torch.randn(k, d, device=dev, generator=g), dim=1)
    desc = torch.nn.functional.normalize(torch.randn(n_img, k, d, device=dev, generator=g), dim=2)
    m = int(0.3 * k)
    for i in range(n_img):
        rows = torch.randperm(k, device=dev, generator=g)[:m]
        src = torch.randperm(k, device=dev, generator=g)[:m]
        noise = 0.15 / d ** 0.5 * torch.randn(m, d, device=dev, generator=g)
        desc[i, rows] = torch.nn.functional.normalize(latent[src] + noise, dim=1)
    return desc.contiguous()


def c3_cpu_baseline(desc: torch.Tensor, threads: int = 16, n_pairs: int = 16) -> dict:
    """Oracle TwoWayMatcher restatement (oracle/twoway.c) on `threads` host threads over n_pairs pairs."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle

    h = desc[: n_pairs + 1].cpu().numpy()
    pairs = [(0, j) for j in range(1, n_pairs + 1)]
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.time()
        list(pool.map(lambda p: oracle.twoway_match(h[p[0]], h[p[1]], RATIO), pairs))
        dt = time.time() - t0
    return {"value": len(pairs) / dt, "unit": "matched image-pairs/s", "cores": threads, "kind": "port",
            "sample": f"oracle twoway_match (oracle/twoway.c, {threads} threads), {len(pairs)} pairs of "
                      f"{h.shape[1]}x{h.shape[2]} descriptors, {dt:.1f} s wall"}


def main_c3(args, world, rank, dev):
    """configs[2] matcher: all pairs of 200 x 4096 x 256-D float descriptors, F16_RERANK + ratio 0.8."""
    n_img, k, d = args.images or 200, args.kpts if args.kpts != 2048 else 4096, 256
    desc = c3_descriptors(n_img, k, d, dev)
    cnt = torch.full((n_img,), k, dtype=torch.int32, device=dev)
    all_pairs = sharding.all_pairs(n_img)
    mine = all_pairs[sharding.rank_pairs(all_pairs, world, rank)]
    pairs = torch.from_numpy(mine.astype(np.int32)).to(dev)
    mode = native.GTSFM_MATCH_F16_RERANK

    def step():
        return hip.match_pairs(desc, cnt, pairs, RATIO, mode)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, m = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    total_pairs = len(all_pairs)
    # shortlist GEMM kernel timed on the call's stream (median of 3)
    lib = native.lib()
    kms = []
    for _ in range(3):
        kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for e in kev:
            e.record()
        native.check(lib.gtsfm_match_set_kernel_events(kev[0].cuda_event, kev[1].cuda_event), "set_kernel_events")
        step()
        torch.cuda.synchronize()
        native.check(lib.gtsfm_match_set_kernel_events(None, None), "set_kernel_events")
        kms.append(kev[0].elapsed_time(kev[1]))
    kernel_ms = float(np.median(kms))
    flops = 2 * 2.0 * k * k * d * len(mine)
    tf = flops / (kernel_ms * 1e-3) / 1e12
    out = {
        "metric": "matched image-pairs/sec (all-pairs SuperPoint-descriptor matching, configs[2])",
        "value": round(total_pairs / (elapsed / args.steps), 2), "unit": "image-pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak" if world > 1 else "strong", "vs_baseline": None,
        "dtype": "fp16 MFMA shortlist / fp32 exact re-rank", "data": "synthetic (seeded unit Gaussian, 30% planted)",
        "config": {"workload": f"C3 matcher: {n_img} images x {k} x {d}-D float descriptors, all {total_pairs} "
                               f"pairs, mutual NN + ratio {RATIO}", "images": n_img, "pairs": total_pairs, "kpts": k,
                   "parallelism": f"pair blocks x{world}"},
        "mean_matches": round(float(m.float().mean().item()), 1),
        "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": None,
                     "kernel": "fl_shortlist_kernel<16> (one launch per step)", "kernel_ms": round(kernel_ms, 3),
                     "work": "2 sides x 2*K1*K2*D flop per pair"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = c3_cpu_baseline(desc)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--images", type=int, default=0)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--kpts", type=int, default=2048)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", default="c2", choices=["c2", "c3-match"])
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    native.lib()
    if args.config == "c3-match":
        return main_c3(args, world, rank, dev)
    n_img = args.images or images_for(world)

    # every rank renders the same seeded scene but keeps only its own images resident
    scene = synthetic.render_scene(n_img, args.height, args.width, device=str(dev))
    local = scene.images[rank::world].contiguous()
    fe = FrontEnd(local, scene.intrinsics, n_img, args.kpts, rank, world)
    if rank != 0 or world > 1 or args.no_cpu_baseline:
        keep_for_cpu = None
    else:
        keep_for_cpu = scene
    del scene
    torch.cuda.empty_cache()

    for _ in range(args.warmup):
        fe.step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_ok = None
    for _ in range(args.steps):
        n_ok, _ = fe.step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    ok = n_ok.to(torch.float64).reshape(1)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.SUM)
    elapsed = float(el.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = fe.total_pairs / (elapsed / args.steps)

    # stage split + roofline of the dominant kernel. HIP events on the stream the kernels run on (torch's current
    # stream): stage events from Python, the distance-GEMM kernel's own pair through gtsfm_match_set_kernel_events.
    names = ["t0", "t1", "t2", "t3", "t4"]
    stage_ms = {"extract": [], "allgather": [], "match": [], "verify": []}
    kernel_ms = []
    lib = native.lib()
    for _ in range(5):
        evs = {k: torch.cuda.Event(enable_timing=True) for k in names}
        kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for e in kev:
            e.record()  # creates the hipEvent_t handle
        native.check(lib.gtsfm_match_set_kernel_events(kev[0].cuda_event, kev[1].cuda_event), "set_kernel_events")
        _, (feats, idx, mcnt, res) = fe.step(evs)
        torch.cuda.synchronize()
        native.check(lib.gtsfm_match_set_kernel_events(None, None), "set_kernel_events")
        kernel_ms.append(kev[0].elapsed_time(kev[1]))
        stage_ms["extract"].append(evs["t0"].elapsed_time(evs["t1"]))
        stage_ms["allgather"].append(evs["t1"].elapsed_time(evs["t2"]))
        stage_ms["match"].append(evs["t2"].elapsed_time(evs["t3"]))
        stage_ms["verify"].append(evs["t3"].elapsed_time(evs["t4"]))
    # medians over the instrumented steps (a single step can catch a clock or paging transient)
    stage = {k: float(np.median(v)) for k, v in stage_ms.items()}
    mnn_ms = float(np.median(kernel_ms))
    counts = feats.count
    (counts_all,) = sharding.allgather_features((counts,), fe.n_per)
    c = counts_all.to(torch.float64)
    pairs = fe.pairs.long()
    match_flops = float((2.0 * c[pairs[:, 0]] * c[pairs[:, 1]] * 128).sum().item())
    match_tflops = match_flops / (mnn_ms * 1e-3) / 1e12
    # algorithmic bytes of the launch: both fp16 operand forms of every image once + the per-keypoint top-2 records
    kpad = -(-args.kpts // 256) * 256
    n_rows = world * fe.n_per
    algo_bytes = 2 * n_rows * kpad * 144 * 2 + 2 * len(pairs) * args.kpts * 8
    traffic = pmc_traffic()
    roof = {"bound": "mfma", "achieved": round(match_tflops, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(match_tflops / MFMA_F16_PEAK_TFLOPS, 4), "traffic": traffic[0] if traffic else None,
            "traffic_source": traffic[1] if traffic else None, "algorithmic_bytes": algo_bytes,
            "kernel": "mnn_mfma_kernel (one launch per step)", "kernel_ms": round(mnn_ms, 3),
            "work": "2*K1*K2*128 flop per pair, summed over the launch's pairs (GFLOP: %.1f)" % (match_flops / 1e9)}
    if traffic:
        # FETCH_SIZE counts L2 -> fabric requests, Infinity Cache hits included (MI355X_MICROARCH.md, HBM section)
        roof["traffic_note"] = ("L2-miss bytes, Infinity-Cache hits included: the A operand (image i2) of each pair is "
                                "re-read past the 4 MiB XCD L2, from a %.0f MB operand set that fits the 256 MiB "
                                "Infinity Cache; %.2f TB/s at kernel_ms, not the bound"
                                % (2 * n_rows * kpad * 144 * 2 / 1e6, traffic[0] / (mnn_ms * 1e-3) / 1e12))

    out = {
        "metric": "verified image-pairs/sec (all-pairs front-end), N images @ 2048 kpts/img",
        "value": round(value, 2),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8 image / fp32 pyramid / fp16-MFMA exact-int distances / fp64 RANSAC solver",
        "data": "synthetic (rendered textured room, seeds 0/1/2)",
        "config": {"workload": f"C2: {n_img} synthetic {args.width}x{args.height} images, all "
                               f"{fe.total_pairs} pairs, SIFT {args.kpts} kpts/img, ratio {RATIO}, "
                               f"5-pt RANSAC {THRESH_PX}px", "images": n_img, "pairs": fe.total_pairs,
                   "kpts": args.kpts, "parallelism": f"pair blocks x{world}"},
        "pairs_passing_isp": int(ok.item()),
        "stage_ms": {k: round(v, 3) for k, v in stage.items()},
        "roofline": roof,
    }
    if keep_for_cpu is not None:
        out["cpu_baseline"] = cpu_baseline(keep_for_cpu, args.kpts)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
