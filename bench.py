#!/usr/bin/env python
"""bench.py — verified image-pairs/sec of the all-pairs two-view front-end on MI355X (BASELINE.json `metric`).

One step = one pass of the front-end over this rank's images (gtsfm_amd/frontend/all_pairs.py). In its
host-to-host form (images in pinned host memory -> per-pair (R, t, v_corr, inlier count) in host
memory):
    H2D of the images in chunks on a copy stream, overlapped with SIFT (2048 kpts/img) of the previous chunk
    -> [N>1: one all-gather of keypoints + descriptors over RCCL] -> mutual-NN + ratio matching of this rank's pairs
    (fp16 MFMA distance GEMM) -> 5-point RANSAC + LO + recoverPose -> compaction of the verified rows + the
    inlier-support filter (>= 15 inliers, ratio >= 0.1) -> D2H of the compact results.
value = all pairs pushed through match + verify (every rank) / max-over-ranks step time, with the images already
resident in HBM when the timed region starts and the results left there (the prompt's measurement rule). The same
steps from pinned host images to host results (SURVEY.md §8(d)'s PCIe-inclusive unit) are timed as well and reported
as `value_host_to_host`.

Workloads:
  --config c2 (default; configs[1] of BASELINE.json): 100 rendered 1920x1080 images, all 4950 pairs. N GPUs share
      that same scene (images round-robin, pairs in N blocks: "scaling": "strong").
  --config c2-weak: the scene grows to the smallest n with n(n-1)/2 >= 4950*N images (per-GPU pair work constant,
      per-GPU extraction falls as 100/sqrt(N): not a constant-work curve, kept for comparison).
  --config c1 (configs[0]): the reference's 12 Lund Door images (1296x1936, tests/golden/lund_door), all 66 pairs,
      sift_front_end.yaml's 5000 keypoints; cpu_baseline is the oracle on the whole workload, nothing extrapolated.
  --config c4 (configs[3]): 1000 rendered 1080p images, all 499,500 pairs, split over the N ranks ("strong").
  --config c3-match: configs[2]'s matcher on SURVEY.md §8(d)'s synthetic descriptors -- 200 images x 4096
      SuperPoint-like 256-D unit vectors, all 19900 pairs through the fp16 MFMA shortlist + certified exact re-rank.
  --config c3: configs[2] end to end -- HIP SuperPoint (4096 kpts, seeded random weights) on 200 rendered 1080p
      images, then all pairs through the same matcher.
  --config c5: a per-GPU slice of configs[4] -- SuperPoint (2048 kpts) + SuperGlue + 5-point RANSAC over all pairs
      of 32 rendered images (configs[4]'s 2000 images x 8 GPUs is ~2M SuperGlue pairs; --images sets the slice).
  --config netvlad: SURVEY §8 f3 -- NetVLAD global descriptors of 64 rendered 1080p images + the retriever's
      similarity / top-20 pairs (images/s; not a BASELINE config).
Pairs and images are dealt round-robin over the ranks (pair p to rank p mod N, image i to rank i mod N).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c2-weak|c4|c3-match|c3|c5] [--images n]
                    [--no-cpu-baseline]

--gpus N > 1 without a launcher starts N fresh rank processes first (gtsfm_amd/launch.py), before anything touches
a GPU; under `torch.distributed.run` the ranks come from the environment.
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

from gtsfm_amd import launch  # noqa: E402

# everything that may touch the GPU is imported lazily, after the launcher has run (see main)

MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0  # HBM3E spec, MI355X_MICROARCH.md
VALU_F32_PEAK_TFLOPS = 157.3  # vector fp32, MI355X_MICROARCH.md (SURVEY.md §8(d) grades RANSAC against it)
VALU_F64_PEAK_TFLOPS = 78.6  # vector fp64, AMD's MI355X spec (half the fp32 vector rate; not in MI355X_MICROARCH.md)
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


def pmc_traffic(config: str):
    """HBM bytes per mnn_pp_kernel launch (the distance GEMM) of THIS config's bench command, from the latest committed
    rocprofv3 --pmc summary for it (profiles/*_<config>_mnn_pmc.json, tools/gpu_pmc_mnn.sh TAG bench <config>;
    for c2 also the untagged profiles/*_mnn_pmc.json of rounds 1-5, which were all taken on the c2 command):
    FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B reads at 64 B) + WRITE_SIZE, in bytes.
    None when no summary of this config is committed (never another config's figure)."""
    import glob
    import re

    files = glob.glob(os.path.join(REPO, "profiles", f"*_{config}_mnn_pmc.json"))
    if config == "c2":
        files += [f for f in glob.glob(os.path.join(REPO, "profiles", "*_mnn_pmc.json"))
                  if re.fullmatch(r"r\d+[a-z]*_mnn_pmc\.json", os.path.basename(f))]
    if not files:
        return None
    latest = max(files, key=lambda f: os.path.basename(f).split("_")[0])
    with open(latest) as f:
        d = json.load(f)
    return float(d["hbm_bytes_per_launch"]), os.path.relpath(latest, REPO)


def deep_pmc(config: str):
    """The latest committed per-kernel PMC summary of a deep config (profiles/*_<config>_pmc.json, written by
    tools/gpu_pmc_deep.sh through tools/pmc_summary.py --kernels): HBM bytes per launch per kernel (FETCH_SIZE doubled +
    WRITE_SIZE, as pmc_traffic) and the profiled step count. None when none is committed."""
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_{config}_pmc.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    d["source"] = os.path.relpath(files[-1], REPO)
    return d


def cpu_baseline(images, intrinsics: np.ndarray, n_img: int, kpts: int, threads: int = 16, n_sift: int = 16,
                 n_pairs: int = 120) -> dict:
    """Oracle restatement (oracle/*.c through ctypes, which drops the GIL) timed on `threads` host threads -- the
    box's CPU share for one GPU -- over a bounded sample: SIFT of n_sift images spread evenly over the scene's n_img
    (so the pairs among them span the same range of baselines as all pairs of the scene), then match + verify of up to
    n_pairs of the pairs among them (a seeded choice when there are more), each stage wall-clocked across the pool and
    scaled to n_img images / all their pairs. When the sample is the whole workload (C1) nothing is scaled.
    `images` holds the sampled images' pixels: (n_sift, H, W, 3) in the order of sample_images(n_img, n_sift)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle

    sample = sample_images(n_img, n_sift)
    imgs = np.asarray(images)
    assert imgs.shape[0] == len(sample)
    rng = np.random.default_rng(0)
    oracle.ransac_E(rng.normal(size=(8, 2)), rng.normal(size=(8, 2)), 1e-3)  # one-time solver tables, untimed
    pairs = [(a, b) for a in range(len(sample)) for b in range(a + 1, len(sample))]
    if len(pairs) > n_pairs:
        pairs = [pairs[i] for i in sorted(rng.choice(len(pairs), n_pairs, replace=False))]
    K = np.asarray(intrinsics, dtype=np.float64)

    def sift_one(im):
        return oracle.sift(oracle.rgb_to_gray(im), kpts)

    def pair_one(p):
        f1, f2 = feats[p[0]], feats[p[1]]
        k1, k2 = K[sample[p[0]]], K[sample[p[1]]]
        m = oracle.twoway_match(f1[1], f2[1], RATIO)
        if len(m) >= 6:
            x1 = ((f1[0][m[:, 0], :2] - k1[1:3]) / k1[0]).astype(np.float64)
            x2 = ((f2[0][m[:, 1], :2] - k2[1:3]) / k2[0]).astype(np.float64)
            oracle.ransac_E(x1, x2, THRESH_PX / max(k1[0], k2[0]))

    with ThreadPoolExecutor(threads) as pool:
        t0 = time.time()
        feats = list(pool.map(sift_one, imgs))
        t_sift_wall = time.time() - t0
        t0 = time.time()
        list(pool.map(pair_one, pairs))
        t_pair_wall = time.time() - t0
    P = n_img * (n_img - 1) // 2
    whole = len(sample) == n_img and len(pairs) == P
    total = t_sift_wall + t_pair_wall if whole else (n_img * t_sift_wall / len(sample) + P * t_pair_wall / len(pairs))
    if whole:
        what = (f"oracle (oracle/*.c, {threads} threads): the whole workload, SIFT of all {n_img} images "
                f"({t_sift_wall:.2f} s wall) + match+verify of all {P} pairs ({t_pair_wall:.2f} s wall), no scaling")
    else:
        what = (f"oracle (oracle/*.c, {threads} threads): SIFT of {len(sample)} of the {n_img} images, evenly spaced "
                f"({t_sift_wall / len(sample) * 1e3:.0f} ms/img wall) + match+verify of {len(pairs)} pairs among them "
                f"({t_pair_wall / len(pairs) * 1e3:.0f} ms/pair wall), scaled to {n_img} images / {P} pairs")
    return {"value": P / total, "unit": "verified image-pairs/sec", "cores": threads,
            "kind": "port" if whole else "port, extrapolated", "sample": what}


def sample_images(n_img: int, n_sift: int) -> np.ndarray:
    """n_sift image indices spread evenly over [0, n_img) (all of them when n_img <= n_sift)."""
    if n_img <= n_sift:
        return np.arange(n_img)
    return np.unique(np.round(np.linspace(0, n_img - 1, n_sift)).astype(np.int64))


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
    return {"value": len(pairs) / dt, "unit": "matched image-pairs/s", "cores": threads, "kind": "port, extrapolated",
            "sample": f"oracle twoway_match (oracle/twoway.c, {threads} threads), {len(pairs)} pairs of "
                      f"{h.shape[1]}x{h.shape[2]} descriptors, {dt:.1f} s wall"}


def main_c3(args, world, rank, dev):
    """configs[2] matcher: all pairs of 200 x 4096 x 256-D float descriptors, F16_RERANK + ratio 0.8."""
    from gtsfm_amd import device as hip
    from gtsfm_amd import native
    from gtsfm_amd.frontend import sharding

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
    flops = 2.0 * k * k * d * len(mine)  # the distance matrix counted once per pair
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
                     "work": "2*K1*K2*D flop per pair (the kernel computes the matrix once per side: 2x this)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = c3_cpu_baseline(desc)
    if rank == 0:
        print(json.dumps(out), flush=True)




def vgg16_conv_flop(H: int, W: int) -> float:
    """Multiply-add flop (2 per MAC) of VGG16 features[:-2] on an H x W image (13 conv3x3, pools floor)."""
    layers = [(3, 64, 0), (64, 64, 1), (64, 128, 0), (128, 128, 1), (128, 256, 0), (256, 256, 0), (256, 256, 1),
              (256, 512, 0), (512, 512, 0), (512, 512, 1), (512, 512, 0), (512, 512, 0), (512, 512, 0)]
    h, w, total = H, W, 0.0
    for cin, cout, pool in layers:
        total += 2.0 * 9 * cin * cout * h * w
        if pool:
            h, w = h // 2, w // 2
    return total


def main_netvlad(args, world, rank, dev):
    """SURVEY §8 row f3 (retrieval), the descriptor half: NetVLAD global descriptors (VGG16 + NetVLAD layer +
    whitening, netvlad_global_descriptor.py / thirdparty/hloc/netvlad.py) of n rendered 1080p images resident in HBM,
    then the NetVLAD retriever's similarity GEMM + top-k pairs (netvlad_retriever.py:77-228, num_matched 20, min_score
    0.3 as sift_front_end.yaml). Seeded random weights (tests/netvlad_weights.py). Images dealt round-robin over ranks;
    each rank describes its own images (replicas: no exchange is timed)."""
    from gtsfm_amd import device as hip
    from gtsfm_amd import native, synthetic
    from gtsfm_amd.frontend.global_descriptor.netvlad_global_descriptor import WORKSPACE_BUDGET, pack_netvlad_weights
    from gtsfm_amd.frontend import sharding

    sys.path.insert(0, os.path.join(REPO, "tests"))
    from netvlad_weights import netvlad_state_dict

    n_img = args.images or 64
    H, W = args.height, args.width
    mine = sharding.local_images(n_img, world, rank)
    scene = synthetic.render_scene(n_img, H, W, device=str(dev), indices=mine)
    imgs = scene.images.contiguous()
    sd = netvlad_state_dict(0)
    w = torch.from_numpy(pack_netvlad_weights(sd)).to(dev)
    lib = native.lib()
    per = int(lib.gtsfm_netvlad_workspace_bytes(1, H, W))
    g = max(1, min(len(mine), WORKSPACE_BUDGET // per))
    ws = torch.empty(int(lib.gtsfm_netvlad_workspace_bytes(g, H, W)), dtype=torch.uint8, device=dev)
    out = torch.empty((len(mine), 4096), dtype=torch.float32, device=dev)

    def step():
        for s0 in range(0, len(mine), g):
            d, _ = hip.netvlad_describe(imgs[s0: s0 + g], w, workspace=ws)
            out[s0: s0 + g] = d
        if world == 1:
            sim = hip.retrieval_similarity(out, 50)
            return hip.retrieval_pairs(sim, 20, 0.3)
        return None

    for _ in range(args.warmup):
        step()
    elapsed = timed_loop(step, args.steps, world, dev)
    # the descriptor stage alone, timed with events on the compute stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for s0 in range(0, len(mine), g):
        hip.netvlad_describe(imgs[s0: s0 + g], w, workspace=ws)
    ev[1].record()
    torch.cuda.synchronize()
    desc_ms = ev[0].elapsed_time(ev[1])
    flop = len(mine) * vgg16_conv_flop(H, W)
    tf = flop / (desc_ms * 1e-3) / 1e12
    split_peak = MFMA_F16_PEAK_TFLOPS / 6.0
    value = n_img / (elapsed / args.steps)
    out_line = {
        "metric": "NetVLAD global descriptors + retrieval pairs, images/sec (f3)",
        "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak" if world > 1 else "strong", "vs_baseline": None,
        "dtype": "u8 image / fp32-accurate bf16x3-MFMA VGG16 / fp32 MFMA VLAD + whitening",
        "data": "synthetic (rendered textured room); seeded random NetVLAD weights (tests/netvlad_weights.py)",
        "config": {"workload": f"f3: {n_img} synthetic {W}x{H} images -> NetVLAD 4096-D descriptors -> "
                               "similarity + top-20 pairs (min_score 0.3)", "images": n_img,
                   "parallelism": f"images x{world}"},
        "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": round(split_peak, 1), "unit": "TFLOP/s",
                     "frac": round(tf / split_peak, 4), "traffic": None, "kernel_ms": round(desc_ms, 3),
                     "kernel": "NetVLAD descriptor launches (conv3_kernel x 12 + input conv + VLAD + whitening)",
                     "work": "VGG16 features[:-2] conv flop %.1f GFLOP per image (2 per MAC) over %d images; convs "
                             "as fp32-accurate bf16x3 split products (peak = dense bf16 MFMA / 6)"
                             % (vgg16_conv_flop(H, W) / 1e9, len(mine))},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import deep

        torch.set_num_threads(16)
        host = imgs[:2].cpu().numpy()
        t0 = time.time()
        for im in host:
            deep.netvlad(im, sd)
        dt = (time.time() - t0) / len(host)
        out_line["cpu_baseline"] = {"value": round(1.0 / dt, 4), "unit": "images/s", "cores": 16,
                                    "kind": "port, extrapolated",
                                    "sample": f"oracle/deep.py netvlad (torch fp32, 16 threads) on 2 of the images: "
                                              f"{dt:.2f} s/image"}
    if rank == 0:
        print(json.dumps(out_line), flush=True)


def timed_loop(step, steps: int, world: int, dev) -> float:
    """Seconds for `steps` calls of step(): barrier + synchronize on both sides, max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    return float(el.item())


def timed_steps(fe, steps: int, resident: bool, world: int, dev) -> float:
    """Seconds for `steps` steps: barrier + synchronize on both sides, max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fe.step(resident=resident)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    return float(el.item())


def sift_bytes_per_image(H: int, W: int, kpts: int) -> float:
    """SURVEY.md §8(d) algorithmic bytes of SIFT extraction per image: 84 * sum_o P_o + H*W + K*(128*4 + 16), with
    sum_o P_o = 4HW * 4/3 (21 fp32 image passes per pyramid pixel over the 2x-upsampled octave pyramid)."""
    return 84.0 * (4.0 * H * W * 4.0 / 3.0) + H * W + kpts * (128 * 4 + 16)


def sift_moved_bytes_per_image(H: int, W: int, kpts: int) -> float:
    """Bytes the SIFT kernels actually move per image (beside §8(d)'s 84 B per pyramid pixel, which counts DoG
    writes and reads that no kernel performs: DoG is formed in LDS / registers): the u8 RGB read and octave 0's base
    level write (gray + 2x upsample + first blur fused), per octave pixel 5 level blurs read + written (40 B), the six
    levels read by the extrema sweep (24 B) and the next octave's base written by the layer-3 blur (1 B per pixel of
    this octave), plus the keypoint records and descriptors written."""
    P = 4.0 * H * W * 4.0 / 3.0  # sum over octaves of the level pixel counts (octave 0 is the 2x-upsampled image)
    return 3.0 * H * W + 4.0 * (4.0 * H * W) + 65.0 * P + kpts * (128 * 4 + 16)


def lund_door_c1():
    """configs[0] (C1): the reference's 12 Lund Door images (tests/data/set1_lund_door, committed byte for byte under
    tests/golden/lund_door/ with their data.mat intrinsics in gt.json), decoded with PIL as the reference loader
    does. 1296 x 1936: max_resolution 1296, the reference CI benchmark's setting, needs no resize."""
    from PIL import Image as PILImage

    root = os.path.join(REPO, "tests", "golden", "lund_door")
    gt = json.load(open(os.path.join(root, "gt.json")))
    imgs = np.stack([np.asarray(PILImage.open(os.path.join(root, n)).convert("RGB")) for n in gt["images"]])
    intr = np.tile(np.asarray(gt["fx_u0_v0"], dtype=np.float64), (len(imgs), 1))
    return torch.from_numpy(imgs), intr


SP_FLOP_PER_PIXEL = 169600.0   # SuperPoint convs ~169,600 FLOP per input pixel (352 GF at 1080p)
SG_FLOP_PER_PAIR_2048 = 254e9   # SuperGlue ~254 GFLOP per pair at K = 2048
# The deep networks compute fp32-accurate products as six bf16 plane products (three-way bf16 split of each fp32
# operand): their ceiling is the dense bf16 MFMA rate (= the fp16 rate) / 6 in fp32-equivalent FLOP/s.


def superglue_flop(k1: np.ndarray, k2: np.ndarray) -> np.ndarray:
    """SURVEY.md 8(d)'s per-pair count 18 * 2 * (20 K d^2 + 4 K^2 d) + 2 K^2 d at K1, K2 keypoints (d = 256), per side
    summed: the projections / MLPs scale with each side's K, the attention and the score matrix with K1 K2."""
    d = 256.0
    lin = 18 * 2 * 20 * d * d * (k1 + k2) / 2.0
    quad = 18 * 2 * 4 * d * k1 * k2 + 2 * d * k1 * k2
    return lin + quad


def deep_weights(dev, superglue: bool, head=True):
    """Seeded random SuperPoint / SuperGlue weights in the ABI's packed layout (the pretrained .pth files are not
    available offline; tests/superpoint_weights.py builds state dicts of the reference architectures). SuperPoint's
    1x1 descriptor layer is the whitening of its seeded encoder's activations over the benchmark scene
    (tests/golden/make_superpoint_whitening.py), so descriptors of the scene behave like trained ones (unrelated
    keypoints near-orthogonal, repeated points similar); SuperGlue's final projection gain is 24 (see
    superglue_state_dict), which gives ~1000 matches on adjacent views. For SuperPoint + SuperGlue the weights change
    what is matched, not the work of a step (every kernel's size is set by the keypoint counts). For C3's
    F16_RERANK matcher they DO change the work: how clustered the descriptors are decides how many keypoints the fp16
    shortlist certifies and how many go to the exact rescans (0.75 s per step with the C3 head against 4.5 s with the
    rank-32 head). C3 (TwoWayMatcher: mutual NN + ratio test, no context) uses the head fitted to its strafe scene,
    head="c3" (32 leading principal directions whitened, the rest at a quarter weight: ~185 putatives per pair, 95 %
    of the pairs verified); since round 4 C3 is that strafe scene with that head, a different workload from round
    3's orbit scene."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from superpoint_weights import superglue_state_dict, superpoint_state_dict

    from gtsfm_amd.frontend.detector_descriptor.superpoint import pack_superpoint_weights

    sd = superpoint_state_dict(0, whitened=head)
    sp = torch.from_numpy(pack_superpoint_weights(sd)).to(dev)
    if not superglue:
        return sd, sp, None, None
    from gtsfm_amd.frontend.matcher.superglue_matcher import pack_superglue_weights

    sgd = superglue_state_dict(0, final_scale=24.0)
    return sd, sp, sgd, torch.from_numpy(pack_superglue_weights(sgd)).to(dev)


def deep_sample(config: str) -> int:
    """Images in the deep configs' CPU-baseline sample: 7 for C3 (21 pairs, ~25 s on 16 threads), 6 for C5 (15
    SuperGlue pairs at ~1.9 s each, ~45 s)."""
    return 7 if config == "c3" else 6


def deep_cpu_baseline(images, intrinsics: np.ndarray, n_img: int, kpts: int, sp_sd, sg_sd, threads: int = 16,
                      n_img_sample: int = 6) -> dict:
    """CPU restatement of the deep front-end timed on `threads` host threads over a bounded sample, scaled to n_img
    images / all their pairs: oracle/deep.py's SuperPoint (torch fp32 on the host, `threads` intra-op threads, as the
    reference's torch modules run on a CPU) on n_img_sample images spread over the scene, then for every pair among
    them the matcher (oracle/deep.py SuperGlue with `threads` intra-op threads, pair after pair; or the oracle
    TwoWayMatcher in C on the float descriptors, `threads` pairs at once) and the oracle 5-point RANSAC."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import deep, oracle

    sample = sample_images(n_img, n_img_sample)
    imgs = np.asarray(images)
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    oracle.ransac_E(rng.normal(size=(8, 2)), rng.normal(size=(8, 2)), 1e-3)
    t0 = time.time()
    feats = [deep.superpoint(oracle.rgb_to_gray(im), sp_sd, max_keypoints=kpts) for im in imgs]
    t_img = (time.time() - t0) / len(imgs)
    pairs = [(a, b) for a in range(len(sample)) for b in range(a + 1, len(sample))]
    K = np.asarray(intrinsics, dtype=np.float64)
    def pair_one(ab):
        a, b = ab
        (k1, s1, d1), (k2, s2, d2) = feats[a], feats[b]
        if sg_sd is not None:
            hw = imgs[a].shape[:2]
            m0, _ = deep.superglue(k1, k2, d1, d2, s1, s2, hw, hw, sg_sd)
            v = m0 >= 0
            m = np.stack([np.flatnonzero(v), m0[v]], 1)
        else:
            m = oracle.twoway_match(d1, d2, RATIO).reshape(-1, 2).astype(np.int64)
        if len(m) >= 6:
            f1, f2 = K[sample[a]], K[sample[b]]
            x1 = (k1[m[:, 0]].astype(np.float64) - f1[1:3]) / f1[0]
            x2 = (k2[m[:, 1]].astype(np.float64) - f2[1:3]) / f2[0]
            oracle.ransac_E(x1, x2, THRESH_PX / max(f1[0], f2[0]))

    t0 = time.time()
    if sg_sd is not None:  # torch on `threads` intra-op threads
        for ab in pairs:
            pair_one(ab)
    else:  # the C matcher / RANSAC drop the GIL: `threads` pairs at once
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(pair_one, pairs))
    t_pair = (time.time() - t0) / len(pairs)
    P = n_img * (n_img - 1) // 2
    total = n_img * t_img + P * t_pair
    what = ("SuperGlue (oracle/deep.py)" if sg_sd is not None else "TwoWayMatcher (oracle/twoway.c)")
    return {"value": P / total, "unit": "verified image-pairs/sec", "cores": threads, "kind": "port, extrapolated",
            "sample": f"CPU restatement on {threads} threads: SuperPoint (oracle/deep.py, torch fp32) of "
                      f"{len(sample)} of the {n_img} images ({t_img:.2f} s/img), {what} + oracle RANSAC on the "
                      f"{len(pairs)} pairs among them ({t_pair:.2f} s/pair wall), scaled to {n_img} images / {P} pairs"}


def parity_statement(config: str, ba: bool) -> dict:
    """How each stage of this line's workload is checked against the reference, and where that check stops (the
    limits are inherent: OpenCV and GTSAM, whose algorithms the oracle restates, are not in /root/reference)."""
    verify = ("5-pt RANSAC + LO + recoverPose: n_hyp, masks, R, t bit-identical to oracle/ransac.c "
              "(tests/test_verifier_gpu.py, tests/test_lund_door_c1_gpu.py); the oracle itself is pinned to the "
              "reference only by tolerance known-answers (two-plane, Argoverse: tests/test_oracle_verifier.py) and C1 "
              "ground truth, because OpenCV's USAC is absent -- GPU == oracle is a self-consistent pair")
    out = {}
    if config in ("c3", "c5"):
        out["extract"] = ("SuperPoint vs goldens produced by the reference's own superpoint.py here, random weights "
                          "only (tests/test_superpoint_gpu.py)")
        if config == "c3":
            out["match"] = ("TwoWayMatcher F16_RERANK: bit-identical to the exact fp32 matcher whenever the "
                            "certificate holds, rescans otherwise (tests/test_matcher_float_gpu.py); the whitened "
                            "descriptor head suits the certificate -- see matcher_certificate and the plain-head line")
        else:
            out["match"] = ("SuperGlue log-assignment within 2e-3 of goldens from the reference's superglue.py, random "
                            "weights only; mismatches only at near-ties (tests/test_superglue_gpu.py)")
    else:
        out["extract"] = ("SIFT bit-exact vs oracle/sift.c (tests/test_sift_gpu.py); the oracle is pinned to the "
                          "reference's OpenCV fixture: >= 99 % of keypoints within 0.005 px, descriptors within 1 for "
                          ">= 95 % (tests/test_oracle_sift.py)")
        out["match"] = ("TwoWayMatcher bit-exact vs the reference's known answers and the 3015-match Lund fixture "
                        "(tests/test_matcher_gpu.py)")
    out["verify"] = verify
    if ba:
        out["bundle_adjust"] = ("two-view BA vs oracle/ba2.c (tests/test_ba2_gpu.py); unpinned vs GTSAM (the "
                                "reference test's data is not in /root/reference)")
    return out


def main_frontend(args, info, config: str):
    """The all-pairs front-end engine (gtsfm_amd/frontend/all_pairs.py) on one BASELINE config:
    c1 (configs[0]: Lund Door, 12 images, 5000 SIFT kpts), c2 (configs[1]: 100 rendered 1080p images, 2048 SIFT kpts;
    N > 1 GPUs share the same scene, "strong"; c2-weak grows the scene instead), c4 (configs[3]: 1000 images,
    "strong"), c3 (configs[2]: 200 images, SuperPoint 4096 kpts + TwoWayMatcher F16_RERANK) and c5 (a slice of
    configs[4]: 32 images, SuperPoint 2048 kpts + SuperGlue), each followed by 5-point RANSAC + inlier support."""
    from gtsfm_amd import native, synthetic
    from gtsfm_amd.frontend import sharding
    from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig, HipSuperPointKernels

    rank, world, dev = info.rank, info.world, info.device
    native.lib()
    deep = config in ("c3", "c5")
    emulate = args.emulate_world > 1
    if emulate:
        # one process runs rank `emulate_rank`'s share of an `emulate_world`-rank job on this GPU (not a scaling run)
        if world != 1:
            raise SystemExit("--emulate-world runs in a single process (--gpus 1)")
        if not 0 <= args.emulate_rank < args.emulate_world:
            raise SystemExit("--emulate-rank must be in [0, --emulate-world)")
        rank, world = args.emulate_rank, args.emulate_world
    elif args.pair_limit:
        raise SystemExit("--pair-limit only applies to --emulate-world runs")
    want_baseline = rank == 0 and world == 1 and not args.no_cpu_baseline
    if config == "c1":
        all_imgs, intrinsics = lund_door_c1()
        n_img, scaling = len(all_imgs), "strong"
        H, W = all_imgs.shape[1], all_imgs.shape[2]
        kpts = args.kpts if args.kpts != 2048 else 5000  # sift_front_end.yaml max_keypoints
        mine = sharding.local_images(n_img, world, rank)
        host_images = all_imgs[torch.from_numpy(mine)].contiguous().pin_memory()
        baseline_images = all_imgs.numpy()[sample_images(n_img, 16)]
    else:
        if config == "c4":
            n_img, scaling = args.images or 1000, "strong"
        elif config == "c2-weak":
            n_img, scaling = args.images or images_for(world), "weak"
        elif config == "c3":
            n_img, scaling = args.images or 200, "strong"
        elif config == "c5":
            n_img, scaling = args.images or 32, "strong"
        else:  # c2: the 100-image scene of configs[1] at every N (the pairs of the same scene split over the ranks)
            n_img, scaling = args.images or 100, "strong"
        H, W = args.height, args.width
        kpts = args.kpts if not (config == "c3" and args.kpts == 2048) else 4096
        mine = sharding.local_images(n_img, world, rank)
        # every rank renders (seeded, identical cameras) only the images it extracts; rendering is data generation
        path = "strafe" if config == "c3" else "orbit"
        scene = synthetic.render_scene(n_img, H, W, device=str(dev), indices=mine, path=path)
        host_images = scene.images.cpu().pin_memory()
        intrinsics = scene.intrinsics
        del scene.images
        torch.cuda.empty_cache()
        baseline_images = None
        n_sample = n_img if args.cpu_baseline_full else (deep_sample(config) if deep else 16)
        if want_baseline:
            baseline_images = host_images.numpy()[sample_images(n_img, n_sample)]
    cfg = FrontEndConfig(kpts=kpts, ratio=RATIO, thresh_px=THRESH_PX, min_inliers=MIN_INLIERS,
                         min_inlier_ratio=MIN_INLIER_RATIO)
    if deep:
        cfg.extract_chunk, cfg.extract_first, cfg.resident_chunk = 8, 4, 16  # ~0.75 GB SuperPoint workspace / image
    if args.extract_chunk:
        cfg.extract_chunk = args.extract_chunk
    if args.extract_first:
        cfg.extract_first = args.extract_first
    if args.resident_chunk:
        cfg.resident_chunk = args.resident_chunk
    if args.pair_chunk:
        cfg.pair_chunk = args.pair_chunk
    cfg.bundle_adjust = args.ba
    kernels = sp_sd = sg_sd = None
    if deep:
        head = True if config == "c5" else ("c3" if args.c3_head == "c3" else False)
        sp_sd, sp_w, sg_sd, sg_w = deep_weights(dev, config == "c5", head=head)
        kernels = HipSuperPointKernels(sp_w, "superglue" if config == "c5" else "twoway", sg_w)
    exchange, kc_all = None, np.zeros(n_img)
    if emulate:
        # untimed: the other ranks' extraction and packed exchange blocks, produced here one rank at a time
        blocks = {}
        for r in range(world):
            if r == rank:
                continue
            idx_r = sharding.local_images(n_img, world, r)
            if config == "c1":
                imgs_r = all_imgs[torch.from_numpy(idx_r)].contiguous()
            else:
                imgs_r = synthetic.render_scene(n_img, H, W, device=str(dev), indices=idx_r, path=path).images.cpu()
            fe_r = AllPairsFrontEnd(imgs_r, intrinsics, n_img, r, world, dev, cfg, kernels=kernels,
                                    image_pairs=np.zeros((0, 2), np.int64))
            fe_r._extract(resident=False)
            blocks[r] = fe_r.packed_features()
            kc_all[idx_r] = fe_r.feats.count.cpu().numpy()
            del fe_r, imgs_r
            torch.cuda.empty_cache()
        nbytes = next(iter(blocks.values())).numel()
        others = torch.zeros((world, nbytes), dtype=torch.uint8, device=dev)
        for r, b in blocks.items():
            others[r].copy_(b)
        del blocks
        exchange = sharding.EmulatedAllGather(others, rank)
    fe = AllPairsFrontEnd(host_images, intrinsics, n_img, rank, world, dev, cfg, kernels=kernels, exchange=exchange,
                          pair_limit=args.pair_limit or None)

    for _ in range(args.warmup):
        res = fe.step()
    tworld = 1 if emulate else world  # the emulated job has one process
    elapsed = timed_steps(fe, args.steps, False, tworld, dev)
    elapsed_res = timed_steps(fe, args.steps, True, tworld, dev)
    # `value` is the device-resident figure (inputs in HBM when the timed region starts); the host-to-host figure of
    # SURVEY.md §8(d) (PCIe copies inside the step) is reported beside it, never as value
    ms_per_step = elapsed_res / args.steps * 1e3
    value = fe.total_pairs / (elapsed_res / args.steps)

    # instrumented steps: per-phase HIP events on the compute / copy streams; the matcher kernel's own events
    # (the distance GEMM, or F16_RERANK's shortlist GEMM) through gtsfm_match_set_kernel_events
    lib = native.lib()
    stage_host, stage_res, kernel_ms = [], [], []
    fe.instrument = True
    for _ in range(3 if not deep else 2):
        res = fe.step(resident=False)
        torch.cuda.synchronize()
        stage_host.append(fe.stage_ms())
        kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for e in kev:
            e.record()  # creates the hipEvent_t handles
        native.check(lib.gtsfm_match_set_kernel_events(kev[0].cuda_event, kev[1].cuda_event), "set_kernel_events")
        fe.step(resident=True)
        torch.cuda.synchronize()
        native.check(lib.gtsfm_match_set_kernel_events(None, None), "set_kernel_events")
        stage_res.append(fe.stage_ms())
        kernel_ms.append(kev[0].elapsed_time(kev[1]))
    fe.instrument = False

    def med(rows):
        keys = sorted(set().union(*[r.keys() for r in rows]))
        return {k: round(float(np.median([r.get(k, 0.0) for r in rows])), 3) for k in keys}

    st_host, st_res = med(stage_host), med(stage_res)
    certificate = None
    if config == "c3" and world == 1 and not emulate:
        # F16_RERANK's certificate on this workload (one more, untimed matching of the step's features): how much of
        # the shortlist the fp16 bound certified, and how the rest was recomputed exactly (whole (pair, side) tiles
        # or per-keypoint rescans) -- the share of the matcher's time the descriptor head decides
        from gtsfm_amd import device as hip

        st = {}
        hip.match_pairs(fe.feats.desc, fe.feats.count, fe.pairs_dev, RATIO, native.GTSFM_MATCH_F16_RERANK, stats=st)
        certificate = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in st.items()}
    n_ok = torch.tensor([float(res.isp_ok.sum())], dtype=torch.float64, device=dev)
    n_inl_rows = torch.tensor([float(len(res.v_corr))], dtype=torch.float64, device=dev)
    # per-stage algorithmic work of this rank
    kc = kc_all
    kc[mine] = res.kp_count
    stats = {k: v.double() for k, v in fe.stats.items()}
    if world > 1 and not emulate:
        t = torch.from_numpy(kc).to(dev)
        torch.distributed.all_reduce(t)
        kc = t.cpu().numpy()
        torch.distributed.all_reduce(n_ok)
        torch.distributed.all_reduce(n_inl_rows)
    pr = fe.my_pairs
    a_last, b_last = fe.pchunks[-1]
    pl = pr[a_last:b_last]  # the kernel events end on the LAST pair chunk's launch: its pairs are that launch's work
    D = fe.desc_dim
    H_p, M_p, S_p = stats["n_hyp"], stats["n_matches"], stats["n_models"]
    solve_flop = float((1.2e4 * H_p).sum().item())  # 5-point solver, fp64 (ransac_solve1 / solve2)
    score_flop = float((36.0 * M_p * S_p).sum().item())  # Sampson scoring, fp32 (ransac_score)
    verify_flop = solve_flop + score_flop
    ex_ms, m_ms, ver_ms = (st_res.get(k, float("nan")) for k in ("extract", "match", "verify"))
    verify_tf = verify_flop / (ver_ms * 1e-3) / 1e12
    # each part against its own vector peak: the stage's time at peak is the sum of the two parts' times at peak
    t_peak = solve_flop / (VALU_F64_PEAK_TFLOPS * 1e12) + score_flop / (VALU_F32_PEAK_TFLOPS * 1e12)
    verify_stage = {"bound": "valu (fp64 solve + fp32 score)", "achieved": round(verify_tf, 2),
                    "peak": round(verify_flop / t_peak / 1e12, 1) if t_peak > 0 else None,
                    "unit": "TFLOP/s", "frac": round(t_peak / (ver_ms * 1e-3), 4) if ver_ms > 0 else None,
                    "ms": ver_ms, "solve_gflop_fp64": round(solve_flop / 1e9, 2),
                    "score_gflop_fp32": round(score_flop / 1e9, 2),
                    "work": "SURVEY 8(d): sum_p H_p*1.2e4 (fp64, vs %.1f TF) + 36*M_p*(models scored)_p (fp32, vs %.1f "
                            "TF); peak = the two parts' flop-weighted peak; H mean %.1f, models/H %.2f"
                            % (VALU_F64_PEAK_TFLOPS, VALU_F32_PEAK_TFLOPS, float(H_p.mean()),
                               float(S_p.sum() / max(float(H_p.sum()), 1.0)))}
    gemm_ms = float(np.median(kernel_ms))
    gemm_flop = float((2.0 * kc[pl[:, 0]] * kc[pl[:, 1]] * D).sum())
    gemm_flop_all = float((2.0 * kc[pr[:, 0]] * kc[pr[:, 1]] * D).sum())
    gemm_tf = gemm_flop / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else float("nan")
    if not deep:
        extract_bytes = fe.n_local * sift_bytes_per_image(H, W, kpts)
        extract_gbs = extract_bytes / (ex_ms * 1e-3) / 1e9
        moved_bytes = fe.n_local * sift_moved_bytes_per_image(H, W, kpts)
        moved_gbs = moved_bytes / (ex_ms * 1e-3) / 1e9
        kpad = -(-kpts // 256) * 256
        # the last launch's operand images (both sides of its pairs) read once, its putatives written once
        n_launch_img = len(np.unique(pl))
        algo_bytes = 2 * n_launch_img * kpad * 144 * 2 + 2 * len(pl) * kpts * 8  # two fp16 forms, K = 144
        traffic = pmc_traffic(config)
        roof = {"bound": "mfma", "achieved": round(gemm_tf, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(gemm_tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None, "algorithmic_bytes": algo_bytes,
                "kernel": "mnn_pp_kernel (one launch per pair chunk)", "kernel_ms": round(gemm_ms, 3),
                "work": "2*K1*K2*128 flop per pair, summed over the last launch's %d pairs (GFLOP: %.1f of %.1f per "
                        "step)" % (len(pl), gemm_flop / 1e9, gemm_flop_all / 1e9)}
        roof["stages"] = {
            "extract": {"bound": "hbm", "achieved": round(extract_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(extract_gbs / HBM_PEAK_GBS, 4), "ms": ex_ms,
                        "work": "SURVEY 8(d): 84*sum_o P_o + H*W + K*528 B/image = %.3f GB x %d images"
                                % (sift_bytes_per_image(H, W, kpts) / 1e9, fe.n_local),
                        "moved_bytes": round(moved_bytes), "frac_moved": round(moved_gbs / HBM_PEAK_GBS, 4),
                        "moved_note": "bytes the SIFT kernels actually move (%.3f GB/image: 3HW + 16HW + 65 B per "
                                      "pyramid pixel + records; DoG is never written): %.1f GB/s"
                                      % (sift_moved_bytes_per_image(H, W, kpts) / 1e9, moved_gbs)},
            "match": {"bound": "mfma", "achieved": round(gemm_tf, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(gemm_tf / MFMA_F16_PEAK_TFLOPS, 4), "ms": round(gemm_ms, 3),
                      "work": "2*K1*K2*128 flop per pair (distance GEMM counted once)"},
            "verify": verify_stage,
        }
        if traffic:
            roof["traffic_note"] = ("L2-miss bytes, Infinity-Cache hits included: the A operand (image i2) of each "
                                    "pair is re-read past the 4 MiB XCD L2, from a %.0f MB operand set that fits the "
                                    "256 MiB Infinity Cache" % (2 * n_launch_img * kpad * 144 * 2 / 1e6))
    else:
        sp_flop = fe.n_local * SP_FLOP_PER_PIXEL * H * W
        sp_tf = sp_flop / (ex_ms * 1e-3) / 1e12
        split_peak = MFMA_F16_PEAK_TFLOPS / 6.0  # bf16x3 split products, fp32-equivalent
        ex_stage = {"bound": "mfma", "achieved": round(sp_tf, 1), "peak": round(split_peak, 1), "unit": "TFLOP/s",
                    "frac": round(sp_tf / split_peak, 4), "ms": ex_ms,
                    "work": "SURVEY 8(d): SuperPoint ~169,600 FLOP per pixel x %d images; convs as fp32-accurate "
                            "bf16x3 split products (peak = dense bf16 MFMA / 6)" % fe.n_local}
        if config == "c5":
            sg_flop = float(superglue_flop(kc[pr[:, 0]], kc[pr[:, 1]]).sum())
            sg_tf = sg_flop / (m_ms * 1e-3) / 1e12
            match_stage = {"bound": "mfma", "achieved": round(sg_tf, 1), "peak": round(split_peak, 1),
                           "unit": "TFLOP/s", "frac": round(sg_tf / split_peak, 4), "ms": m_ms,
                           "work": "SURVEY 8(d): SuperGlue 18*2*(20*K*d^2 + 4*K1*K2*d) + 2*K1*K2*d per pair "
                                   "(d = 256; ~254 GFLOP at K = 2048) over %d pairs, all SuperGlue kernels of the "
                                   "stage (GEMMs, attention, Sinkhorn) timed together; products as fp32-accurate "
                                   "bf16x3 split (peak = dense bf16 MFMA / 6)" % len(pr)}
            roof = dict(match_stage)
            roof["kernel"] = "SuperGlue stage (sg_gemm3 / sg_attention3 / Sinkhorn kernels), HIP events on its stream"
            pmc = deep_pmc("c5")
            roof["traffic"] = round(pmc["hbm_bytes_per_step"]) if pmc else None
            if pmc:
                roof["traffic_source"] = pmc["source"]
                roof["traffic_note"] = ("HBM bytes per step of the SuperGlue stage's kernels (FETCH_SIZE x 2 + "
                                        "WRITE_SIZE, separate --pmc passes); per launch: " + ", ".join(
                                            f"{k} {v['hbm_bytes_per_launch'] / 1e6:.1f} MB x {v['launches']}"
                                            for k, v in pmc["kernels"].items()))
        else:
            match_stage = {"bound": "mfma", "achieved": round(gemm_tf, 1), "peak": MFMA_F16_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(gemm_tf / MFMA_F16_PEAK_TFLOPS, 4),
                           "ms": round(gemm_ms, 3), "stage_ms": m_ms,
                           "work": "2*K1*K2*256 flop per pair over the last launch's %d pairs (the shortlist kernel "
                                   "computes the matrix once per side: 2x this)" % len(pl)}
            roof = dict(match_stage)
            roof["kernel"] = "fl_shortlist_kernel (F16_RERANK fp16 MFMA shortlist; one launch per pair chunk)"
            pmc = deep_pmc("c3")
            ks = pmc["kernels"].get("fl_shortlist_kernel") if pmc else None
            roof["traffic"] = round(ks["hbm_bytes_per_launch"]) if ks else None
            if ks:
                roof["traffic_source"] = pmc["source"]
                roof["traffic_note"] = ("HBM bytes per fl_shortlist_kernel launch (FETCH_SIZE x 2 + WRITE_SIZE, "
                                        "separate --pmc passes); also per launch: " + ", ".join(
                                            f"{k} {v['hbm_bytes_per_launch'] / 1e6:.1f} MB x {v['launches']}"
                                            for k, v in pmc["kernels"].items() if k != "fl_shortlist_kernel"))
        roof["stages"] = {"extract": ex_stage, "match": match_stage, "verify": verify_stage}
    wl = {"c1": "C1", "c4": "C4", "c3": "C3", "c5": "C5 slice"}.get(config, "C2")
    if deep:
        desc = (f"{wl}: {n_img} synthetic {W}x{H} images, all {fe.total_pairs} pairs, SuperPoint {kpts} kpts/img + "
                + ("SuperGlue 18 layers / 20 Sinkhorn iterations" if config == "c5" else
                   f"TwoWayMatcher ratio {RATIO} (F16_RERANK)") + f", 5-pt RANSAC {THRESH_PX}px + inlier support")
        dtype = ("u8 image / fp32-accurate bf16x3-MFMA SuperPoint / " + ("fp32-accurate bf16x3-MFMA SuperGlue"
                                                                      if config == "c5" else
                 "fp16-MFMA shortlist + fp32 exact re-rank") + " / fp64 RANSAC solver")
        data = ("synthetic (rendered textured room, seeds 0/1/2" + ("; 1 m strafe path" if config == "c3" else "")
                + "); seeded random network weights with " +
                ("the plain seeded SuperPoint descriptor head (tests/superpoint_weights.py seed 0, not whitened)"
                 if head is False else "a whitened SuperPoint descriptor head "
                 "(tests/golden/make_superpoint_whitening.py" + (" --c3" if config == "c3" else "") + ")"))
    else:
        desc = (f"{wl}: {n_img} {'Lund Door' if config == 'c1' else 'synthetic'} {W}x{H} images, all "
                f"{fe.total_pairs} pairs, SIFT {kpts} kpts/img, ratio {RATIO}, 5-pt RANSAC {THRESH_PX}px"
                + (" + two-view BA" if args.ba else "") + " + inlier support")
        dtype = "u8 image / fp32 pyramid / fp16-MFMA exact-int distances / fp64 RANSAC solver"
        data = ("the reference's Lund Door images (tests/data/set1_lund_door)" if config == "c1" else
                "synthetic (rendered textured room, seeds 0/1/2)")
    out = {
        "metric": "verified image-pairs/sec (all-pairs front-end), N images @ 2048 kpts/img",
        "value": round(value, 2),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dtype,
        "data": data,
        "config": {"workload": desc, "images": n_img, "pairs": fe.total_pairs, "kpts": kpts,
                   "parallelism": f"pair blocks x{world}",
                   "world_size": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1},
        "value_host_to_host": round(fe.total_pairs / (elapsed / args.steps), 2),
        "ms_per_step_host_to_host": round(elapsed / args.steps * 1e3, 3),
        "pairs_passing_isp": int(n_ok.item()),
        "verified_rows": int(n_inl_rows.item()),
        "mean_putatives": round(float(M_p.mean()), 1) if len(M_p) else 0.0,
        "stage_ms": st_res,
        "stage_ms_host_to_host": st_host,
        "roofline": roof,
        "parity": parity_statement(config, args.ba),
    }
    if certificate is not None:
        out["matcher_certificate"] = certificate
    if emulate:
        # a per-rank measurement, not a scaling curve: value = this rank's pairs per second of its own step
        out["metric"] = "per-rank verified image-pairs/sec (one rank's share of an N-GPU job, emulated on one GPU)"
        out["value"] = round(fe.P / (elapsed_res / args.steps), 2)
        out["n_gpus"] = 1
        out["scaling"] = "per-rank"
        out["emulated"] = {
            "rank": rank, "world": world, "rank_images": fe.n_local, "rank_pairs": fe.P, "job_pairs": fe.total_pairs,
            "implied_job_pairs_per_s_if_ranks_equal": None if args.pair_limit else
            round(fe.total_pairs / (elapsed_res / args.steps), 2),
            "pair_limit": args.pair_limit or None,
            "note": "rank `rank` of a `world`-rank job run alone on one GPU: its images extracted, the exchange's "
                    "packing + the gathered buffer's write (the other ranks' blocks extracted untimed beforehand; "
                    "the xGMI transfer of the all-gather is NOT included), its pair share (every N-th pair) matched, "
                    "verified and compacted"}
    if want_baseline:
        if deep:
            out["cpu_baseline"] = deep_cpu_baseline(baseline_images, intrinsics, n_img, kpts, sp_sd, sg_sd,
                                                    n_img_sample=n_sample)
        elif config == "c1":
            out["cpu_baseline"] = cpu_baseline(baseline_images, intrinsics, n_img, kpts)
        else:
            out["cpu_baseline"] = cpu_baseline(baseline_images, intrinsics, n_img, kpts, n_sift=n_sample,
                                               n_pairs=n_img * (n_img - 1) // 2 if args.cpu_baseline_full else 120)
    if rank == 0 or emulate:
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--images", type=int, default=0)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--kpts", type=int, default=2048)
    ap.add_argument("--extract-chunk", type=int, default=0)
    ap.add_argument("--extract-first", type=int, default=0)
    ap.add_argument("--resident-chunk", type=int, default=0)
    ap.add_argument("--pair-chunk", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-full", action="store_true",
                    help="time the CPU baseline on the whole workload (C2: ~100 s on 16 threads) instead of a sample")
    ap.add_argument("--c3-head", choices=("c3", "plain"), default="c3",
                    help="C3's SuperPoint descriptor head: the PCA-whitened one fitted to the scene, or the plain "
                         "seeded random-weight head")
    ap.add_argument("--ba", action="store_true",
                    help="add the two-view triangulation + bundle adjustment stage (TwoViewEstimator bundle_adjust_2view)")
    ap.add_argument("--config", default="c2",
                    choices=["c1", "c2", "c2-weak", "c4", "c3-match", "c3", "c5", "netvlad"])
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="run ONE rank's share of an N-rank job on this GPU (per-rank step time; not a scaling run)")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--pair-limit", type=int, default=0,
                    help="with --emulate-world: only the first K pairs of the rank's share (a bounded partial run)")
    ap.add_argument("--launch-probe", action="store_true",
                    help="each rank joins a gloo group, prints what it sees and exits (tests the launch path on CPU)")
    args = ap.parse_args()

    if args.gpus > 1 and launch.launched_world() == 1:
        # no launcher: start the ranks now, before this process touches a GPU, and exit with their status
        sys.exit(launch.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if args.launch_probe:
        info = launch.init_rank("gloo")
        print(json.dumps({"rank": info.rank, "world": info.world, "dist_world": torch.distributed.get_world_size()
                          if torch.distributed.is_initialized() else 1}), flush=True)
        launch.finish_rank(info)
        return
    if launch.launched_world() != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {launch.launched_world()} ranks; "
              "using the launcher's world size", file=sys.stderr)
    info = launch.init_rank("nccl")
    try:
        if args.config == "c3-match":
            main_c3(args, info.world, info.rank, info.device)
        elif args.config == "netvlad":
            main_netvlad(args, info.world, info.rank, info.device)
        else:
            main_frontend(args, info, args.config)
    finally:
        launch.finish_rank(info)


if __name__ == "__main__":
    main()
