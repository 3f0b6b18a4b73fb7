"""Throughput of the HIP SuperPoint (per 1080p image) and SuperGlue (per pair at K keypoints), synthetic data and
seeded random weights (pretrained weights are not available offline). Prints one JSON line per network."""
import json
import sys
import time

import numpy as np
import torch

_REPO = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, _REPO)
sys.path.insert(0, __import__("os").path.join(_REPO, "tests"))
from gtsfm_amd import device, native, synthetic  # noqa: E402
from gtsfm_amd.frontend.detector_descriptor.superpoint import pack_superpoint_weights  # noqa: E402
from gtsfm_amd.frontend.matcher.superglue_matcher import pack_superglue_weights  # noqa: E402
from superpoint_weights import superglue_state_dict, superpoint_state_dict  # noqa: E402


def timeit(fn, steps=3, warmup=1):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    dev = torch.device("cuda")
    native.lib()
    n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    scene = synthetic.render_scene(n_img, 1080, 1920, device="cuda")
    wsp = torch.from_numpy(pack_superpoint_weights(superpoint_state_dict(0))).to(dev)
    t = timeit(lambda: device.superpoint_extract(scene.images, wsp, 4096))
    H, W = 1080, 1920
    flops = 2 * (9 * 64 * H * W + 9 * 64 * 64 * H * W + 9 * 64 * 64 * H * W / 4 * 2 + 9 * 64 * 128 * H * W / 16
                 + 9 * 128 * 128 * H * W / 16 + 9 * 128 * 128 * H * W / 64 * 2 + 9 * 128 * 512 * H * W / 64
                 + 256 * 65 * H * W / 64 + 256 * 256 * H * W / 64)
    print(json.dumps({"net": "superpoint", "images": n_img, "ms_per_image": t / n_img * 1e3,
                      "gflop_per_image": flops / 1e9, "tflops": flops * n_img / t / 1e12}), flush=True)
    rng = np.random.default_rng(0)
    n = 2 * n_pairs
    kp = np.stack([rng.uniform(0, 1920, (n, K)), rng.uniform(0, 1080, (n, K))], -1).astype(np.float32)
    sc = rng.uniform(0, 1, (n, K)).astype(np.float32)
    de = rng.standard_normal((n, K, 256)).astype(np.float32)
    de /= np.linalg.norm(de, axis=-1, keepdims=True)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    args = (tt(kp), tt(sc), tt(de), tt(np.full(n, K, np.int32)), tt(np.tile([1080, 1920], (n, 1)).astype(np.int32)),
            tt(np.arange(n, dtype=np.int32).reshape(-1, 2)),
            torch.from_numpy(pack_superglue_weights(superglue_state_dict(0))).to(dev))
    t = timeit(lambda: device.superglue_match(*args))
    flops = 18 * 2 * (2 * K * (4 * 65536 + 393216) + 4 * K * K * 256) + 2 * K * K * 256
    print(json.dumps({"net": "superglue", "pairs": n_pairs, "kpts": K, "ms_per_pair": t / n_pairs * 1e3,
                      "gflop_per_pair": flops / 1e9, "tflops": flops * n_pairs / t / 1e12}), flush=True)


if __name__ == "__main__":
    main()
