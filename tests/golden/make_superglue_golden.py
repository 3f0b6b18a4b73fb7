"""Golden SuperGlue outputs from the reference's own module (build container only; the GPU box reads the .npz).

thirdparty/SuperGluePretrainedNetwork/models/superglue.py is imported as-is and run on CPU (torch fp32) with the
seeded random weights of tests/superpoint_weights.superglue_state_dict (the pretrained outdoor weights are absent
offline; torch.load is redirected while the module is constructed), sinkhorn_iterations = 20 as
gtsfm/frontend/matcher/superglue_matcher.py:25-41 configures it. Inputs: seeded synthetic keypoint sets (x, y in the
image, scores in (0, 1)) with unit 256-D descriptors; 40 % of the points of image 1 are noisy copies of points of
image 0 so that matches exist. Recorded per case: inputs, matches0 / matching_scores0, and for the small case the
full log-assignment matrix; for the 2048 x 2048 case (BASELINE config C5's keypoint count) every 32nd row of it.

    python tests/golden/make_superglue_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

from superpoint_weights import superglue_state_dict  # noqa: E402


def reference_superglue(seed=0):
    from thirdparty.SuperGluePretrainedNetwork.models import superglue as sg_mod

    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in superglue_state_dict(seed).items()}
    real_load = torch.load
    torch.load = lambda *a, **k: sd
    try:
        model = sg_mod.SuperGlue({"descriptor_dim": 256, "weights": "outdoor", "sinkhorn_iterations": 20}).eval()
    finally:
        torch.load = real_load
    return model


def make_case(rng, n0, n1, H, W):
    kp0 = np.stack([rng.uniform(0, W, n0), rng.uniform(0, H, n0)], 1).astype(np.float32)
    d0 = rng.standard_normal((n0, 256)).astype(np.float32)
    n_sh = int(0.4 * min(n0, n1))
    src = rng.choice(n0, n_sh, replace=False)
    kp1 = np.stack([rng.uniform(0, W, n1), rng.uniform(0, H, n1)], 1).astype(np.float32)
    d1 = rng.standard_normal((n1, 256)).astype(np.float32)
    dst = rng.choice(n1, n_sh, replace=False)
    d1[dst] = d0[src] + 0.3 * rng.standard_normal((n_sh, 256)).astype(np.float32)
    kp1[dst] = kp0[src] + rng.normal(0, 20, (n_sh, 2)).astype(np.float32)
    d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    s0 = rng.uniform(0.01, 1, n0).astype(np.float32)
    s1 = rng.uniform(0.01, 1, n1).astype(np.float32)
    return kp0, kp1, d0, d1, s0, s1


def run(model, kp0, kp1, d0, d1, s0, s1, H, W, want_Z=False):
    data = {"keypoints0": torch.from_numpy(kp0)[None], "keypoints1": torch.from_numpy(kp1)[None],
            "descriptors0": torch.from_numpy(d0).T[None].contiguous(),
            "descriptors1": torch.from_numpy(d1).T[None].contiguous(),
            "scores0": torch.from_numpy(s0)[None], "scores1": torch.from_numpy(s1)[None],
            "image0": torch.empty((1, 1, H, W)), "image1": torch.empty((1, 1, H, W))}
    Z = {}
    if want_Z:
        from thirdparty.SuperGluePretrainedNetwork.models import superglue as sg_mod

        real = sg_mod.log_optimal_transport

        def spy(scores, alpha, iters):
            out = real(scores, alpha, iters)
            Z["Z"] = out[0].numpy().copy()
            Z["S"] = scores[0].numpy().copy()
            return out

        sg_mod.log_optimal_transport = spy
    with torch.no_grad():
        r = model(data)
    if want_Z:
        sg_mod.log_optimal_transport = real
    return r["matches0"][0].numpy(), r["matching_scores0"][0].numpy(), Z


def main():
    model = reference_superglue(0)
    rng = np.random.default_rng(7)
    out = {}
    for name, (n0, n1, H, W, want_Z) in {"small_150x170": (150, 170, 480, 640, True),
                                         "mid_700x650": (700, 650, 1080, 1920, False),
                                         "c5_2048x2048": (2048, 2048, 1080, 1920, True)}.items():
        kp0, kp1, d0, d1, s0, s1 = make_case(rng, n0, n1, H, W)
        m0, ms0, Z = run(model, kp0, kp1, d0, d1, s0, s1, H, W, want_Z)
        out.update({f"{name}__kp0": kp0, f"{name}__kp1": kp1, f"{name}__d0": d0, f"{name}__d1": d1,
                    f"{name}__s0": s0, f"{name}__s1": s1, f"{name}__hw": np.array([H, W]),
                    f"{name}__matches0": m0, f"{name}__mscores0": ms0})
        if want_Z and n0 <= 256:
            out[f"{name}__Z"] = Z["Z"]
            out[f"{name}__scores"] = Z["S"]
        elif want_Z:  # BASELINE config C5 size: every 32nd row of the log-assignment + the dustbin row (16 MB in full)
            rows = np.concatenate([np.arange(0, n0, 32), [n0]])
            out[f"{name}__Z_rows"] = rows.astype(np.int32)
            out[f"{name}__Z_sub"] = Z["Z"][rows].copy()
        print(name, "matches", int((m0 >= 0).sum()), "of", n0, "mscore range", float(ms0.max()))
    np.savez_compressed(os.path.join(HERE, "superglue_random_w0.npz"), **out)


if __name__ == "__main__":
    main()
