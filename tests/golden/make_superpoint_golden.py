"""Golden SuperPoint outputs from the reference's own module (run in the build container, where /root/reference
exists; the GPU box has no reference and only reads the .npz this writes).

The reference module thirdparty/SuperGluePretrainedNetwork/models/superpoint.py is imported as-is and run on CPU
(torch fp32) with the seeded random weights of tests/superpoint_weights.py (its __init__ loads
weights/superpoint_v1.pth, which is absent offline, so torch.load is redirected to those tensors while the module is
constructed). Inputs: the committed Lund-door gray image (crops) and a rendered synthetic image. Outputs per case:
keypoints (N, 2) float32 in the reference's raster order, scores (N,), and descriptors of every 8th keypoint (the full
256 x N array would be megabytes).

    python tests/golden/make_superpoint_golden.py
"""
import os
import sys

import numpy as np
import torch
from PIL import Image as PILImage

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))  # tests/ (the reference has a `tests` package of its own)

from superpoint_weights import superpoint_state_dict  # noqa: E402


def reference_superpoint(seed=0):
    from thirdparty.SuperGluePretrainedNetwork.models import superpoint as sp_mod

    sd = {k: torch.from_numpy(v) for k, v in superpoint_state_dict(seed).items()}
    real_load = torch.load
    torch.load = lambda *a, **k: sd
    try:
        model = sp_mod.SuperPoint({}).eval()
    finally:
        torch.load = real_load
    return model


LUND_1080P_CROP = (slice(8, 1928), slice(108, 1188))
TOPK_C3 = 4096  # BASELINE config C3: 4096 keypoints per image


def cases():
    gray = np.asarray(PILImage.open(os.path.join(HERE, "lund_door_DSC_0001_gray.png")))
    out = {"lund_480x640": np.ascontiguousarray(gray[300:780, 200:840]),
           "lund_250x333": np.ascontiguousarray(gray[100:350, 500:833])}
    from gtsfm_amd import synthetic

    sc = synthetic.render_scene(1, 240, 320, device="cpu")
    rgb = sc.images[0].numpy()
    # cv2.COLOR_RGB2GRAY fixed point (oracle restatement is pinned to the reference's OpenCV fixture)
    from oracle import oracle

    out["synthetic_240x320"] = oracle.rgb_to_gray(rgb)
    # BASELINE config C3 resolution: a 1920 x 1080 (portrait) crop of the full Lund image (not stored: the test
    # re-crops the committed PNG with LUND_1080P_CROP)
    out["lund_1920x1080"] = np.ascontiguousarray(gray[LUND_1080P_CROP])
    return out


def main():
    model = reference_superpoint(0)
    res = {}
    for name, g in cases().items():
        x = torch.from_numpy(g.astype(np.float32)[None, None] / 255.0)
        with torch.no_grad():
            r = model({"image": x})
        kp = r["keypoints"][0].numpy().astype(np.float32)
        sc = r["scores"][0].numpy().astype(np.float32)
        desc = r["descriptors"][0].numpy().astype(np.float32)  # (256, N)
        if name == "lund_1920x1080":
            # descriptors of every 8th keypoint of the top-4096 set (the drop-in's get_top_k(4096))
            top = np.sort(np.argsort(-sc, kind="stable")[:TOPK_C3])
            sel = top[::8]
        else:
            sel = np.arange(0, kp.shape[0], 8)
            res[f"{name}__image"] = g
        res[f"{name}__keypoints"] = kp
        res[f"{name}__scores"] = sc
        res[f"{name}__desc_rows"] = sel.astype(np.int32)
        res[f"{name}__desc"] = desc[:, sel].T.copy()
        print(name, g.shape, "kpts", kp.shape[0])
    res["torch_version"] = np.array(torch.__version__)
    np.savez_compressed(os.path.join(HERE, "superpoint_random_w0.npz"), **res)


if __name__ == "__main__":
    main()
