"""Seeded random NetVLAD weights (test infrastructure).

The reference's NetVLAD checkpoint (VGG16-NetVLAD-Pitts30K_struct.mat, fetched by thirdparty/hloc/netvlad.py:100-106)
is not in the image, so parity is pinned on random weights, under the reference module's parameter names:
- backbone.{0,2,5,7,10,12,14,17,19,21,24,26,28}.weight / .bias: VGG16 `features[:-2]` (13 conv3x3; torchvision's
  configuration "D": 64 64 M 128 128 M 256 256 256 M 512 512 512 M 512 512 512 [M removed]), He-normal by fan-in
  (std sqrt(2 / fan_in)) so activations stay O(1..100) through 13 layers;
- netvlad.score_proj.weight (64, 512, 1), netvlad.centers (512, 64) (netvlad.py:45-48);
- whiten.weight (4096, 32768), whiten.bias (4096) (netvlad.py:109-110), nn.Linear's default uniform range;
- preprocess_mean (3,): the checkpoint's meta.normalization.averageImage (netvlad.py:149-152), here ImageNet-like.
"""
import os

import numpy as np

VGG16_CONVS = [  # (backbone index, cin, cout, max-pool after its ReLU)
    (0, 3, 64, False), (2, 64, 64, True), (5, 64, 128, False), (7, 128, 128, True),
    (10, 128, 256, False), (12, 256, 256, False), (14, 256, 256, True),
    (17, 256, 512, False), (19, 512, 512, False), (21, 512, 512, True),
    (24, 512, 512, False), (26, 512, 512, False), (28, 512, 512, False),
]
DIM, K, WHITE = 512, 64, 4096


def netvlad_state_dict(seed: int = 0, whiten: bool = True) -> dict:
    rng = np.random.default_rng(seed)
    sd = {}
    for idx, cin, cout, _ in VGG16_CONVS:
        sd[f"backbone.{idx}.weight"] = (rng.standard_normal((cout, cin, 3, 3), dtype=np.float32)
                                        * np.float32(np.sqrt(2.0 / (cin * 9))))
        sd[f"backbone.{idx}.bias"] = rng.uniform(-0.05, 0.05, size=cout).astype(np.float32)
    # logits of a unit-norm feature ~ N(0, 4): soft but not uniform cluster assignments
    sd["netvlad.score_proj.weight"] = rng.standard_normal((K, DIM, 1), dtype=np.float32) * np.float32(2.0)
    lim = np.sqrt(6.0 / (DIM + K))
    sd["netvlad.centers"] = rng.uniform(-lim, lim, size=(DIM, K)).astype(np.float32)
    if whiten:
        b = np.float32(1.0 / np.sqrt(DIM * K))
        sd["whiten.weight"] = (rng.random((WHITE, DIM * K), dtype=np.float32) * 2 - 1) * b
        sd["whiten.bias"] = (rng.random(WHITE, dtype=np.float32) * 2 - 1) * b
    sd["preprocess_mean"] = np.array([123.68, 116.78, 103.94], np.float32)
    return sd


def netvlad_cases() -> dict:
    """The golden's inputs: (n, H, W, 3) uint8 crops of the committed Lund-door images (two same-sized crops for the
    batched path, an odd size for the pools' floors, a larger one)."""
    from PIL import Image as PILImage

    lund = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lund_door")
    names = sorted(n for n in os.listdir(lund) if n.endswith(".JPG"))
    a0 = np.asarray(PILImage.open(os.path.join(lund, names[0])).convert("RGB"))
    a1 = np.asarray(PILImage.open(os.path.join(lund, names[1])).convert("RGB"))
    return {
        "lund_240x320": np.stack([a0[500:740, 700:1020], a1[500:740, 700:1020]]),
        "lund_250x333": np.ascontiguousarray(a0[900:1150, 300:633])[None],
        "lund_480x640": np.ascontiguousarray(a1[200:680, 400:1040])[None],
    }
