"""Seeded random SuperPoint / SuperGlue weights (test infrastructure).

The reference's pretrained weights are not in the image (thirdparty/.../download_model_weights.sh fetches them from
the network), so parity is pinned on random-init weights: the golden script loads these exact tensors into the
reference's own SuperPoint module and records its outputs; the GPU tests load the same tensors into the HIP path.
Kaiming-normal scale (std = sqrt(2 / fan_in)) keeps activations O(1) through the 8-layer encoder.
"""
import numpy as np

SUPERPOINT_LAYERS = [  # (name, cin, cout, kernel) in the reference module's order (superpoint.py:120-134)
    ("conv1a", 1, 64, 3), ("conv1b", 64, 64, 3), ("conv2a", 64, 64, 3), ("conv2b", 64, 64, 3),
    ("conv3a", 64, 128, 3), ("conv3b", 128, 128, 3), ("conv4a", 128, 128, 3), ("conv4b", 128, 128, 3),
    ("convPa", 128, 256, 3), ("convPb", 256, 65, 1), ("convDa", 128, 256, 3), ("convDb", 256, 256, 1),
]


def superpoint_state_dict(seed: int = 0) -> dict:
    """name.weight (cout, cin, k, k) float32 and name.bias (cout,) float32 for every SuperPoint conv."""
    rng = np.random.default_rng(seed)
    sd = {}
    for name, cin, cout, k in SUPERPOINT_LAYERS:
        fan_in = cin * k * k
        sd[f"{name}.weight"] = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / fan_in)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-0.05, 0.05, size=cout).astype(np.float32)
    return sd
