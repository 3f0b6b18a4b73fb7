"""Seeded random SuperPoint / SuperGlue weights (test infrastructure).

The reference's pretrained weights are not in the image (thirdparty/.../download_model_weights.sh fetches them from
the network), so parity is pinned on random-init weights: the golden script loads these exact tensors into the
reference's own SuperPoint module and records its outputs; the GPU tests load the same tensors into the HIP path.
Kaiming-normal scale (std = sqrt(2 / fan_in)) keeps activations O(1) through the 8-layer encoder.
"""
import os

import numpy as np

SUPERPOINT_LAYERS = [  # (name, cin, cout, kernel) in the reference module's order (superpoint.py:120-134)
    ("conv1a", 1, 64, 3), ("conv1b", 64, 64, 3), ("conv2a", 64, 64, 3), ("conv2b", 64, 64, 3),
    ("conv3a", 64, 128, 3), ("conv3b", 128, 128, 3), ("conv4a", 128, 128, 3), ("conv4b", 128, 128, 3),
    ("convPa", 128, 256, 3), ("convPb", 256, 65, 1), ("convDa", 128, 256, 3), ("convDb", 256, 256, 1),
]


WHITENED_CONVDB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "superpoint_w0_convDb_whitened.npz")
C3_CONVDB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "superpoint_w0_convDb_pca32_strafe.npz")


def superpoint_state_dict(seed: int = 0, whitened=False) -> dict:
    """name.weight (cout, cin, k, k) float32 and name.bias (cout,) float32 for every SuperPoint conv.

    whitened=True (seed 0 only): convDb replaced by the ZCA whitening of convDa's activations over the benchmark
    scene (tests/golden/make_superpoint_whitening.py), so that descriptors of unrelated keypoints are decorrelated
    and repeated scene points match -- the descriptor statistics the matchers see with trained weights.
    whitened="c3": the head fitted for config C3's strafe scene (32 leading principal directions whitened, the rest
    at a quarter weight)."""
    rng = np.random.default_rng(seed)
    sd = {}
    for name, cin, cout, k in SUPERPOINT_LAYERS:
        fan_in = cin * k * k
        sd[f"{name}.weight"] = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / fan_in)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-0.05, 0.05, size=cout).astype(np.float32)
    if whitened:
        assert seed == 0, "the whitened head is fitted to the seed-0 encoder"
        with np.load(C3_CONVDB if whitened == "c3" else WHITENED_CONVDB) as z:
            sd["convDb.weight"] = np.ascontiguousarray(z["weight"], dtype=np.float32)
            sd["convDb.bias"] = np.ascontiguousarray(z["bias"], dtype=np.float32)
    return sd


def superglue_state_dict(seed: int = 0, n_layers: int = 18, final_scale: float = 12.0) -> dict:
    """Seeded random weights with the reference SuperGlue module's parameter names (superglue.py:165-211):
    kenc.encoder.{0,3,6,9,12} conv1d (+ BatchNorm1d at 1,4,7,10), gnn.layers.i.attn.{proj.0-2,merge},
    gnn.layers.i.mlp.{0 (conv 512->512), 1 (BN), 3 (conv 512->256)}, final_proj, bin_score.
    Conv weights: std 1/sqrt(fan_in), 0.1x on the residual branches' last conv (keypoint encoder, MLP), so the 18
    residual updates perturb the descriptors by ~10 % each instead of replacing them; final_proj = 12 I + noise, so
    planted correspondences (cosine ~0.95) get peaked assignments and the golden pairs have matches to compare.
    final_scale sets that identity gain: bench.py's C5 slice uses 24, which on the whitened SuperPoint descriptors of
    the rendered scene (cosine ~0.4-0.6 for repeated points, ~0 otherwise) gives ~1000 matches on adjacent views.
    BN: gamma U(0.8, 1.2), beta U(-0.1, 0.1), running mean U(-0.1, 0.1), running var U(0.5, 1.5)."""
    rng = np.random.default_rng(seed)
    sd = {}

    def conv(name, cin, cout, scale=1.0):
        sd[f"{name}.weight"] = (rng.standard_normal((cout, cin, 1)) * scale / np.sqrt(cin)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-0.05, 0.05, size=cout).astype(np.float32)

    def bn(name, c):
        sd[f"{name}.weight"] = rng.uniform(0.8, 1.2, size=c).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-0.1, 0.1, size=c).astype(np.float32)
        sd[f"{name}.running_mean"] = rng.uniform(-0.1, 0.1, size=c).astype(np.float32)
        sd[f"{name}.running_var"] = rng.uniform(0.5, 1.5, size=c).astype(np.float32)
        sd[f"{name}.num_batches_tracked"] = np.array(0, dtype=np.int64)

    chans = [3, 32, 64, 128, 256, 256]
    for i in range(5):
        conv(f"kenc.encoder.{3 * i}", chans[i], chans[i + 1], 0.1 if i == 4 else 1.0)
        if i < 4:
            bn(f"kenc.encoder.{3 * i + 1}", chans[i + 1])
    for l in range(n_layers):
        p = f"gnn.layers.{l}"
        for j in range(3):
            conv(f"{p}.attn.proj.{j}", 256, 256)
        conv(f"{p}.attn.merge", 256, 256)
        conv(f"{p}.mlp.0", 512, 512)
        bn(f"{p}.mlp.1", 512)
        conv(f"{p}.mlp.3", 512, 256, 0.1)
    conv("final_proj", 256, 256, 0.05)
    sd["final_proj.weight"][:, :, 0] += np.float32(final_scale) * np.eye(256, dtype=np.float32)
    sd["bin_score"] = np.array(1.0, dtype=np.float32)
    return sd
