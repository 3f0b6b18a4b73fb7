"""SuperGlue matcher on the MI355X.

Drop-in for gtsfm/frontend/matcher/superglue_matcher.py:28-111 (SuperGlueMatcher): same constructor (use_cuda,
use_outdoor_model), same checks (responses required -> ValueError; descriptors must be 256-D -> Exception), same
output: (M, 2) uint32 (i1, i2) in ascending i1 order, from matches0 of the network
(thirdparty/SuperGluePretrainedNetwork/models/superglue.py:228-283) with 20 Sinkhorn iterations and match
threshold 0.2. The network runs in libgtsfm_hip.so (gtsfm_superglue_batched) on the fp32 matrix cores.

Weights: a state dict with the reference module's parameter names, from `weights_path` (superglue_outdoor.pth /
superglue_indoor.pth, torch.load(weights_only=True)) or passed in as `state_dict`.
"""
from pathlib import Path
from typing import Dict, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.matcher.matcher_base import MatcherBase

SUPERGLUE_DESC_DIM = 256
DEFAULT_NUM_SINKHORN_ITERATIONS = 20
MATCH_THRESHOLD = 0.2  # superglue.py:169 default_config
WEIGHTS_DIR = Path("thirdparty/SuperGluePretrainedNetwork/models/weights")
BN_EPS = 1e-5


def _head_major(c: np.ndarray) -> np.ndarray:
    """Channel permutation: new index h * 64 + d <- reference channel 4 d + h (view(b, 64, 4, n))."""
    h, d = np.meshgrid(np.arange(4), np.arange(64), indexing="ij")
    return c[(4 * d + h).ravel()]


def _bn(sd, name):
    scale = sd[f"{name}.weight"] / np.sqrt(sd[f"{name}.running_var"] + np.float32(BN_EPS))
    shift = sd[f"{name}.bias"] - sd[f"{name}.running_mean"] * scale
    return scale.astype(np.float32), shift.astype(np.float32)


def pack_superglue_weights(state_dict: Dict[str, np.ndarray], n_layers: int = 18) -> np.ndarray:
    """Reference state dict -> the packed fp32 blob of include/gtsfm_hip.h / superglue.hip."""
    sd = {k: np.asarray(v, dtype=np.float32) for k, v in state_dict.items() if not k.endswith("num_batches_tracked")}
    parts = []
    cins = [16, 32, 64, 128, 256]
    for i in range(5):
        w = sd[f"kenc.encoder.{3 * i}.weight"][:, :, 0]  # (cout, cin)
        wt = np.zeros((cins[i], w.shape[0]), np.float32)
        wt[: w.shape[1]] = w.T
        parts += [wt.ravel(), sd[f"kenc.encoder.{3 * i}.bias"]]
        if i < 4:
            parts += list(_bn(sd, f"kenc.encoder.{3 * i + 1}"))
    for l in range(n_layers):
        p = f"gnn.layers.{l}"
        wq = [_head_major(sd[f"{p}.attn.proj.{j}.weight"][:, :, 0]) for j in range(3)]  # rows = cout, permuted
        bq = [_head_major(sd[f"{p}.attn.proj.{j}.bias"]) for j in range(3)]
        parts += [np.concatenate([w.T for w in wq], axis=1).ravel(), np.concatenate(bq)]
        wm = sd[f"{p}.attn.merge.weight"][:, :, 0]  # (cout, cin): permute cin
        parts += [_head_major(wm.T).ravel(), sd[f"{p}.attn.merge.bias"]]
        parts += [sd[f"{p}.mlp.0.weight"][:, :, 0].T.ravel(), sd[f"{p}.mlp.0.bias"]]
        parts += list(_bn(sd, f"{p}.mlp.1"))
        parts += [sd[f"{p}.mlp.3.weight"][:, :, 0].T.ravel(), sd[f"{p}.mlp.3.bias"]]
    parts += [sd["final_proj.weight"][:, :, 0].T.ravel(), sd["final_proj.bias"], sd["bin_score"].reshape(1)]
    return np.ascontiguousarray(np.concatenate([np.ascontiguousarray(x).ravel() for x in parts]), dtype=np.float32)


class SuperGlueMatcher(MatcherBase):
    """SuperGlue computed by HIP kernels."""

    def __init__(self, use_cuda: bool = True, use_outdoor_model: bool = True,
                 state_dict: Optional[Dict[str, np.ndarray]] = None, weights_path: Optional[Union[str, Path]] = None,
                 n_layers: int = 18) -> None:
        super().__init__()
        self._config = {"descriptor_dim": SUPERGLUE_DESC_DIM, "weights": "outdoor" if use_outdoor_model else "indoor",
                        "sinkhorn_iterations": DEFAULT_NUM_SINKHORN_ITERATIONS}
        self._use_cuda = use_cuda
        self._state_dict = state_dict
        self._weights_path = weights_path or WEIGHTS_DIR / f"superglue_{self._config['weights']}.pth"
        self._n_layers = n_layers
        self._blob: Optional[torch.Tensor] = None

    def __getstate__(self):
        s = self.__dict__.copy()
        s["_blob"] = None
        return s

    def weights(self) -> torch.Tensor:
        if self._blob is None:
            native.require_gpu()
            sd = self._state_dict
            if sd is None:
                sd = {k: v.numpy() for k, v in
                      torch.load(str(self._weights_path), map_location="cpu", weights_only=True).items()}
            self._blob = torch.from_numpy(pack_superglue_weights(sd, self._n_layers)).to(torch.device("cuda"))
        return self._blob

    def match_batch(self, keypoints: Sequence[Keypoints], descriptors: Sequence[np.ndarray],
                    image_shapes: Sequence[Tuple[int, ...]], pairs: Sequence[Tuple[int, int]]
                    ) -> Dict[Tuple[int, int], np.ndarray]:
        """All pairs in one batched launch sequence; same per-pair output as match()."""
        native.require_gpu()
        n = len(keypoints)
        kmax = max([len(k) for k in keypoints] + [1])
        kmax = (kmax + 63) // 64 * 64
        kp = np.zeros((n, kmax, 2), np.float32)
        sc = np.zeros((n, kmax), np.float32)
        de = np.zeros((n, kmax, SUPERGLUE_DESC_DIM), np.float32)
        cnt = np.zeros(n, np.int32)
        hw = np.zeros((n, 2), np.int32)
        for i, (k, d, s) in enumerate(zip(keypoints, descriptors, image_shapes)):
            if k.responses is None:
                raise ValueError("Responses for keypoints required for SuperGlue")
            if d.shape[1] != SUPERGLUE_DESC_DIM:
                raise Exception("Superglue pretrained network only works on 256 dimensional descriptors")
            m = len(k)
            kp[i, :m] = k.coordinates
            sc[i, :m] = k.responses
            de[i, :m] = d
            cnt[i] = m
            hw[i] = (s[0], s[1])
        out = {}
        run = [p for p in pairs if cnt[p[0]] > 0 and cnt[p[1]] > 0]
        for p in pairs:
            out[tuple(p)] = np.zeros((0, 2), np.uint32)
        if run:
            dev = torch.device("cuda")
            t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
            idx, c, _ = device.superglue_match(t(kp), t(sc), t(de), t(cnt), t(hw),
                                               t(np.asarray(run, np.int32).reshape(-1, 2)), self.weights(),
                                               self._n_layers, self._config["sinkhorn_iterations"], MATCH_THRESHOLD)
            c = c.cpu().numpy()
            w = int(c.max()) if len(c) else 0
            idx = idx[:, :w].cpu().numpy().view(np.uint32)
            for j, p in enumerate(run):
                out[tuple(p)] = idx[j, : c[j]].copy()
        return out

    def match(self, keypoints_i1: Keypoints, keypoints_i2: Keypoints, descriptors_i1: np.ndarray,
              descriptors_i2: np.ndarray, im_shape_i1: Tuple[int, int, int], im_shape_i2: Tuple[int, int, int]
              ) -> np.ndarray:
        return self.match_batch([keypoints_i1, keypoints_i2], [descriptors_i1, descriptors_i2],
                                [im_shape_i1, im_shape_i2], [(0, 1)])[(0, 1)]
