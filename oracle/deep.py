"""CPU restatement (torch fp32 on the host) of the reference's deep front-end networks. TEST INFRASTRUCTURE ONLY:
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it as the checker / CPU baseline; the product path
(gtsfm_amd/) never imports it.

Follows the vendored modules the reference runs (/root/reference/thirdparty/SuperGluePretrainedNetwork/models/):
- superpoint(): SuperPoint.forward (superpoint.py:145-202) -- shared VGG encoder, score head (softmax over 65, 8x8
  pixel shuffle), simple_nms (:47-62), threshold, remove_borders (:65-71), optional top-k, descriptor head with
  L2 normalisation and sample_descriptors (:80-92; align_corners False on torch >= 2.10 through the reference's
  `int(torch.__version__[2]) > 2` test), then gtsfm's get_top_k(max_keypoints) (gtsfm/common/keypoints.py:89-110)
  as SuperPointDetectorDescriptor applies it (frontend/detector_descriptor/superpoint.py:48-74);
- superglue(): SuperGlue.forward (superglue.py:228-283) -- normalize_keypoints (:60-67), KeypointEncoder MLP
  (:70-82), 18 AttentionalPropagation layers self/cross (:85-138; 4 heads, head-interleaved channels d*4 + h),
  final_proj, scores / sqrt(256), log_optimal_transport with 20 Sinkhorn iterations (:141-170;
  superglue_matcher.py:25), mutual argmax + exp(score) > 0.2 (:266-276).
- netvlad(): NetVLAD.forward (thirdparty/hloc/netvlad.py:160-191) as NetVLADGlobalDescriptor.describe drives it
  (netvlad_global_descriptor.py:36-46): x / 255 * 255, clamp, - averageImage, VGG16 features[:-2] (torchvision's
  configuration "D": 13 conv3x3 + ReLU except the last, max-pools after conv 2, 4, 7, 10), per-location L2
  pre-normalisation, NetVLADLayer (:56-71; the residual sums written as sum_n s x - c sum_n s), whitening, L2.
Pinned against the reference modules' own outputs on seeded random weights (tests/golden/superpoint_random_w0.npz,
superglue_random_w0.npz, netvlad_random_w0.npz, written in this container by tests/golden/make_*_golden.py): tests/test_oracle_deep.py.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

_ENC = [("conv1a", "conv1b"), ("conv2a", "conv2b"), ("conv3a", "conv3b"), ("conv4a", "conv4b")]


def _t(sd: Dict[str, np.ndarray], name: str) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(sd[name]))


def _conv(x, sd, name, relu=True):
    w = _t(sd, name + ".weight")
    y = F.conv2d(x, w, _t(sd, name + ".bias"), padding=w.shape[-1] // 2)
    return F.relu(y) if relu else y


def superpoint_encoder(gray: np.ndarray, sd: Dict[str, np.ndarray]) -> torch.Tensor:
    """(1, 128, H/8, W/8) shared encoder output of a uint8 gray image (superpoint.py:147-158)."""
    x = torch.from_numpy(np.ascontiguousarray(gray, dtype=np.float32) / 255.0)[None, None]
    for i, (a, b) in enumerate(_ENC):
        x = _conv(_conv(x, sd, a), sd, b)
        if i < 3:
            x = F.max_pool2d(x, 2, 2)
    return x


def simple_nms(scores: torch.Tensor, r: int) -> torch.Tensor:
    def mp(t):
        return F.max_pool2d(t, kernel_size=2 * r + 1, stride=1, padding=r)

    zeros = torch.zeros_like(scores)
    mask = scores == mp(scores)
    for _ in range(2):
        supp = mp(mask.float()) > 0
        ss = torch.where(supp, zeros, scores)
        mask = mask | ((ss == mp(ss)) & ~supp)
    return torch.where(mask, scores, zeros)


def superpoint(gray: np.ndarray, sd: Dict[str, np.ndarray], max_keypoints: int = -1, keypoint_threshold: float = 0.005,
               nms_radius: int = 4, border: int = 4, mask: Optional[np.ndarray] = None
               ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """keypoints (N, 2) float32 (x, y), scores (N,), descriptors (N, 256) of one uint8 gray image. Raster order
    (torch.nonzero's) when max_keypoints < 0, else the max_keypoints highest scores (ties: raster order).
    mask: (H, W) or None; as gtsfm's SuperPointDetectorDescriptor (superpoint.py:68-72), a keypoint is kept iff
    mask[round(y), round(x)] == 1 (Keypoints.filter_by_mask, keypoints.py:112-127), before the top-k."""
    with torch.no_grad():
        x = superpoint_encoder(gray, sd)
        semi = _conv(_conv(x, sd, "convPa"), sd, "convPb", relu=False)
        sc = F.softmax(semi, 1)[:, :-1]
        b, _, h, w = sc.shape
        sc = sc.permute(0, 2, 3, 1).reshape(b, h, w, 8, 8).permute(0, 1, 3, 2, 4).reshape(b, h * 8, w * 8)
        sc = simple_nms(sc[:, None], nms_radius)[:, 0][0]
        kp = torch.nonzero(sc > keypoint_threshold)
        s = sc[kp[:, 0], kp[:, 1]]
        H, W = h * 8, w * 8
        keep = (kp[:, 0] >= border) & (kp[:, 0] < H - border) & (kp[:, 1] >= border) & (kp[:, 1] < W - border)
        kp, s = kp[keep], s[keep]
        if mask is not None:
            mk = torch.from_numpy(np.asarray(mask)[kp[:, 0].numpy(), kp[:, 1].numpy()] == 1)
            kp, s = kp[mk], s[mk]
        if 0 <= max_keypoints < len(kp):
            order = np.argsort(-s.numpy(), kind="stable")[:max_keypoints]
            order = torch.from_numpy(np.sort(order))
            kp, s = kp[order], s[order]
        xy = torch.flip(kp, [1]).float()
        d = F.normalize(_conv(_conv(x, sd, "convDa"), sd, "convDb", relu=False), p=2, dim=1)
        g = xy - 8 / 2 + 0.5
        g = g / torch.tensor([(w * 8 - 8 / 2 - 0.5), (h * 8 - 8 / 2 - 0.5)])[None]
        g = g * 2 - 1
        args = {"align_corners": int(torch.__version__[2]) > 2}  # the reference's version test (superpoint.py:87)
        desc = F.grid_sample(d, g.view(1, 1, -1, 2), mode="bilinear", **args)
        desc = F.normalize(desc.reshape(1, d.shape[1], -1), p=2, dim=1)[0].T
    return xy.numpy(), s.numpy(), np.ascontiguousarray(desc.numpy())


def _mlp(x, sd, prefix, n, bn=True):
    """Conv1d stack of superglue.py:50-58: conv (+ BatchNorm eval) + ReLU except after the last conv."""
    for i in range(n):
        j = 3 * i if bn else 2 * i
        x = F.conv1d(x, _t(sd, f"{prefix}.{j}.weight"), _t(sd, f"{prefix}.{j}.bias"))
        if i < n - 1:
            if bn:
                q = f"{prefix}.{j + 1}"
                x = F.batch_norm(x, _t(sd, q + ".running_mean"), _t(sd, q + ".running_var"), _t(sd, q + ".weight"),
                                 _t(sd, q + ".bias"), False, 0.0, 1e-5)
            x = F.relu(x)
    return x


def _attn_layer(x, src, sd, p):
    b, c, n = x.shape
    q, k, v = (F.conv1d(t, _t(sd, f"{p}.attn.proj.{i}.weight"), _t(sd, f"{p}.attn.proj.{i}.bias")).view(b, 64, 4, -1)
               for i, t in enumerate((x, src, src)))
    s = torch.einsum("bdhn,bdhm->bhnm", q, k) / 64 ** 0.5
    msg = torch.einsum("bhnm,bdhm->bdhn", F.softmax(s, dim=-1), v).contiguous().view(b, c, -1)
    msg = F.conv1d(msg, _t(sd, f"{p}.attn.merge.weight"), _t(sd, f"{p}.attn.merge.bias"))
    return _mlp(torch.cat([x, msg], 1), sd, f"{p}.mlp", 2)


def superglue(kp0, kp1, d0, d1, s0, s1, hw0, hw1, sd: Dict[str, np.ndarray], sinkhorn_iterations: int = 20,
              match_threshold: float = 0.2, n_layers: int = 18) -> Tuple[np.ndarray, np.ndarray]:
    """matches0 (N0,) int64 (-1 = none) and matching_scores0 (N0,) of one pair; d0 (N0, 256), kp (N, 2) x, y."""
    if len(kp0) == 0 or len(kp1) == 0:
        return np.full(len(kp0), -1, np.int64), np.zeros(len(kp0), np.float32)
    with torch.no_grad():
        def norm(kp, hw):
            size = torch.tensor([float(hw[1]), float(hw[0])])[None]
            return (torch.from_numpy(np.asarray(kp, np.float32)) - size / 2) / (size.max() * 0.7)

        def enc(kp, s, hw):
            inp = torch.cat([norm(kp, hw).T[None], torch.from_numpy(np.asarray(s, np.float32))[None, None]], 1)
            return _mlp(inp, sd, "kenc.encoder", 5)

        x0 = torch.from_numpy(np.asarray(d0, np.float32)).T[None] + enc(kp0, s0, hw0)
        x1 = torch.from_numpy(np.asarray(d1, np.float32)).T[None] + enc(kp1, s1, hw1)
        for layer in range(n_layers):
            p = f"gnn.layers.{layer}"
            src0, src1 = (x1, x0) if layer % 2 else (x0, x1)
            x0, x1 = x0 + _attn_layer(x0, src0, sd, p), x1 + _attn_layer(x1, src1, sd, p)
        w, bias = _t(sd, "final_proj.weight"), _t(sd, "final_proj.bias")
        m0, m1 = F.conv1d(x0, w, bias), F.conv1d(x1, w, bias)
        scores = torch.einsum("bdn,bdm->bnm", m0, m1) / 256 ** 0.5
        Z = log_optimal_transport(scores, _t(sd, "bin_score"), sinkhorn_iterations)
        mx0, mx1 = Z[:, :-1, :-1].max(2), Z[:, :-1, :-1].max(1)
        i0, i1 = mx0.indices, mx1.indices
        mutual0 = torch.arange(i0.shape[1])[None] == i1.gather(1, i0)
        ms0 = torch.where(mutual0, mx0.values.exp(), torch.zeros(()))
        valid0 = mutual0 & (ms0 > match_threshold)
        i0 = torch.where(valid0, i0, torch.full_like(i0, -1))
    return i0[0].numpy().astype(np.int64), ms0[0].numpy()


def log_optimal_transport(scores: torch.Tensor, alpha: torch.Tensor, iters: int) -> torch.Tensor:
    """superglue.py:141-170: dustbin-augmented couplings, log-space Sinkhorn, times M + N."""
    b, m, n = scores.shape
    one = scores.new_tensor(1)
    ms, ns = (m * one).to(scores), (n * one).to(scores)
    couplings = torch.cat([torch.cat([scores, alpha.expand(b, m, 1)], -1),
                           torch.cat([alpha.expand(b, 1, n), alpha.expand(b, 1, 1)], -1)], 1)
    norm = -(ms + ns).log()
    log_mu = torch.cat([norm.expand(m), ns.log()[None] + norm])[None].expand(b, -1)
    log_nu = torch.cat([norm.expand(n), ms.log()[None] + norm])[None].expand(b, -1)
    u, v = torch.zeros_like(log_mu), torch.zeros_like(log_nu)
    for _ in range(iters):
        u = log_mu - torch.logsumexp(couplings + v.unsqueeze(1), dim=2)
        v = log_nu - torch.logsumexp(couplings + u.unsqueeze(2), dim=1)
    return couplings + u.unsqueeze(2) + v.unsqueeze(1) - norm


NETVLAD_CONVS = [(0, False), (2, True), (5, False), (7, True), (10, False), (12, False), (14, True), (17, False),
                 (19, False), (21, True), (24, False), (26, False), (28, False)]  # (backbone index, pool after)


def netvlad(image: np.ndarray, sd: Dict[str, np.ndarray], whiten: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """(desc (4096,), vlad (32768,)) float32 of one (H, W, 3) uint8 RGB image; desc is vlad when whiten is False."""
    with torch.no_grad():
        x = torch.from_numpy(np.ascontiguousarray(image)).permute(2, 0, 1)[None].float() / 255
        x = torch.clamp(x * 255, 0.0, 255.0) - _t(sd, "preprocess_mean").view(1, 3, 1, 1)
        for i, (idx, pool) in enumerate(NETVLAD_CONVS):
            x = F.conv2d(x, _t(sd, f"backbone.{idx}.weight"), _t(sd, f"backbone.{idx}.bias"), padding=1)
            if i + 1 < len(NETVLAD_CONVS):
                x = F.relu(x)
            if pool:
                x = F.max_pool2d(x, 2, 2)
        x = F.normalize(x.reshape(1, x.shape[1], -1), dim=1)[0]  # (512, N)
        s = F.softmax(_t(sd, "netvlad.score_proj.weight")[:, :, 0] @ x, dim=0)  # (64, N)
        c = _t(sd, "netvlad.centers")  # (512, 64)
        v = x @ s.T - c * s.sum(1)[None]  # sum_n s[k, n] (x[:, n] - c[:, k])
        v = F.normalize(v, dim=0).reshape(-1)
        vlad = v / torch.clamp(v.norm(), min=1e-12)
        if not whiten:
            return vlad.numpy(), vlad.numpy()
        y = _t(sd, "whiten.weight") @ vlad + _t(sd, "whiten.bias")
        return (y / torch.clamp(y.norm(), min=1e-12)).numpy(), vlad.numpy()
