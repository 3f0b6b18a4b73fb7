"""Seeded synthetic all-pairs scenes for the front-end benchmark.

A textured room (floor, three walls, a few free-standing boxes) is rendered by ray casting into N cameras on a jittered
orbit, at 1920x1080 by default. f = 1.2 * max(W, H) and the principal point at the image centre, i.e. the reference's
default intrinsics (gtsfm/common/image.py:150-168). Seeds: 0 scene, 1 cameras, 2 texture. Rendering uses torch (GPU
when available): it is data generation, not part of the measured path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


@dataclass
class SyntheticScene:
    images: torch.Tensor          # (N, H, W, 3) uint8
    K: np.ndarray                 # (3, 3) shared intrinsics
    wRc: np.ndarray               # (N, 3, 3) camera-to-world rotations
    wtc: np.ndarray               # (N, 3) camera centres

    @property
    def intrinsics(self) -> np.ndarray:
        """(N, 3) float64 rows (f, u0, v0) for the verifier, one per camera of the scene."""
        n = self.wRc.shape[0]
        return np.tile(np.array([self.K[0, 0], self.K[0, 2], self.K[1, 2]]), (n, 1))

    def relative_pose(self, i1: int, i2: int) -> Tuple[np.ndarray, np.ndarray]:
        """Ground-truth i2Ri1, unit i2ti1 (x2 = R x1 + t in camera coordinates)."""
        R1, R2 = self.wRc[i1], self.wRc[i2]
        R = R2.T @ R1
        t = R2.T @ (self.wtc[i1] - self.wtc[i2])
        return R, t / np.linalg.norm(t)


def make_texture(size: int = 2048, seed: int = 2, device: str = "cpu") -> torch.Tensor:
    """(size, size) float texture in [0, 255]: multi-scale value noise + blobs + rectangles (corners, edges)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    tex = torch.zeros((1, 1, size, size))
    for cells, amp in ((8, 40.0), (32, 40.0), (128, 50.0), (512, 45.0)):
        noise = torch.rand((1, 1, cells, cells), generator=g)
        tex += amp * torch.nn.functional.interpolate(noise, size=(size, size), mode="bicubic", align_corners=False)
    tex = tex[0, 0]
    yy, xx = torch.meshgrid(torch.arange(size, dtype=torch.float32), torch.arange(size, dtype=torch.float32),
                            indexing="ij")
    n_rect = size * size // 2500
    r = torch.rand((n_rect, 5), generator=g)
    for k in range(n_rect):
        cx, cy = float(r[k, 0]) * size, float(r[k, 1]) * size
        hw, hh = 2 + float(r[k, 2]) * 10, 2 + float(r[k, 3]) * 10
        x0, x1 = int(max(cx - hw, 0)), int(min(cx + hw, size))
        y0, y1 = int(max(cy - hh, 0)), int(min(cy + hh, size))
        tex[y0:y1, x0:x1] += (float(r[k, 4]) - 0.5) * 160.0
    n_blob = size * size // 1500
    b = torch.rand((n_blob, 4), generator=g)
    for k in range(n_blob):
        cx, cy, s = float(b[k, 0]) * size, float(b[k, 1]) * size, 1.0 + float(b[k, 2]) * 4.0
        x0, x1 = int(max(cx - 4 * s, 0)), int(min(cx + 4 * s + 1, size))
        y0, y1 = int(max(cy - 4 * s, 0)), int(min(cy + 4 * s + 1, size))
        patch = torch.exp(-((xx[y0:y1, x0:x1] - cx) ** 2 + (yy[y0:y1, x0:x1] - cy) ** 2) / (2 * s * s))
        tex[y0:y1, x0:x1] += (float(b[k, 3]) - 0.5) * 200.0 * patch
    tex = (tex - tex.min()) / (tex.max() - tex.min()) * 235.0 + 10.0
    return tex.to(device)


def _look_at(center: np.ndarray, target: np.ndarray, up=np.array([0.0, 0.0, 1.0])) -> np.ndarray:
    """Camera-to-world rotation with camera z forward, x right, y down."""
    z = target - center
    z /= np.linalg.norm(z)
    x = np.cross(z, up)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


# planes: (normal n, offset d with n.p + d = 0, texture origin o, axis u, axis v, extent (u, v), texture scale)
def _room_planes() -> List[Tuple]:
    P = []
    P.append((np.array([0, 0, 1.0]), 0.0, np.array([-10, -10, 0.0]), np.array([1, 0, 0.0]), np.array([0, 1, 0.0]), 20, 20))
    P.append((np.array([1, 0, 0.0]), 10.0, np.array([-10, -10, 0.0]), np.array([0, 1, 0.0]), np.array([0, 0, 1.0]), 20, 8))
    P.append((np.array([0, 1, 0.0]), 10.0, np.array([-10, -10, 0.0]), np.array([1, 0, 0.0]), np.array([0, 0, 1.0]), 20, 8))
    P.append((np.array([-1, 0, 0.0]), 10.0, np.array([10, -10, 0.0]), np.array([0, 1, 0.0]), np.array([0, 0, 1.0]), 20, 8))
    P.append((np.array([0, -1, 0.0]), 10.0, np.array([-10, 10, 0.0]), np.array([1, 0, 0.0]), np.array([0, 0, 1.0]), 20, 8))
    return P


def render_scene(n_images: int = 100, height: int = 1080, width: int = 1920, seed_scene: int = 0,
                 seed_cameras: int = 1, seed_texture: int = 2, device: str = "cuda",
                 tex_size: int = 2048, indices: Optional[Sequence[int]] = None,
                 path: str = "orbit") -> SyntheticScene:
    """Renders the scene's cameras `indices` (default: all n_images); `images` holds them in that order, while K,
    wRc and wtc always describe all n_images cameras (a rank renders only the images it extracts).

    path "orbit" (default; configs C2 / C4): the cameras on a jittered circle around the room, looking inwards.
    path "strafe" (config C3): the cameras on a jittered 1 m line 7.5 m in front of the room's centre, all looking at
    the far wall 17.5 m away (the boxes in between give parallax): every pair of views overlaps by > 90 % with a mostly
    translational image motion, the regime in which descriptors of a network without trained invariances (the seeded
    random SuperPoint weights) repeat."""
    dev = torch.device(device)
    indices = list(range(n_images)) if indices is None else [int(i) for i in indices]
    tex = make_texture(tex_size, seed_texture, "cpu").to(dev)[None, None]
    rng_s = np.random.default_rng(seed_scene)
    planes = _room_planes()
    for _ in range(4):  # free-standing boxes: two visible faces each
        c = rng_s.uniform(-5, 5, 2)
        h = rng_s.uniform(1.0, 3.0)
        planes.append((np.array([1, 0, 0.0]), -(c[0] + 1.0), np.array([c[0] + 1.0, c[1] - 1, 0]),
                       np.array([0, 1, 0.0]), np.array([0, 0, 1.0]), 2.0, h))
        planes.append((np.array([0, 1, 0.0]), -(c[1] + 1.0), np.array([c[0] - 1, c[1] + 1.0, 0]),
                       np.array([1, 0, 0.0]), np.array([0, 0, 1.0]), 2.0, h))
    rng_c = np.random.default_rng(seed_cameras)
    f = 1.2 * max(width, height)
    K = np.array([[f, 0, width / 2.0], [0, f, height / 2.0], [0, 0, 1.0]])
    wRc, wtc = [], []
    assert path in ("orbit", "strafe"), path
    for i in range(n_images):
        if path == "orbit":
            ang = 2 * math.pi * i / n_images + rng_c.normal(0, 0.02)
            rad = 7.5 + rng_c.normal(0, 0.3)
            center = np.array([rad * math.cos(ang), rad * math.sin(ang), 1.6 + rng_c.normal(0, 0.2)])
            target = np.array([0.0, 0.0, 0.8]) + rng_c.normal(0, 0.5, 3) * np.array([1, 1, 0.3])
        else:
            s_i = -0.5 + 1.0 * i / max(n_images - 1, 1)
            center = np.array([s_i + rng_c.normal(0, 0.01), -7.5 + rng_c.normal(0, 0.05), 1.6 + rng_c.normal(0, 0.05)])
            target = center + np.array([0.0, 17.5, -0.6]) + rng_c.normal(0, 0.05, 3)
        wRc.append(_look_at(center, target))
        wtc.append(center)
    wRc = np.stack(wRc)
    wtc = np.stack(wtc)
    ys, xs = torch.meshgrid(torch.arange(height, device=dev, dtype=torch.float32) + 0.5,
                            torch.arange(width, device=dev, dtype=torch.float32) + 0.5, indexing="ij")
    rays_c = torch.stack([(xs - K[0, 2]) / f, (ys - K[1, 2]) / f, torch.ones_like(xs)], -1)  # (H, W, 3)
    images = torch.empty((len(indices), height, width, 3), dtype=torch.uint8, device=dev)
    for slot, i in enumerate(indices):
        R = torch.tensor(wRc[i], dtype=torch.float32, device=dev)
        o = torch.tensor(wtc[i], dtype=torch.float32, device=dev)
        d = rays_c @ R.T  # world directions
        best_t = torch.full((height, width), float("inf"), device=dev)
        val = torch.full((height, width), 128.0, device=dev)
        for pi, (n_, d_, org, ua, va, ext_u, ext_v) in enumerate(planes):
            n_t = torch.tensor(n_, dtype=torch.float32, device=dev)
            denom = d @ n_t
            t = -(float(n_ @ wtc[i]) + d_) / torch.where(denom.abs() < 1e-6, torch.full_like(denom, 1e-6), denom)
            p = o + t[..., None] * d
            rel = p - torch.tensor(org, dtype=torch.float32, device=dev)
            u = rel @ torch.tensor(ua, dtype=torch.float32, device=dev)
            v = rel @ torch.tensor(va, dtype=torch.float32, device=dev)
            ok = (t > 0.05) & (t < best_t) & (u >= 0) & (u <= ext_u) & (v >= 0) & (v <= ext_v)
            # texture coordinates: the atlas tiles every 5 m, each plane from its own offset
            gu = ((u / 5.0 + 0.37 * pi) % 1.0) * 2 - 1
            gv = ((v / 5.0 + 0.61 * pi) % 1.0) * 2 - 1
            grid = torch.stack([gu, gv], -1)[None]
            samp = torch.nn.functional.grid_sample(tex, grid, mode="bilinear", padding_mode="border",
                                                   align_corners=False)[0, 0]
            shade = 0.75 + 0.25 * abs(float(n_[2]))
            val = torch.where(ok, samp * shade, val)
            best_t = torch.where(ok, t, best_t)
        img = val.clamp(0, 255).round().to(torch.uint8)
        images[slot] = torch.stack([img, (img.float() * 0.95).round().to(torch.uint8), img], -1)
    return SyntheticScene(images=images, K=K, wRc=wRc, wtc=wtc)


def all_pairs(n: int) -> np.ndarray:
    i1, i2 = np.triu_indices(n, k=1)
    return np.stack([i1, i2], 1).astype(np.int32)
