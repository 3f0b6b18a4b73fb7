"""Synthetic two-view scenes for the two-view bundle adjustment tests (oracle/ba2.c, gtsfm_ba2_batched).

A pair = GT relative pose i2Ti1 (R, unit t), 3D points in front of both cameras, pixel measurements with Gaussian
noise, some gross outliers, and a perturbed initial pose (what a verifier would hand to BA).
"""
import numpy as np
from scipy.spatial.transform import Rotation


def make_pair(rng, n, noise_px=0.3, n_out=0, f=1000.0, u0=640.0, v0=360.0, rot_deg=10.0, init_err_deg=0.3):
    K = np.array([[f, 0, u0], [0, f, v0], [0, 0, 1.0]])
    R = Rotation.from_rotvec(np.deg2rad(rot_deg) * rng.normal(size=3) / np.sqrt(3)).as_matrix()
    t = np.array([1.0, rng.normal(0, 0.1), rng.normal(0, 0.1)])
    t /= np.linalg.norm(t)
    X = rng.uniform([-3, -2, 6], [3, 2, 14], size=(n, 3))  # camera-1 frame
    x1 = X @ K.T
    x1 = x1[:, :2] / x1[:, 2:]
    X2 = X @ R.T + t
    x2 = X2 @ K.T
    x2 = x2[:, :2] / x2[:, 2:]
    x1 = x1 + rng.normal(0, noise_px, x1.shape)
    x2 = x2 + rng.normal(0, noise_px, x2.shape)
    if n_out:
        k = rng.choice(n, n_out, replace=False)
        x2[k] += rng.uniform(-40, 40, (n_out, 2))
    R0 = Rotation.from_rotvec(np.deg2rad(init_err_deg) * rng.normal(size=3) / np.sqrt(3)).as_matrix() @ R
    t0 = t + rng.normal(0, np.deg2rad(init_err_deg), 3)
    t0 /= np.linalg.norm(t0)
    return dict(K=(f, u0, v0), R=R, t=t, R0=R0, t0=t0, x1=x1.astype(np.float32).astype(np.float64),
                x2=x2.astype(np.float32).astype(np.float64))


def angle_deg(Ra, Rb):
    return float(np.rad2deg(np.linalg.norm(Rotation.from_matrix(Ra.T @ Rb).as_rotvec())))


def dir_deg(a, b):
    return float(np.rad2deg(np.arccos(np.clip(np.dot(a, b) / np.linalg.norm(a) / np.linalg.norm(b), -1, 1))))
