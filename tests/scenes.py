"""Geometry helpers for the verifier tests (test infrastructure; numpy restatements of the GTSAM conventions the
reference's tests use: Rot3.RzRyRx, Pose3.between, EssentialMatrix = [t]x R, PinholeCamera projection)."""
import numpy as np


def rot_rz_ry_rx(x: float, y: float, z: float) -> np.ndarray:
    """gtsam.Rot3.RzRyRx(x, y, z) = Rz(z) @ Ry(y) @ Rx(x)."""
    cx, sx, cy, sy, cz, sz = np.cos(x), np.sin(x), np.cos(y), np.sin(y), np.cos(z), np.sin(z)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def relative_pose(wRi1, wti1, wRi2, wti2):
    """i2Ti1 = wTi2.between(wTi1): i2Ri1 = wRi2^T wRi1, i2ti1 = wRi2^T (wti1 - wti2)."""
    return wRi2.T @ wRi1, wRi2.T @ (wti1 - wti2)


def project(wRi, wti, pts, f=1.0, u0=0.0, v0=0.0):
    pc = (pts - wti) @ wRi  # rows: wRi^T (p - t)
    return np.stack([f * pc[:, 0] / pc[:, 2] + u0, f * pc[:, 1] / pc[:, 2] + v0], axis=1), pc[:, 2]


def sample_points_on_plane(coeffs, rx, ry, n):
    """gtsfm/utils/sampling.py:13-42 (np.random global state)."""
    a, b, c, d = coeffs
    x = np.random.uniform(low=rx[0], high=rx[1], size=(n, 1))
    y = np.random.uniform(low=ry[0], high=ry[1], size=(n, 1))
    z = -(a * x + b * y + d) / c
    return np.hstack([x, y, z])


def two_planes_scene(M: int, N: int, seed: int = 15):
    """tests/frontend/verifier/test_verifier_base.py:235-294 simulate_two_planes_scene (f=1 Cal3Bundler)."""
    np.random.seed(seed)
    p1 = sample_points_on_plane((-10, -1, -20, 150), (-5, 7), (-10, 10), M)
    p2 = sample_points_on_plane((15, -2, -35, 200), (-5, 7), (-10, 10), N)
    pts = np.vstack([p1, p2])
    wti1, wti2 = np.array([0.1, 0, -20]), np.array([1, -2, -20.4])
    wRi1, wRi2 = rot_rz_ry_rx(np.pi / 20, 0, 0.0), rot_rz_ry_rx(0.0, np.pi / 6, 0.0)
    R, t = relative_pose(wRi1, wti1, wRi2, wti2)
    uv1, _ = project(wRi1, wti1, pts)
    uv2, _ = project(wRi2, wti2, pts)
    return uv1, uv2, R, t / np.linalg.norm(t)


def rotation_angle_deg(R1, R2) -> float:
    c = (np.trace(R1.T @ R2) - 1) / 2
    return float(np.degrees(np.arccos(np.clip(c, -1, 1))))


def direction_angle_deg(t1, t2) -> float:
    c = np.dot(t1, t2) / np.linalg.norm(t1) / np.linalg.norm(t2)
    return float(np.degrees(np.arccos(np.clip(c, -1, 1))))


def random_two_view(rng, n_in: int, n_out: int, noise_px: float = 0.5, f: float = 1000.0, w=1920, h=1080):
    """Random relative pose + 3D points in front of both cameras; returns pixel coords, K, R, unit t, inlier flags."""
    ang = rng.normal(size=3)
    ang = ang / np.linalg.norm(ang) * np.radians(rng.uniform(5, 25))
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1.0]])
    th = np.linalg.norm(ang)
    k = ang / th
    R = np.eye(3) + np.sin(th) * skew(k) + (1 - np.cos(th)) * skew(k) @ skew(k)
    t = rng.normal(size=3)
    t = t / np.linalg.norm(t)
    X = np.stack([rng.uniform(-4, 4, n_in), rng.uniform(-3, 3, n_in), rng.uniform(6, 15, n_in)], 1)
    X2 = X @ R.T + t
    ok = X2[:, 2] > 0.5
    X, X2 = X[ok], X2[ok]
    uv1 = X[:, :2] / X[:, 2:] * f + K[:2, 2]
    uv2 = X2[:, :2] / X2[:, 2:] * f + K[:2, 2]
    uv1 += rng.normal(scale=noise_px, size=uv1.shape)
    uv2 += rng.normal(scale=noise_px, size=uv2.shape)
    o1 = np.stack([rng.uniform(0, w, n_out), rng.uniform(0, h, n_out)], 1)
    o2 = np.stack([rng.uniform(0, w, n_out), rng.uniform(0, h, n_out)], 1)
    kp1 = np.vstack([uv1, o1])
    kp2 = np.vstack([uv2, o2])
    perm = rng.permutation(len(kp1))
    inl = np.zeros(len(kp1), bool)
    inl[: len(uv1)] = True
    return kp1[perm], kp2[perm], K, R, t, inl[perm]
