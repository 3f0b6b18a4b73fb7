"""Calibration / rotation / direction types used at the plugin boundary.

The reference passes gtsam.Cal3Bundler in and returns gtsam.Rot3 / gtsam.Unit3 (verifier_base.py:59-82). GTSAM is
not part of this image, so when it is not importable these light stand-ins with the same constructors and the
accessors the front-end uses are returned instead; when it is importable the gtsam classes themselves are used.
"""
from typing import Optional

import numpy as np

try:  # pragma: no cover - exercised only where gtsam is installed
    import gtsam  # type: ignore

    Cal3Bundler = gtsam.Cal3Bundler
    Rot3 = gtsam.Rot3
    Unit3 = gtsam.Unit3
    Pose3 = gtsam.Pose3
    PinholeCameraCal3Bundler = gtsam.PinholeCameraCal3Bundler
    HAVE_GTSAM = True
except ImportError:
    HAVE_GTSAM = False

    class Cal3Bundler:  # type: ignore[no-redef]
        """Cal3Bundler(fx=1, k1=0, k2=0, u0=0, v0=0): f, radial k1/k2 (must be 0 on this path), principal point."""

        def __init__(self, fx: float = 1.0, k1: float = 0.0, k2: float = 0.0, u0: float = 0.0, v0: float = 0.0):
            self._f, self._k1, self._k2, self._u0, self._v0 = float(fx), float(k1), float(k2), float(u0), float(v0)

        def fx(self) -> float:
            return self._f

        def px(self) -> float:
            return self._u0

        def py(self) -> float:
            return self._v0

        def k1(self) -> float:
            return self._k1

        def k2(self) -> float:
            return self._k2

        def K(self) -> np.ndarray:
            return np.array([[self._f, 0.0, self._u0], [0.0, self._f, self._v0], [0.0, 0.0, 1.0]])

        def __reduce__(self):
            return (Cal3Bundler, (self._f, self._k1, self._k2, self._u0, self._v0))

    class Rot3:  # type: ignore[no-redef]
        def __init__(self, R: Optional[np.ndarray] = None):
            self._R = np.eye(3) if R is None else np.asarray(R, dtype=np.float64).reshape(3, 3)

        def matrix(self) -> np.ndarray:
            return self._R.copy()

        def inverse(self) -> "Rot3":
            return Rot3(self._R.T)

        def __reduce__(self):
            return (Rot3, (self._R,))

    class Unit3:  # type: ignore[no-redef]
        def __init__(self, v=(1.0, 0.0, 0.0)):
            v = np.asarray(v, dtype=np.float64).reshape(3)
            self._v = v / np.linalg.norm(v)

        def point3(self) -> np.ndarray:
            return self._v.copy()

        def __reduce__(self):
            return (Unit3, (self._v,))

    class Pose3:  # type: ignore[no-redef]
        """wTc: rotation (Rot3) and translation (3,) -- the accessors the front-end uses."""

        def __init__(self, R=None, t=(0.0, 0.0, 0.0)):
            self._R = R if isinstance(R, Rot3) else Rot3(R)
            self._t = np.asarray(t, dtype=np.float64).reshape(3)

        def rotation(self) -> "Rot3":
            return self._R

        def translation(self) -> np.ndarray:
            return self._t.copy()

        def matrix(self) -> np.ndarray:
            T = np.eye(4)
            T[:3, :3], T[:3, 3] = self._R.matrix(), self._t
            return T

        def __reduce__(self):
            return (Pose3, (self._R.matrix(), self._t))

    class PinholeCameraCal3Bundler:  # type: ignore[no-redef]
        """Ground-truth camera: pose wTc (Pose3) and Cal3Bundler calibration."""

        def __init__(self, pose=None, K=None):
            self._pose = pose if pose is not None else Pose3()
            self._K = K if K is not None else Cal3Bundler()

        def pose(self) -> "Pose3":
            return self._pose

        def calibration(self) -> "Cal3Bundler":
            return self._K

        def __reduce__(self):
            return (PinholeCameraCal3Bundler, (self._pose, self._K))


def calibration_params(cal) -> np.ndarray:
    """(f, u0, v0) of a Cal3Bundler; the device path requires k1 == k2 == 0 (true for every reference loader)."""
    if abs(cal.k1()) > 0 or abs(cal.k2()) > 0:
        raise NotImplementedError("radial distortion is not supported on the MI355X verifier path")
    return np.array([cal.fx(), cal.px(), cal.py()], dtype=np.float64)


def rotation_matrix(R) -> np.ndarray:
    return np.asarray(R.matrix(), dtype=np.float64)


def unit_vector(U) -> np.ndarray:
    return np.asarray(U.point3(), dtype=np.float64).reshape(3)


def skew(v) -> np.ndarray:
    x, y, z = np.asarray(v, dtype=np.float64).reshape(3)
    return np.array([[0.0, -z, y], [z, 0.0, -x], [-y, x, 0.0]])


def camera_pose(camera):
    """(wRc, wtc) of a ground-truth camera: a camera with .pose() (gtsam or stand-in), a Pose3, or a 4x4 / 3x4 wTc."""
    if camera is None:
        return None
    p = camera.pose() if hasattr(camera, "pose") else camera
    if hasattr(p, "rotation"):
        return (np.asarray(p.rotation().matrix(), np.float64),
                np.asarray(p.translation(), np.float64).reshape(3))
    T = np.asarray(p, np.float64)
    return T[:3, :3], T[:3, 3]


def is_pinhole_cal3bundler(camera) -> bool:
    """The reference computes GT correspondence metrics only for PinholeCameraCal3Bundler cameras
    (two_view_estimator.py:241-243)."""
    return isinstance(camera, PinholeCameraCal3Bundler)


def calibration_matrix(camera) -> np.ndarray:
    K = camera.calibration()
    return np.asarray(K.K(), dtype=np.float64)
