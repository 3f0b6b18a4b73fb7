"""bz2-pickle cache files in the reference's on-disk format (reference gtsfm/utils/io.py:610-630).

A cache entry is `pickle.dump(data, BZ2File(path, "wb"))` at the interpreter's default protocol, exactly as the
reference writes it. Two things differ, both so that cache directories move between the reference and this package:

- Writing: the package's own front-end types are stored under the reference's class paths (`_REFERENCE_NAMES`), so a
  reference process unpickles a `gtsfm_amd` Keypoints as `gtsfm.common.keypoints.Keypoints`. The attribute layout of
  those types is the reference's, so the pickled state needs no translation.
- Reading: a restricted unpickler resolves only numpy array/scalar reconstruction and the front-end types (under
  either name); any other global is treated like a corrupted file. The reference's loader (io.py:613-623) unpickles
  anything; cache directories are shared between machines, so this one does not.

Corrupted files (bz2 or pickle decode errors) are removed and read as a miss, as in the reference (io.py:619-621).
A file the allowlist refuses is read as a miss and KEPT: it may be a valid entry written by the reference into a
shared cache directory (e.g. a two-view entry holding gtsam Rot3 / Unit3 objects read where gtsam is absent). When
gtsam is importable, its Rot3 / Unit3 / Cal3Bundler classes are allowed, so such entries load.
"""
import io
import logging
import os
import pickle
from bz2 import BZ2File
from pathlib import Path
from typing import Any, Dict, Optional, Tuple

logger = logging.getLogger(__name__)

# our class path -> the reference's class path (same attribute layout)
_REFERENCE_NAMES: Dict[Tuple[str, str], Tuple[str, str]] = {
    ("gtsfm_amd.common.keypoints", "Keypoints"): ("gtsfm.common.keypoints", "Keypoints"),
    ("gtsfm_amd.common.two_view_estimation_report", "TwoViewEstimationReport"):
        ("gtsfm.common.two_view_estimation_report", "TwoViewEstimationReport"),
}
_OUR_NAMES = {ref: ours for ours, ref in _REFERENCE_NAMES.items()}

_NUMPY_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.numeric", "_frombuffer"),
    ("numpy._core.numeric", "_frombuffer"), ("copyreg", "_reconstructor"), ("builtins", "object"),
}
_PACKAGE_GLOBALS = {
    ("gtsfm_amd.common.keypoints", "Keypoints"),
    ("gtsfm_amd.common.two_view_estimation_report", "TwoViewEstimationReport"),
    ("gtsfm_amd.common.geometry", "Rot3"), ("gtsfm_amd.common.geometry", "Unit3"),
    ("gtsfm_amd.common.geometry", "Cal3Bundler"),
}
# gtsam's pybind11 classes (what the reference's two-view cache entries hold), only where gtsam itself is importable
_GTSAM_GLOBALS = {(m, n) for m in ("gtsam", "gtsam.gtsam") for n in ("Rot3", "Unit3", "Cal3Bundler")} | {
    ("copyreg", "__newobj__")}


def _allowed_globals():
    from gtsfm_amd.common import geometry

    return _NUMPY_GLOBALS | _PACKAGE_GLOBALS | (_GTSAM_GLOBALS if geometry.HAVE_GTSAM else set())


class RefusedGlobal(pickle.UnpicklingError):
    """A cache file names a class outside the allowlist: a miss, not a corrupted file."""


class _ReferenceNamePickler(pickle._Pickler):
    """Pure-Python pickler that writes the aliased classes under the reference's module path."""

    def save(self, obj, save_persistent_id=True):
        alias = None
        if isinstance(obj, type):
            alias = _REFERENCE_NAMES.get((obj.__module__, obj.__qualname__))
        if alias is None or self.proto < 4:
            return super().save(obj, save_persistent_id)
        self.framer.commit_frame()
        memo = self.memo.get(id(obj))
        if memo is not None:
            self.write(self.get(memo[0]))
            return
        self.save(alias[0])
        self.save(alias[1])
        self.write(pickle.STACK_GLOBAL)
        self.memoize(obj)


class _CacheUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str) -> Any:
        module, name = _OUR_NAMES.get((module, name), (module, name))
        if (module, name) in _allowed_globals():
            return super().find_class(module, name)
        raise RefusedGlobal(f"global {module}.{name} is not allowed in a front-end cache file")


def dumps(data: Any) -> bytes:
    buf = io.BytesIO()
    _ReferenceNamePickler(buf, protocol=pickle.DEFAULT_PROTOCOL).dump(data)
    return buf.getvalue()


def loads(blob: bytes) -> Any:
    return _CacheUnpickler(io.BytesIO(blob)).load()


def read_from_bz2_file(file_path: Path) -> Optional[Any]:
    """Reads a cache entry if it exists (io.py:613-623). Corrupted files are removed and read as None; files naming a
    class outside the allowlist are read as None and kept."""
    file_path = Path(file_path)
    if not file_path.exists():
        return None
    try:
        with BZ2File(file_path, "rb") as f:
            return loads(f.read())
    except RefusedGlobal as e:
        logger.warning("Cache file %s not loaded (%s); treated as a miss and kept", file_path, e)
        return None
    except Exception:
        logger.exception("Cache file was corrupted, removing it...")
        os.remove(file_path)
        return None


def write_to_bz2_file(data: Any, file_path: Path) -> None:
    """Writes a cache entry (io.py:626-630), creating parent directories."""
    file_path = Path(file_path)
    file_path.parent.mkdir(exist_ok=True, parents=True)
    with BZ2File(file_path, "wb") as f:
        f.write(dumps(data))
    if not file_path.exists():
        logger.debug("Cache file could not be written!")
