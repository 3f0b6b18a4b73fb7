"""Loader for libgtsfm_hip.so, the gfx950 C-ABI library behind every gtsfm_amd plugin.

There is no fallback: if the library is missing or cannot be loaded, importing the product path raises.
torch is imported first so that the process has exactly one HIP runtime (torch's bundled libamdhip64.so.7 and
ours share the SONAME, so the loader reuses torch's copy).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load: one HIP runtime per process)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# GTSFM_HIP_LIB: development override (instrumented or experimental builds of the same ABI); unset in production
LIB_PATH = os.environ.get("GTSFM_HIP_LIB") or os.path.join(_PKG_DIR, "_lib", "libgtsfm_hip.so")
CSRC_DIR = os.path.join(_PKG_DIR, "csrc")

_lib: Optional[ctypes.CDLL] = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_double = ctypes.c_double
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
c_uint64 = ctypes.c_uint64

# Mirrors include/gtsfm_hip.h
ABI_VERSION = 402  # GTSFM_HIP_ABI_VERSION: lib() refuses a library built for another ABI
GTSFM_OK = 0
GTSFM_ERR_ARG = -1
GTSFM_ERR_HIP = -2
GTSFM_ERR_CAPACITY = -3
GTSFM_MATCH_EXACT_F32 = 0
GTSFM_MATCH_INT_F16 = 1
GTSFM_MATCH_F16_RERANK = 2
GTSFM_SAMPSON_F64 = 0
GTSFM_SAMPSON_F32_VERIFIER = 1
RANSAC_STATUS_OK = 0
RANSAC_STATUS_TOO_FEW = 1
RANSAC_STATUS_NO_MODEL = 2
RANSAC_DEFAULT_SEED = 0x5EED5EED
GTSFM_RANSAC_SCORING_RANSAC = 0
GTSFM_RANSAC_SCORING_MSAC = 1
BA2_STATUS_OK = 0
BA2_STATUS_NO_TRACKS = 1
BA2_STATUS_NONE_VALID = 2
BA2_STATUS_NOT_RUN = 3

# (name, restype, argtypes) of every symbol declared in include/gtsfm_hip.h
SIGNATURES = {
    "gtsfm_hip_abi_version": (c_int, []),
    "gtsfm_hip_target": (ctypes.c_char_p, []),
    "gtsfm_match_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "gtsfm_match_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_double, c_int, c_void_p, c_size_t, c_void_p,
         c_void_p, c_void_p],
    ),
    "gtsfm_match_batched_grouped": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_double, c_int, c_void_p,
         c_size_t, c_void_p, c_void_p, c_void_p],
    ),
    "gtsfm_match_max_group": (c_int, [c_int, c_int]),
    "gtsfm_match_set_kernel_events": (c_int, [c_void_p, c_void_p]),
    "gtsfm_match_rerank_stats": (c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gtsfm_ransac_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gtsfm_ransac_E_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_double, c_double, c_int, c_int,
         c_uint64, c_int, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p],
    ),
    "gtsfm_ransac_F_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gtsfm_ransac_F_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_double, c_double, c_int,
         c_uint64, c_int, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
    "gtsfm_superpoint_weights_floats": (c_size_t, []),
    "gtsfm_superpoint_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gtsfm_superpoint_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_size_t,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "gtsfm_superglue_weights_floats": (c_size_t, [c_int]),
    "gtsfm_superglue_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gtsfm_superglue_batched": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
         c_float, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "gtsfm_superglue_log_assignment": (c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_void_p, c_void_p]),
    "gtsfm_retrieval_similarity": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "gtsfm_retrieval_pairs": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, ctypes.c_float, c_int, c_void_p, c_void_p,
                                      c_void_p]),
    "gtsfm_netvlad_weights_floats": (c_size_t, []),
    "gtsfm_netvlad_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "gtsfm_netvlad_batched": (
        c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gtsfm_compact_verified": (
        c_int,
        [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double, c_void_p, c_void_p,
         c_int, c_void_p, c_void_p],
    ),
    "gtsfm_ba2_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gtsfm_ba2_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_int, c_int, c_double, c_double, c_void_p, c_size_t, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "gtsfm_sampson_sq_batched": (
        c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gtsfm_sift_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gtsfm_sift_batched": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p],
    ),
}


class NativeError(RuntimeError):
    pass


def build(jobs: int = 8) -> str:
    """Compiles every HIP source under gtsfm_amd/csrc for gfx950 into gtsfm_amd/_lib/libgtsfm_hip.so."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC_DIR], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(the gtsfm_amd product path has no CPU fallback)"
            )
        handle = ctypes.CDLL(LIB_PATH)
        ver = getattr(handle, "gtsfm_hip_abi_version", None)
        if ver is None:
            raise NativeError(f"{LIB_PATH} does not export gtsfm_hip_abi_version")
        ver.restype, ver.argtypes = c_int, []
        if ver() != ABI_VERSION:
            raise NativeError(f"{LIB_PATH} implements ABI {ver()}, this binding expects {ABI_VERSION}: rebuild it")
        for name, (restype, argtypes) in SIGNATURES.items():
            fn = getattr(handle, name, None)
            if fn is None:
                raise NativeError(f"{LIB_PATH} does not export {name}")
            fn.restype = restype
            fn.argtypes = argtypes
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != GTSFM_OK:
        raise NativeError(f"{what} failed with status {rc}")


def stream_handle(stream: Optional["torch.cuda.Stream"] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise NativeError("gtsfm_amd needs an MI355X (gfx950) GPU: torch.cuda.is_available() is False")
