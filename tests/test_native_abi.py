"""The C-ABI library loads on the CPU host and exports every symbol include/gtsfm_hip.h declares."""
import os
import re

import numpy as np

from tests.conftest import REPO


def _declared_functions():
    text = open(os.path.join(REPO, "include", "gtsfm_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gtsfm_[A-Za-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = _declared_functions()
    assert "gtsfm_match_batched" in names and "gtsfm_hip_abi_version" in names


def test_library_exports_every_declared_symbol():
    from gtsfm_amd import native

    lib = native.lib()
    for name in _declared_functions():
        assert hasattr(lib, name), name
        assert name in native.SIGNATURES, f"{name} has no ctypes signature in gtsfm_amd/native.py"
    assert lib.gtsfm_hip_abi_version() >= 100
    assert lib.gtsfm_hip_target() == b"gfx950"


def test_workspace_queries_without_gpu():
    from gtsfm_amd import native

    lib = native.lib()
    ws = lib.gtsfm_match_workspace_bytes(100, 2048, 128, 4950, native.GTSFM_MATCH_INT_F16)
    assert ws > 2 * 4950 * 2048 * 8
    assert lib.gtsfm_match_workspace_bytes(0, 2048, 128, 10, 1) == 0


def test_superpoint_weight_blob_layout():
    """The packed blob the Python side builds has exactly the size the library expects (include/gtsfm_hip.h)."""
    from gtsfm_amd import native
    from gtsfm_amd.frontend.detector_descriptor.superpoint import pack_superpoint_weights
    from superpoint_weights import superpoint_state_dict

    sd = superpoint_state_dict(0)
    blob = pack_superpoint_weights(sd)
    assert blob.dtype == np.float32 and blob.size == native.lib().gtsfm_superpoint_weights_floats()
    # conv1a occupies the first 9*64 weights + 64 biases: W[ky*3+kx][0][co] = weight[co][0][ky][kx]
    w = sd["conv1a.weight"]
    np.testing.assert_array_equal(blob[: 9 * 64].reshape(9, 64), w[:, 0].reshape(64, 9).T)
    np.testing.assert_array_equal(blob[9 * 64: 9 * 64 + 64], sd["conv1a.bias"])


def test_superglue_weight_blob_layout():
    from gtsfm_amd import native
    from gtsfm_amd.frontend.matcher.superglue_matcher import _head_major, pack_superglue_weights
    from superpoint_weights import superglue_state_dict

    sd = superglue_state_dict(0)
    blob = pack_superglue_weights(sd)
    assert blob.dtype == np.float32 and blob.size == native.lib().gtsfm_superglue_weights_floats(18)
    assert blob[-1] == sd["bin_score"]
    # head-major permutation: new channel h * 64 + d <- reference channel 4 d + h
    c = np.arange(256)
    perm = _head_major(c)
    assert perm[1] == 4 and perm[64] == 1 and sorted(perm.tolist()) == c.tolist()
