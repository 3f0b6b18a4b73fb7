"""INTEGRATION.md's reference-side binding cannot drift from the ABI: its ctypes block is executed against a recording
stand-in for the library, and every argtypes / restype it sets must equal gtsfm_amd.native.SIGNATURES, which must in
turn match the header's parameter counts (include/gtsfm_hip.h)."""
import ctypes
import os
import re

from tests.conftest import REPO


def _header_abi_version() -> int:
    text = open(os.path.join(REPO, "include", "gtsfm_hip.h")).read()
    return int(re.search(r"#define GTSFM_HIP_ABI_VERSION (\d+)", text).group(1))


class _Fn:
    def __init__(self):
        self.argtypes = None
        self.restype = "unset"

    def __call__(self):  # only the version query is called at bind time
        return _header_abi_version()


class _RecordingLib:
    def __init__(self):
        self.fns = {}

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return self.fns.setdefault(name, _Fn())


def _binding_block() -> str:
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"```python\n(# gtsfm/frontend/hip/_lib\.py.*?)```", text, flags=re.S)
    assert m, "INTEGRATION.md lost its ctypes binding block"
    return m.group(1)


def _header_arity():
    text = open(os.path.join(REPO, "include", "gtsfm_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for name, params in re.findall(r"\b(gtsfm_[A-Za-z0-9_]+)\s*\(([^)]*)\)\s*;", text, flags=re.S):
        params = params.strip()
        out[name] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_integration_binding_equals_native_signatures():
    from gtsfm_amd import native

    rec = _RecordingLib()
    src = _binding_block()
    # the block loads the library by name and imports torch; run everything after the CDLL line against the recorder
    body = src.split("_LIB = ctypes.CDLL", 1)[1].split("\n", 1)[1]
    ns = {"ctypes": ctypes, "_LIB": rec}
    exec(body, ns)
    missing = sorted(set(native.SIGNATURES) - set(rec.fns))
    assert not missing, f"INTEGRATION.md does not bind {missing}"
    for name, fn in rec.fns.items():
        assert name in native.SIGNATURES, f"INTEGRATION.md binds {name}, which the ABI does not declare"
        restype, argtypes = native.SIGNATURES[name]
        assert fn.argtypes == argtypes, f"{name}: INTEGRATION.md argtypes {fn.argtypes} != native {argtypes}"
        assert fn.restype == restype, f"{name}: INTEGRATION.md restype {fn.restype} != native {restype}"


def test_native_signatures_match_header_arity():
    from gtsfm_amd import native

    arity = _header_arity()
    for name, (_, argtypes) in native.SIGNATURES.items():
        assert name in arity, f"{name} is not declared in include/gtsfm_hip.h"
        assert len(argtypes) == arity[name], f"{name}: native.py has {len(argtypes)} args, header {arity[name]}"


def test_abi_version_agrees_everywhere():
    """header #define == native.ABI_VERSION == INTEGRATION.md's check == what the library returns."""
    from gtsfm_amd import native

    v = _header_abi_version()
    assert native.ABI_VERSION == v
    assert f"GTSFM_HIP_ABI_VERSION = {v}" in _binding_block()
    assert native.lib().gtsfm_hip_abi_version() == v
