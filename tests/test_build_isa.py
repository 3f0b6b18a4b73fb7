"""Checks on the built gfx950 code object (CPU only: disassembly, no GPU).

The streaming blur (`blur_stream_kernel<R>`, gtsfm_amd/csrc/sift.hip) issues its LDS-DMA loads
(`global_load_lds_dword`, whose LDS address is taken from M0) from inline asm. Until round 5 the asm wrote M0 itself
and listed it as a clobber, which the compiler ignores for reserved registers (1408 -Winline-asm warnings): nothing
but a manual ISA read guaranteed that no compiler-held value lived in M0 across those statements. Now the address is
an M0 operand ("{m0}" constraint), so the compiler writes M0 and knows it is read. These tests pin that down on the
code object actually built:
- no inline-asm statement in the kernels lists M0 as a clobber;
- in every streaming-blur kernel, each `global_load_lds_dword` is preceded, in the same straight-line block, by a
  scalar write of M0 (`s_mov_b32 m0, ...` / `s_add_i32 m0, ...`) and then the hazard `s_nop`, and nothing between that write and the load touches M0.
"""
import os
import re
import subprocess

import pytest

from tests.conftest import REPO

LLVM = "/opt/rocm/lib/llvm/bin"
CSRC = os.path.join(REPO, "gtsfm_amd", "csrc")
OBJ = os.path.join(REPO, "gtsfm_amd", "_lib", "obj", "sift.o")


def test_no_m0_clobbers_in_sources():
    for name in os.listdir(CSRC):
        if name.endswith((".hip", ".hpp")):
            src = open(os.path.join(CSRC, name)).read()
            assert not re.search(r':\s*"[^"]*"\s*,\s*"m0"|"m0"\s*\)', src), name


@pytest.fixture(scope="module")
def sift_isa(tmp_path_factory):
    if not (os.path.exists(os.path.join(LLVM, "llvm-objdump")) and os.path.exists("/opt/rocm/bin/hipcc")):
        pytest.skip("ROCm LLVM tools absent")
    if not os.path.exists(OBJ):
        subprocess.run(["make", "-s", "-j8", "-C", CSRC], check=True)
    d = tmp_path_factory.mktemp("isa")
    fat, co = str(d / "fat.bin"), str(d / "sift.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", OBJ, str(d / "host.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    kernels, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            kernels[cur] = []
        elif cur is not None and line.strip():
            kernels[cur].append(line.split("//")[0].strip())
    return kernels


def test_stream_blur_lds_dma_m0_writes(sift_isa):
    stream = {k: v for k, v in sift_isa.items() if "blur_stream_kernel" in k}
    assert len(stream) >= 3, sorted(sift_isa)[:10]
    n_loads = 0
    for name, ins in stream.items():
        for i, text in enumerate(ins):
            if not text.startswith("global_load_lds_dword"):
                continue
            n_loads += 1
            assert ins[i - 1].startswith("s_nop"), (name, i, ins[i - 2: i + 1])
            j = i - 2
            while j >= 0 and not re.match(r"s_\w+ m0,", ins[j]):  # s_mov_b32 / s_add_i32 m0, ...
                # straight-line: no label / branch between the M0 write and the load, and no other M0 access
                assert not re.match(r"s_(cbranch|branch|setpc|swappc)", ins[j]), (name, i, ins[j])
                assert "m0" not in ins[j], (name, i, ins[j])
                j -= 1
            assert j >= 0, (name, i)
    assert n_loads >= 16 * len(stream)
