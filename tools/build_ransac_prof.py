"""Builds gtsfm_amd/_lib/prof/libgtsfm_hip.so: ransac.hip with phase timers (s_memtime) for tools/ransac_phases.py.
Not part of the product; the instrumented copy lives in /tmp."""
import os, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "gtsfm_amd/csrc/ransac.hip")).read()
anchors = [  # (text that starts a line, mark id) -- mark k times the code since the previous mark
    ("    if (!nullspace_5x9(x1, x2, m, N)) return 0;", 0),
    ("    LaneArr<double> A = m.u;  // [10][20]", 1),
    ("    double EEt[3][3][10], tr[10], tmp[10];", 2),
    ("    double B[3][3][5];", 3),
    ("    int nsol = 0;", 4),
    ("    double R[kChain];", 5),
    ("    double lo[kMaxSol], hi[kMaxSol], flo[kMaxSol];", 6),
    ("    LaneArr<double> roots = iv_a;", 7),
    ("    nsol[(size_t)p * kBatch + lane] = ns;", 8),
]
for text, k in anchors:
    assert s.count(text) == 1, text
    s = s.replace(text, f"    prof_mark({k});\n" + text)
s = s.replace("    if (sample5(seed, pair_ids ? pair_ids[p] : pair_id_base + p, done + lane, M, idx)) {",
              "    prof_mark(-1);\n    if (sample5(seed, pair_ids ? pair_ids[p] : pair_id_base + p, done + lane, M, idx)) {")
hdr = """
__device__ unsigned long long g_prof[16];
__device__ __forceinline__ void prof_mark(int k) {
    __shared__ unsigned long long t_prev;
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (k >= 0 && threadIdx.x == 0) atomicAdd(&g_prof[k], now - t_prev);
    if (threadIdx.x == 0) t_prev = now;
}
"""
s = s.replace("namespace {", "namespace {" + hdr, 1)
s = s.replace('extern "C" {', '''extern "C" {
int gtsfm_ransac_profile(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)) == hipSuccess ? 0 : -1;
}''', 1)
os.makedirs("/tmp/prof", exist_ok=True)
open("/tmp/prof/ransac_prof.hip", "w").write(s)
hipcc = "/opt/rocm/bin/hipcc"
flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{REPO}/include", f"-I{REPO}/gtsfm_amd/csrc"]
subprocess.check_call([hipcc, *flags, "-c", "/tmp/prof/ransac_prof.hip", "-o", "/tmp/prof/ransac_prof.o"])
obj = f"{REPO}/gtsfm_amd/_lib/obj"
os.makedirs(f"{REPO}/gtsfm_amd/_lib/prof", exist_ok=True)
subprocess.check_call([hipcc, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", f"{REPO}/gtsfm_amd/_lib/prof/libgtsfm_hip.so",
                       *[os.path.join(obj, f) for f in sorted(os.listdir(obj)) if f.endswith(".o") and f != "ransac.o"],
                       "/tmp/prof/ransac_prof.o"])
print("built")
