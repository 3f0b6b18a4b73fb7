// Micro-benchmark: cycles per v_med3_u32 / v_min3_u32 when the three sources share a VGPR bank vs not.
// Build: hipcc -O3 --offload-arch=gfx950 -o bank tools/ubench/bank.hip ; one wave per SIMD, s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(x) x x x x x x x x
template <int MODE>
__global__ __launch_bounds__(64) void k(unsigned long long* out, int iters) {
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n"
                 "v_mov_b32 v44, 5\n v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n"
                 "v_mov_b32 v48, 9\n v_mov_b32 v52, 10\n v_mov_b32 v56, 11\n" ::: "v40", "v41", "v42", "v43", "v44",
                 "v45", "v46", "v47", "v48", "v52", "v56");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0)  // sources in one bank (40, 44, 48 mod 4 == 0); 8 independent destinations
            asm volatile(REP8("v_med3_u32 v60, v40, v44, v48\n v_med3_u32 v61, v40, v44, v48\n"
                              "v_med3_u32 v62, v40, v44, v48\n v_med3_u32 v63, v40, v44, v48\n")
                         ::: "v60", "v61", "v62", "v63");
        else if (MODE == 1)  // sources in three banks (40, 41, 42)
            asm volatile(REP8("v_med3_u32 v60, v40, v41, v42\n v_med3_u32 v61, v40, v41, v42\n"
                              "v_med3_u32 v62, v40, v41, v42\n v_med3_u32 v63, v40, v41, v42\n")
                         ::: "v60", "v61", "v62", "v63");
        else if (MODE == 2)  // two sources share a bank (the row insert's pattern: 40, 44 + 41)
            asm volatile(REP8("v_med3_u32 v60, v41, v40, v44\n v_med3_u32 v61, v41, v40, v44\n"
                              "v_med3_u32 v62, v41, v40, v44\n v_med3_u32 v63, v41, v40, v44\n")
                         ::: "v60", "v61", "v62", "v63");
        else  // two-source VALU reference (v_min_u32, distinct banks)
            asm volatile(REP8("v_min_u32 v60, v40, v41\n v_min_u32 v61, v40, v41\n"
                              "v_min_u32 v62, v40, v41\n v_min_u32 v63, v40, v41\n")
                         ::: "v60", "v61", "v62", "v63");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
int main() {
    unsigned long long* d;
    hipMalloc(&d, 1024 * 8);
    const int iters = 2000;
    const char* names[4] = {"med3 same bank x3", "med3 3 banks", "med3 2 of 3 same bank", "min_u32 2 src"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1024), dim3(64), 0, 0, d, iters);
            if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1024), dim3(64), 0, 0, d, iters);
            if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1024), dim3(64), 0, 0, d, iters);
            if (m == 3) hipLaunchKernelGGL(k<3>, dim3(1024), dim3(64), 0, 0, d, iters);
            hipDeviceSynchronize();
        }
        unsigned long long h[1024];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 1024; ++i) s += h[i];
        printf("%-24s %.2f cycles per instruction (one wave per SIMD)\n", names[m], s / 1024 / (iters * 32.0));
    }
    return 0;
}
