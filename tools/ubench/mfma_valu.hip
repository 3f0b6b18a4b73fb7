// Micro-benchmark: VALU issue rate of the distance-GEMM epilogue's v_min3/v_med3 insert chains beside waves streaming
// MFMAs on the same SIMD. 1024-thread workgroups, one per CU: waves w, w + 4, w + 8, w + 12 share a SIMD; the first
// n_mfma of a SIMD's four waves stream v_mfma_f32_32x32x16_f16 (VGPR accumulators), the next n_valu run the insert
// chains, the rest exit. Build: hipcc -O3 --offload-arch=gfx950 -o mfma_valu tools/ubench/mfma_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define REP4(x) x x x x

template <int VOP>  // 0: ins2x4 (VOP3 med3/min3 + min), 1: VOP2 only (max/min/min per value), 2: v_pk_min_u16 chains
__global__ __launch_bounds__(1024, 1) void k(unsigned long long* out, float* sink, int n_mfma, int n_valu,
                                             int mfma_iters, int valu_iters, int prio_m, int prio_v) {
    const int wave = threadIdx.x >> 6, role = wave >> 2;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = t0;
    if (role < n_mfma) {
        if (prio_m == 2) __builtin_amdgcn_s_setprio(2);
        half8 a, b;
        for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x + i); b[i] = (_Float16)(i - 3); }
        f32x16 c0 = {}, c1 = {};
        t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < mfma_iters; ++it)
            asm volatile(REP4("v_mfma_f32_32x32x16_f16 %0, %2, %3, %0\n v_mfma_f32_32x32x16_f16 %1, %2, %3, %1\n")
                         : "+v"(c0), "+v"(c1) : "v"(a), "v"(b));
        asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
        t1 = __builtin_amdgcn_s_memtime();
        float s = 0.f;
        for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
        sink[blockIdx.x * 1024 + threadIdx.x] = s;
    } else if (role < n_mfma + n_valu) {
        if (prio_v == 1) __builtin_amdgcn_s_setprio(1);
        unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y0 = x0 * 3, y1 = y0 + 5, y2 = y0 + 7,
                 y3 = y0 + 9, v0 = x0 ^ 77, v1 = x0 ^ 99, m0, m1, m2, m3;
        t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < valu_iters; ++it) {
            if (VOP == 0)
                asm volatile(
                    "v_med3_u32 %8, %0, %12, %13\n v_med3_u32 %9, %2, %12, %13\n"
                    "v_med3_u32 %10, %4, %12, %13\n v_med3_u32 %11, %6, %12, %13\n"
                    "v_min3_u32 %0, %0, %12, %13\n v_min3_u32 %2, %2, %12, %13\n"
                    "v_min3_u32 %4, %4, %12, %13\n v_min3_u32 %6, %6, %12, %13\n"
                    "v_min_u32 %1, %1, %8\n v_min_u32 %3, %3, %9\n v_min_u32 %5, %5, %10\n v_min_u32 %7, %7, %11\n"
                    : "+v"(x0), "+v"(y0), "+v"(x1), "+v"(y1), "+v"(x2), "+v"(y2), "+v"(x3), "+v"(y3), "=&v"(m0),
                      "=&v"(m1), "=&v"(m2), "=&v"(m3)
                    : "v"(v0), "v"(v1));
            else if (VOP == 1)
                asm volatile(
                    "v_max_u32 %8, %0, %12\n v_max_u32 %9, %2, %12\n v_max_u32 %10, %4, %12\n v_max_u32 %11, %6, %12\n"
                    "v_min_u32 %1, %1, %8\n v_min_u32 %3, %3, %9\n v_min_u32 %5, %5, %10\n v_min_u32 %7, %7, %11\n"
                    "v_min_u32 %0, %0, %12\n v_min_u32 %2, %2, %12\n v_min_u32 %4, %4, %12\n v_min_u32 %6, %6, %12\n"
                    : "+v"(x0), "+v"(y0), "+v"(x1), "+v"(y1), "+v"(x2), "+v"(y2), "+v"(x3), "+v"(y3), "=&v"(m0),
                      "=&v"(m1), "=&v"(m2), "=&v"(m3)
                    : "v"(v0), "v"(v1));
            else
                asm volatile(
                    "v_pk_max_u16 %8, %0, %12\n v_pk_max_u16 %9, %2, %12\n v_pk_max_u16 %10, %4, %12\n v_pk_max_u16 %11, %6, %12\n"
                    "v_pk_min_u16 %1, %1, %8\n v_pk_min_u16 %3, %3, %9\n v_pk_min_u16 %5, %5, %10\n v_pk_min_u16 %7, %7, %11\n"
                    "v_pk_min_u16 %0, %0, %12\n v_pk_min_u16 %2, %2, %12\n v_pk_min_u16 %4, %4, %12\n v_pk_min_u16 %6, %6, %12\n"
                    : "+v"(x0), "+v"(y0), "+v"(x1), "+v"(y1), "+v"(x2), "+v"(y2), "+v"(x3), "+v"(y3), "=&v"(m0),
                      "=&v"(m1), "=&v"(m2), "=&v"(m3)
                    : "v"(v0), "v"(v1));
            v0 += 13;
        }
        t1 = __builtin_amdgcn_s_memtime();
        sink[blockIdx.x * 1024 + threadIdx.x] = (float)(x0 + y0 + x1 + y1 + x2 + y2 + x3 + y3);
    }
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + wave] = t1 - t0;
}

template <int VOP>
void run(unsigned long long* d, float* sink, int nm, int nv, int pm, int pv) {
    static unsigned long long h[256 * 16];
    const int mi = 2000, vi = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<VOP>, dim3(256), dim3(1024), 0, 0, d, sink, nm, nv, mi, vi, pm, pv);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double mf = 0, va = 0, vmax = 0;
    int cm = 0, cv = 0;
    for (int b = 0; b < 256; ++b)
        for (int w = 0; w < 16; ++w) {
            const int role = w >> 2;
            if (role < nm) { mf += h[b * 16 + w]; ++cm; }
            else if (role < nm + nv) { va += h[b * 16 + w]; ++cv; if (h[b * 16 + w] > vmax) vmax = h[b * 16 + w]; }
        }
    const char* vn[3] = {"ins2x4 VOP3", "VOP2 max/min/min", "v_pk_min/max_u16"};
    printf("%-18s mfma waves/SIMD %d valu waves/SIMD %d prio m%d v%d: cycles/MFMA %5.1f  cycles/VALU per wave %5.2f "
           "(slowest %5.2f) -> per SIMD %5.2f\n",
           vn[VOP], nm, nv, pm, pv, cm ? mf / cm / (8.0 * mi) : 0.0, cv ? va / cv / (13.0 * vi) : 0.0,
           vmax / (13.0 * vi), cv ? va / cv / (13.0 * vi) / nv : 0.0);
}

int main() {
    unsigned long long* d;
    float* sink;
    (void)hipMalloc(&d, 256 * 16 * 8);
    (void)hipMalloc(&sink, 256 * 1024 * 4);
    for (int nv = 1; nv <= 4; ++nv) run<0>(d, sink, 0, nv, 0, 0);
    for (int nv = 1; nv <= 3; ++nv) run<0>(d, sink, 1, nv, 0, 0);
    for (int nv = 1; nv <= 2; ++nv) run<0>(d, sink, 2, nv, 0, 0);
    run<0>(d, sink, 1, 3, 2, 0);
    run<0>(d, sink, 2, 2, 2, 0);
    for (int nv = 1; nv <= 3; ++nv) run<1>(d, sink, 0, nv, 0, 0);
    run<1>(d, sink, 1, 3, 0, 0);
    for (int nv = 1; nv <= 3; ++nv) run<2>(d, sink, 0, nv, 0, 0);
    run<2>(d, sink, 1, 3, 0, 0);
    return 0;
}
