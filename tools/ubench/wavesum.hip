// Checks the fp64 wave reduction of ransac.hip (wave_sum_f64: DPP row_shr 1/2/4/8 scan, row_bcast 15/31) against the
// host restatement oracle/ransac.c wave_sum_order uses, bit for bit, on random data.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/wavesum.hip -o tools/ubench/wavesum && ./tools/ubench/wavesum
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#pragma clang fp contract(off)

__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
    const long long b = __double_as_longlong(v);
    int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    switch (ctrl_sel) {
        case 0: lo = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, false); break;
        case 1: lo = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xf, 0xf, false); break;
        case 2: lo = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xf, 0xf, false); break;
        case 3: lo = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xf, 0xf, false); break;
        case 4: lo = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xa, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xa, 0xf, false); break;
        default: lo = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xc, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xc, 0xf, false); break;
    }
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ void k(const double* in, double* out, double* lanes) {
    double v = in[blockIdx.x * 64 + threadIdx.x];
#pragma unroll
    for (int c = 0; c < 6; ++c) v += dpp_f64(v, c);
    lanes[blockIdx.x * 64 + threadIdx.x] = v;
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    if (threadIdx.x == 0) out[blockIdx.x] = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

static double host_order(const double* in, double* lanes_out) {
    double v[64], t[64];
    memcpy(v, in, sizeof(v));
    for (int n = 1; n <= 8; n <<= 1) {
        memcpy(t, v, sizeof(t));
        for (int i = 0; i < 64; ++i) v[i] = t[i] + ((i & 15) >= n ? t[i - n] : 0.0);
    }
    memcpy(t, v, sizeof(t));
    for (int i = 0; i < 64; ++i) {
        const int r = i >> 4;
        v[i] = t[i] + ((r == 1 || r == 3) ? t[16 * r - 1] : 0.0);
    }
    memcpy(t, v, sizeof(t));
    for (int i = 0; i < 64; ++i) v[i] = t[i] + ((i >> 4) >= 2 ? t[31] : 0.0);
    memcpy(lanes_out, v, sizeof(v));
    return v[63];
}

int main() {
    const int n = 4096;
    double* h = (double*)malloc(n * 64 * sizeof(double));
    srand(7);
    for (int i = 0; i < n * 64; ++i) {
        const double u = (double)rand() / RAND_MAX - 0.5, e = (double)(rand() % 40 - 20);
        h[i] = (i % 5 == 0) ? 0.0 : u * __builtin_pow(2.0, e);
    }
    double *din, *dout, *dl;
    hipMalloc(&din, n * 64 * 8); hipMalloc(&dout, n * 8); hipMalloc(&dl, n * 64 * 8);
    hipMemcpy(din, h, n * 64 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n), dim3(64), 0, 0, din, dout, dl);
    double* o = (double*)malloc(n * 8);
    double* l = (double*)malloc(n * 64 * 8);
    hipMemcpy(o, dout, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(l, dl, n * 64 * 8, hipMemcpyDeviceToHost);
    int bad = 0, bad_lanes = 0;
    for (int b = 0; b < n; ++b) {
        double hl[64];
        const double r = host_order(h + 64 * b, hl);
        if (memcmp(&r, &o[b], 8)) {
            if (bad < 3) printf("block %d: device %.17g host %.17g\n", b, o[b], r);
            ++bad;
        }
        for (int i = 0; i < 64; ++i)
            if (memcmp(&hl[i], &l[64 * b + i], 8)) {
                if (bad_lanes < 5) printf("block %d lane %d: device %.17g host %.17g\n", b, i, l[64 * b + i], hl[i]);
                ++bad_lanes;
            }
    }
    printf("wave_sum_f64 vs host order: %d of %d totals differ, %d of %d lane values differ\n", bad, n, bad_lanes, n * 64);
    return bad ? 1 : 0;
}
