// Diagnostic: the Householder null space written twice, as in ransac.hip (registers, unrolled) and as in
// oracle/ransac.c (arrays, loops), both on the GPU, printing the first quantity where they diverge.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#pragma clang fp contract(off)

struct Trace { double nrm[5], beta[5], v[5][9], a[5][9], N[4][9]; };

__device__ void ns_hip(const double* x1, const double* x2, Trace& T) {
    double a[5][9], v[5][9], beta[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        a[i][0] = u2 * u1; a[i][1] = u2 * v1; a[i][2] = u2;
        a[i][3] = v2 * u1; a[i][4] = v2 * v1; a[i][5] = v2;
        a[i][6] = u1; a[i][7] = v1; a[i][8] = 1.0;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        double sq = 0.0;
#pragma unroll
        for (int r = k; r < 9; ++r) sq = __builtin_fma(a[k][r], a[k][r], sq);
        const double nrm = sqrt(sq);
        T.nrm[k] = nrm;
        const double alpha = a[k][k] >= 0.0 ? -nrm : nrm;
#pragma unroll
        for (int r = k; r < 9; ++r) v[k][r] = a[k][r];
        v[k][k] = v[k][k] - alpha;
        double vv = 0.0;
#pragma unroll
        for (int r = k; r < 9; ++r) vv = __builtin_fma(v[k][r], v[k][r], vv);
        beta[k] = 2.0 / vv;
        T.beta[k] = beta[k];
#pragma unroll
        for (int r = 0; r < 9; ++r) T.v[k][r] = r >= k ? v[k][r] : 0.0;
#pragma unroll
        for (int c = k + 1; c < 5; ++c) {
            double d = 0.0;
#pragma unroll
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], a[c][r], d);
            d = d * beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) a[c][r] = __builtin_fma(-d, v[k][r], a[c][r]);
        }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int r = 0; r < 9; ++r) T.a[i][r] = a[i][r];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        double y[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) y[j] = j == 5 + n ? 1.0 : 0.0;
#pragma unroll
        for (int k = 4; k >= 0; --k) {
            double d = 0.0;
#pragma unroll
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], y[r], d);
            d = d * beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) y[r] = __builtin_fma(-d, v[k][r], y[r]);
        }
#pragma unroll
        for (int j = 0; j < 9; ++j) T.N[n][j] = y[j];
    }
}

__device__ __noinline__ void ns_oracle(const double* x1, const double* x2, Trace& T) {
    double q[5][9];
    for (int i = 0; i < 5; ++i) {
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        const double row[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        memcpy(q[i], row, sizeof(row));
    }
    double a[5][9], v[5][9], beta[5];
    memcpy(a, q, sizeof(a));
    memset(v, 0, sizeof(v));
    for (int k = 0; k < 5; ++k) {
        double s = 0.0;
        for (int r = k; r < 9; ++r) s = __builtin_fma(a[k][r], a[k][r], s);
        const double nrm = sqrt(s);
        T.nrm[k] = nrm;
        const double alpha = a[k][k] >= 0.0 ? -nrm : nrm;
        for (int r = k; r < 9; ++r) v[k][r] = a[k][r];
        v[k][k] = v[k][k] - alpha;
        double vv = 0.0;
        for (int r = k; r < 9; ++r) vv = __builtin_fma(v[k][r], v[k][r], vv);
        beta[k] = 2.0 / vv;
        T.beta[k] = beta[k];
        for (int r = 0; r < 9; ++r) T.v[k][r] = v[k][r];
        for (int c = k + 1; c < 5; ++c) {
            double d = 0.0;
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], a[c][r], d);
            d = d * beta[k];
            for (int r = k; r < 9; ++r) a[c][r] = __builtin_fma(-d, v[k][r], a[c][r]);
        }
    }
    memcpy(T.a, a, sizeof(a));
    for (int n = 0; n < 4; ++n) {
        double y[9] = {0};
        y[5 + n] = 1.0;
        for (int k = 4; k >= 0; --k) {
            double d = 0.0;
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], y[r], d);
            d = d * beta[k];
            for (int r = k; r < 9; ++r) y[r] = __builtin_fma(-d, v[k][r], y[r]);
        }
        for (int j = 0; j < 9; ++j) T.N[n][j] = y[j];
    }
}

__global__ void kk(const double* x1, const double* x2, Trace* th, Trace* to, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ns_hip(x1 + 10 * i, x2 + 10 * i, th[i]);
    ns_oracle(x1 + 10 * i, x2 + 10 * i, to[i]);
}

int main() {
    const int n = 256;
    double *x1 = (double*)malloc(n * 80), *x2 = (double*)malloc(n * 80);
    srand(3);
    for (int i = 0; i < n * 10; ++i) { x1[i] = (double)rand() / RAND_MAX - 0.5; x2[i] = (double)rand() / RAND_MAX - 0.5; }
    double *d1, *d2; Trace *th, *to;
    (void)hipMalloc(&d1, n * 80); (void)hipMalloc(&d2, n * 80);
    (void)hipMalloc(&th, n * sizeof(Trace)); (void)hipMalloc(&to, n * sizeof(Trace));
    (void)hipMemcpy(d1, x1, n * 80, hipMemcpyHostToDevice); (void)hipMemcpy(d2, x2, n * 80, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kk, dim3(n / 64), dim3(64), 0, 0, d1, d2, th, to, n);
    Trace* H = (Trace*)malloc(n * sizeof(Trace));
    Trace* O = (Trace*)malloc(n * sizeof(Trace));
    (void)hipMemcpy(H, th, n * sizeof(Trace), hipMemcpyDeviceToHost);
    (void)hipMemcpy(O, to, n * sizeof(Trace), hipMemcpyDeviceToHost);
    int shown = 0, diff_samples = 0;
    for (int s = 0; s < n; ++s) {
        const double* h = (const double*)&H[s];
        const double* o = (const double*)&O[s];
        const int cnt = sizeof(Trace) / 8;
        int first = -1;
        for (int i = 0; i < cnt; ++i)
            if (memcmp(&h[i], &o[i], 8)) { first = i; break; }
        if (first < 0) continue;
        ++diff_samples;
        if (shown++ < 3) {
            printf("sample %d differs at:", s);
            for (int i = 0; i < 100; ++i)
                if (memcmp(&h[i], &o[i], 8)) {
                    if (i < 5) printf(" nrm[%d]", i);
                    else if (i < 10) printf(" beta[%d]", i - 5);
                    else if (i < 55) printf(" v[%d][%d]", (i - 10) / 9, (i - 10) % 9);
                    else printf(" a[%d][%d]", (i - 55) / 9, (i - 55) % 9);
                }
            printf("\n");
        }
    }
    printf("samples with any divergence: %d of %d\n", diff_samples, n);
    return 0;
}
