// Diagnostic: ransac.hip's five-point null space (nullspace_5x9) against oracle/ransac.c's, both compiled for the GPU
// from their own sources, on the same random samples (built by tools/ubench/og_build.sh's generated oracle source).
#include "../../gtsfm_amd/csrc/ransac.hip"
#pragma clang attribute push(__attribute__((device)), apply_to = function)
namespace og {
#include "ransac_dev.c"
}
#pragma clang attribute pop

__global__ void kns(const double* x1, const double* x2, int n, double* Nh, double* No, int* okh, int* oko) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double N[4][9];
    okh[i] = nullspace_5x9(x1 + 10 * i, x2 + 10 * i, N) ? 1 : 0;
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 9; ++j) Nh[36 * i + 9 * k + j] = N[k][j];
    double q[5][9], M[4][9];
    for (int r = 0; r < 5; ++r) {
        const double u1 = x1[10 * i + 2 * r], v1 = x1[10 * i + 2 * r + 1], u2 = x2[10 * i + 2 * r], v2 = x2[10 * i + 2 * r + 1];
        const double row[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        for (int j = 0; j < 9; ++j) q[r][j] = row[j];
    }
    oko[i] = og::nullspace_5x9(q, M);
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 9; ++j) No[36 * i + 9 * k + j] = M[k][j];
}

int main() {
    const int n = 4096;
    double* x1 = (double*)malloc(n * 80);
    double* x2 = (double*)malloc(n * 80);
    srand(3);
    for (int i = 0; i < n * 10; ++i) {
        x1[i] = (double)rand() / RAND_MAX - 0.5;
        x2[i] = (double)rand() / RAND_MAX - 0.5;
    }
    double *d1, *d2, *dh, *dO;
    int *okh, *oko;
    (void)hipMalloc(&d1, n * 80); (void)hipMalloc(&d2, n * 80); (void)hipMalloc(&dh, n * 288); (void)hipMalloc(&dO, n * 288);
    (void)hipMalloc(&okh, n * 4); (void)hipMalloc(&oko, n * 4);
    (void)hipMemcpy(d1, x1, n * 80, hipMemcpyHostToDevice);
    (void)hipMemcpy(d2, x2, n * 80, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kns, dim3(n / 64), dim3(64), 0, 0, d1, d2, n, dh, dO, okh, oko);
    double* h = (double*)malloc(n * 288);
    double* o = (double*)malloc(n * 288);
    (void)hipMemcpy(h, dh, n * 288, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o, dO, n * 288, hipMemcpyDeviceToHost);
    int bad = 0;
    double worst = 0;
    for (int i = 0; i < n * 36; ++i) {
        const double d = fabs(h[i] - o[i]);
        if (d > 0) ++bad;
        if (d > worst) worst = d;
    }
    printf("nullspace_5x9 HIP vs oracle (both on the GPU): %d of %d values differ, max %.3e\n", bad, n * 36, worst);
    if (bad) {
        for (int i = 0; i < 4; ++i) printf("  sample 0 N[0][%d]: hip %.17g oracle %.17g\n", i, h[i], o[i]);
    }
    return 0;
}
