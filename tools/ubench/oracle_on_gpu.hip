// Diagnostic: oracle/ransac.c's five-point solver compiled as GPU device code (tools/ubench/og_build.sh), to tell
// hardware / compiler arithmetic differences from restatement differences in the HIP solver.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#pragma clang fp contract(off)
#pragma clang attribute push(__attribute__((device)), apply_to = function)
#define static_globals
namespace og {
#include "ransac_dev.c"
}
#pragma clang attribute pop
__global__ void kfp(const double* x1, const double* x2, int n, double* Es, int* ns, double* N, double* Rt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ns[i] = og::oracle_five_point(x1 + 10 * i, x2 + 10 * i, Es + 90 * i, N + 36 * i, Rt + 60 * i);
}
// per sample: up to 10 E (90 doubles), the solution count, N (36) and the reduced rows (60)
extern "C" int og_five_point_batch(const double* x1, const double* x2, int n, double* Es, int* ns, double* N,
                                   double* Rt) {
    double *d1, *d2, *dE, *dN, *dR; int* dn;
    hipMalloc(&d1, n * 80); hipMalloc(&d2, n * 80); hipMalloc(&dE, n * 720); hipMalloc(&dn, n * 4);
    hipMalloc(&dN, n * 36 * 8); hipMalloc(&dR, n * 60 * 8);
    hipMemcpy(d1, x1, n * 80, hipMemcpyHostToDevice); hipMemcpy(d2, x2, n * 80, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kfp, dim3((n + 63) / 64), dim3(64), 0, 0, d1, d2, n, dE, dn, dN, dR);
    hipMemcpy(Es, dE, n * 720, hipMemcpyDeviceToHost); hipMemcpy(ns, dn, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(N, dN, n * 36 * 8, hipMemcpyDeviceToHost); hipMemcpy(Rt, dR, n * 60 * 8, hipMemcpyDeviceToHost);
    hipFree(d1); hipFree(d2); hipFree(dE); hipFree(dn); hipFree(dN); hipFree(dR);
    return (int)hipGetLastError();
}
