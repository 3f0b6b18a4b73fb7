// Squared Sampson distances of correspondences to per-pair fundamental / essential matrices.
//
// Reference: gtsfm/utils/verification.py:170-214 compute_epipolar_distances_sq_sampson, used by the two-view report's
// ground-truth metrics (gtsfm/utils/metrics.py:99-128: inlier iff d^2 < eval_threshold^2):
//   l2 = F x1, l1 = F^T x2, d^2 = (x2^T F x1)^2 / (l1_x^2 + l1_y^2 + l2_x^2 + l2_y^2).
// Two arithmetics: GTSFM_SAMPSON_F64 is the reference's numpy float64 evaluation (the GT metrics);
// GTSFM_SAMPSON_F32_VERIFIER evaluates exactly the fp32 FMA expression the RANSAC score kernel thresholds
// (ransac.hip sampson_inlier), so tests can pin the verifier's arithmetic to the reference's known answers.
// Thread per correspondence; rows of all pairs in one launch.
#include "common.hpp"

namespace {

__global__ __launch_bounds__(256) void sampson_f64_kernel(const double* __restrict__ F, const int* __restrict__ row_pair,
                                                          const double* __restrict__ x1, const double* __restrict__ x2,
                                                          int n, double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double* f = F + 9 * (size_t)row_pair[i];
    const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
    const double l2x = f[0] * u1 + f[1] * v1 + f[2], l2y = f[3] * u1 + f[4] * v1 + f[5];
    const double l2z = f[6] * u1 + f[7] * v1 + f[8];
    const double l1x = f[0] * u2 + f[3] * v2 + f[6], l1y = f[1] * u2 + f[4] * v2 + f[7];
    const double num = u2 * l2x + v2 * l2y + l2z;
    out[i] = num * num / (l1x * l1x + l1y * l1y + l2x * l2x + l2y * l2y);
}

// ransac.hip sampson_inlier's expression with E in float (a: E x1 rows, b: E^T x2 rows)
__global__ __launch_bounds__(256) void sampson_f32_kernel(const double* __restrict__ F, const int* __restrict__ row_pair,
                                                          const double* __restrict__ x1, const double* __restrict__ x2,
                                                          int n, double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double* fd = F + 9 * (size_t)row_pair[i];
    float E[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) E[k] = (float)fd[k];
    const float px = (float)x1[2 * i], py = (float)x1[2 * i + 1], pz = (float)x2[2 * i], pw = (float)x2[2 * i + 1];
    const float a0 = fmaf(E[1], py, fmaf(E[0], px, E[2]));
    const float a1 = fmaf(E[4], py, fmaf(E[3], px, E[5]));
    const float a2 = fmaf(E[7], py, fmaf(E[6], px, E[8]));
    const float b0 = fmaf(E[3], pw, fmaf(E[0], pz, E[6]));
    const float b1 = fmaf(E[4], pw, fmaf(E[1], pz, E[7]));
    const float num = fmaf(pw, a1, fmaf(pz, a0, a2));
    const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, __fmul_rn(a0, a0))));
    out[i] = (double)__fmul_rn(num, num) / (double)den;
}

}  // namespace

extern "C" {

int gtsfm_sampson_sq_batched(const double* d_F, int n_mats, const int* d_row_pair, const double* d_x1,
                             const double* d_x2, int n_rows, int precision, double* d_out, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_rows < 0 || n_mats < 0) return GTSFM_ERR_ARG;
    if (n_rows == 0) return GTSFM_OK;
    if (!d_F || !d_row_pair || !d_x1 || !d_x2 || !d_out || n_mats == 0) return GTSFM_ERR_ARG;
    const dim3 grid((n_rows + 255) / 256);
    if (precision == GTSFM_SAMPSON_F64)
        hipLaunchKernelGGL(sampson_f64_kernel, grid, dim3(256), 0, stream, d_F, d_row_pair, d_x1, d_x2, n_rows, d_out);
    else if (precision == GTSFM_SAMPSON_F32_VERIFIER)
        hipLaunchKernelGGL(sampson_f32_kernel, grid, dim3(256), 0, stream, d_F, d_row_pair, d_x1, d_x2, n_rows, d_out);
    else
        return GTSFM_ERR_ARG;
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
