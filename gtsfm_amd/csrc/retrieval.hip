// Global-descriptor retrieval (gfx950): the NetVLAD similarity matrix and the top-k pair selection.
//
// Replaces gtsfm/retriever/netvlad_retriever.py:77-133 (NetVLADRetriever.compute_similarity_matrix: a blocked
// einsum "id,jd->ij" over the upper block-triangle, blocks of `blocksize` images, aggregated into an N x N matrix that
// is zero below the block diagonal, :146-159) and :150-235 (compute_pairs_from_similarity_matrix +
// pairs_from_score_matrix: scores below min_score and the non-strict-upper triangle masked to -inf, torch.topk per
// row, the finite entries emitted row by row in rank order).
//
// similarity_kernel: one fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32) over 64 x 64 output tiles of the upper block
// triangle, K streamed through LDS in 32-deep chunks (fp32 accumulation like the reference's fp32 einsum; the
// summation order differs, so parity is a tolerance). Tiles entirely below the block diagonal are skipped, and their
// elements -- and every element with block(j) < block(i) -- are written as 0 exactly as the reference's aggregate.
// pairs_kernel: one 256-thread workgroup per row; k rounds of a block-wide argmax in torch.topk order (NaN, then score
// descending, ties by lowest column) over the valid columns (j > i, not score < min_score); finite winners are
// emitted in rank order.
#include "common.hpp"

namespace {

constexpr int kSimTile = 64, kSimK = 32, kSimThreads = 256;

__global__ __launch_bounds__(kSimThreads) void similarity_kernel(const float* __restrict__ desc, int n, int d,
                                                                 int blocksize, int n_tiles, float* __restrict__ sim) {
    __shared__ float As[kSimK][kSimTile + 4];  // [k][row]
    __shared__ float Bs[kSimK][kSimTile + 4];  // [k][col]
    const int ti = blockIdx.y, tj = blockIdx.x;
    const int i0 = ti * kSimTile, j0 = tj * kSimTile;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // row / column images of this tile; a tile with every column block below every row block is all zero
    const int last_j = min(j0 + kSimTile, n) - 1;
    const bool any_upper = (last_j / blocksize) >= (i0 / blocksize);
    f32x16 acc = {};
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;  // this wave's 32 x 32 quadrant
    if (any_upper) {
        for (int k0 = 0; k0 < d; k0 += kSimK) {
            // stage A (rows i0.., k0..) and B (rows j0.., k0..) transposed to [k][row]: 64 x 32 floats each
            for (int e = tid; e < kSimTile * kSimK; e += kSimThreads) {
                const int r = e / kSimK, k = e % kSimK;
                const int gi = i0 + r, gj = j0 + r, gk = k0 + k;
                As[k][r] = (gi < n && gk < d) ? desc[(size_t)gi * d + gk] : 0.f;
                Bs[k][r] = (gj < n && gk < d) ? desc[(size_t)gj * d + gk] : 0.f;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kSimK; k += 2) {
                // lane l: A[row = l % 32][k + l / 32], B[k + l / 32][col = l % 32]
                const float a = As[k + (lane >> 5)][wr + (lane & 31)];
                const float b = Bs[k + (lane >> 5)][wc + (lane & 31)];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            }
            __syncthreads();
        }
    }
    // store: lane holds column wc + (lane & 31), rows wr + (g & 3) + 8 (g >> 2) + 4 (lane >> 5)
    const int j = j0 + wc + (lane & 31);
    if (j >= n) return;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        const int i = i0 + wr + (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5);
        if (i >= n) continue;
        sim[(size_t)i * n + j] = (j / blocksize >= i / blocksize) ? acc[g] : 0.f;
    }
    (void)n_tiles;
}

constexpr int kPairThreads = 256;

// Total order of torch.topk over one masked row: NaN first (torch sorts NaN above +inf), then value descending; equal
// keys by ascending column (torch leaves tie order unspecified; the oracle uses this same rule).
__device__ __forceinline__ bool pair_before(float v, int j, float w, int q) {
    const bool vn = v != v, wn = w != w;
    if (vn != wn) return vn;
    if (!vn && v != w) return v > w;
    return j < q;
}

__global__ __launch_bounds__(kPairThreads) void pairs_kernel(const float* __restrict__ sim, int n, int n_cols,
                                                             const uint8_t* __restrict__ invalid, int k,
                                                             float min_score, int use_min, int* __restrict__ out,
                                                             int* __restrict__ row_count) {
    __shared__ float red_v[kPairThreads];
    __shared__ int red_j[kPairThreads];
    const int i = blockIdx.x, tid = threadIdx.x;
    const float* row = sim + (size_t)i * n_cols;
    const uint8_t* bad = invalid ? invalid + (size_t)i * n_cols : nullptr;
    const int j_first = invalid ? 0 : i + 1;  // no mask given: the retriever's strict upper triangle
    // rank r selects the best valid column strictly after the rank r-1 selection in pair_before order, so no
    // selected-set bookkeeping is needed. Valid: j > i (the strict upper triangle) and not (score < min_score) --
    // NaN passes the min_score mask exactly as in the reference and occupies a top-k slot, but is never emitted.
    float last_v = 0.f;
    int last_j = -1, cnt = 0;
    for (int r = 0; r < k; ++r) {
        float bv = 0.f;
        int bj = -1;
        for (int j = j_first + tid; j < n_cols; j += kPairThreads) {
            if (bad && bad[j]) continue;
            const float v = row[j];
            if (v == -__builtin_inff()) continue;  // the reference's -inf fill: never finite, never emitted
            if (use_min && v < min_score) continue;
            if (last_j >= 0 && !pair_before(last_v, last_j, v, j)) continue;
            if (bj < 0 || pair_before(v, j, bv, bj)) { bv = v; bj = j; }
        }
        red_v[tid] = bv;
        red_j[tid] = bj;
        __syncthreads();
        for (int s = kPairThreads / 2; s > 0; s >>= 1) {
            if (tid < s) {
                const float ov = red_v[tid + s];
                const int oj = red_j[tid + s];
                if (oj >= 0 && (red_j[tid] < 0 || pair_before(ov, oj, red_v[tid], red_j[tid]))) {
                    red_v[tid] = ov;
                    red_j[tid] = oj;
                }
            }
            __syncthreads();
        }
        const float vbest = red_v[0];
        const int jbest = red_j[0];
        __syncthreads();
        if (jbest < 0) break;  // only -inf left: the reference's remaining top-k values are not finite
        if (__builtin_isfinite(vbest)) {
            if (tid == 0) {
                out[((size_t)i * k + cnt) * 2] = i;
                out[((size_t)i * k + cnt) * 2 + 1] = jbest;
            }
            ++cnt;
        }
        last_v = vbest;
        last_j = jbest;
    }
    if (tid == 0) row_count[i] = cnt;
}

}  // namespace

extern "C" {

int gtsfm_retrieval_similarity(const float* d_desc, int n_img, int dim, int blocksize, float* d_sim, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_img == 0) return GTSFM_OK;
    if (!d_desc || !d_sim || n_img < 0 || dim <= 0 || blocksize <= 0) return GTSFM_ERR_ARG;
    const int nt = (n_img + kSimTile - 1) / kSimTile;
    hipLaunchKernelGGL(similarity_kernel, dim3(nt, nt), dim3(kSimThreads), 0, stream, d_desc, n_img, dim, blocksize,
                       nt, d_sim);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

int gtsfm_retrieval_pairs(const float* d_scores, int n_rows, int n_cols, const uint8_t* d_invalid, int num_select,
                          float min_score, int use_min_score, int* d_out_pairs, int* d_row_count, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_rows < 0 || n_cols < 0 || num_select < 0) return GTSFM_ERR_ARG;
    if (n_rows == 0) return GTSFM_OK;
    if (!d_scores || !d_out_pairs || !d_row_count) return GTSFM_ERR_ARG;
    const int k = num_select < n_rows ? num_select : n_rows;  // netvlad_retriever.py:213-215
    if (k > n_cols) return GTSFM_ERR_ARG;                     // torch.topk: k out of range
    hipLaunchKernelGGL(pairs_kernel, dim3(n_rows), dim3(kPairThreads), 0, stream, d_scores, n_rows, n_cols,
                       d_invalid, k, min_score, use_min_score, d_out_pairs, d_row_count);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

}  // extern "C"
