// Verified-correspondence compaction + inlier-support filter: the device side of the hand-off from the batched
// verifier to the host (the step ends with per-pair (R, t, v_corr, inlier count) in host memory).
//
// Reference semantics:
//   v_corr_idxs = match_indices[np.where(mask == 1)]            opencv_verifier_base.py:98-100 (matcher order kept)
//   inlier_ratio = mean(mask)                                   opencv_verifier_base.py:101
//   ISP failure iff ratio < min_ratio or 0 < n_inliers < min_n  inlier_support_processor.py:73-87
// A pair whose verification failed (status != 0) contributes no rows, as the reference's failure tuple carries an
// empty index array (verifier_base.py:56).
//
// Two kernels: an exclusive scan of the per-pair row counts (one workgroup: P is at most a few 10^5, one pass of
// ~P/1024 sequential elements per thread), then one wave per pair that streams its mask 64 putatives at a time and
// writes the surviving (i1, i2) rows with a ballot / mbcnt rank, so the output keeps matcher order.
#include "common.hpp"

namespace {

constexpr int kScanThreads = 1024;

__device__ __forceinline__ int pair_rows(const int* status, const int* n_inl, int p) {
    return status[p] == 0 ? n_inl[p] : 0;
}

__global__ __launch_bounds__(kScanThreads) void scan_rows_kernel(const int* __restrict__ status,
                                                                 const int* __restrict__ n_inl, int n_pairs,
                                                                 int* __restrict__ offsets) {
    __shared__ long long part[kScanThreads];
    const int tid = threadIdx.x;
    const int per = (n_pairs + kScanThreads - 1) / kScanThreads;
    const int a = min(tid * per, n_pairs), b = min(a + per, n_pairs);
    long long s = 0;
    for (int p = a; p < b; ++p) s += pair_rows(status, n_inl, p);
    part[tid] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan over the 1024 partial sums
    for (int d = 1; d < kScanThreads; d <<= 1) {
        const long long v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    long long run = part[tid] - s;  // exclusive prefix of this thread's block
    for (int p = a; p < b; ++p) {
        offsets[p] = (int)run;
        run += pair_rows(status, n_inl, p);
    }
    if (tid == kScanThreads - 1) offsets[n_pairs] = (int)part[kScanThreads - 1];
}

__global__ __launch_bounds__(256) void compact_rows_kernel(const uint2* __restrict__ match_idx,
                                                           const int* __restrict__ match_count, int mcap,
                                                           const uint8_t* __restrict__ mask,
                                                           const int* __restrict__ status,
                                                           const int* __restrict__ n_inl,
                                                           const int* __restrict__ ratio_inl, int n_pairs,
                                                           int min_inliers, double min_ratio,
                                                           const int* __restrict__ offsets, int capacity,
                                                           uint2* __restrict__ v_corr, uint8_t* __restrict__ isp_ok) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (p >= n_pairs) return;
    const int st = status[p], n = n_inl[p], M = match_count[p];
    if (lane == 0) {
        const int nr = ratio_inl ? ratio_inl[p] : n;
        const double ratio = (st == 0 && M > 0) ? (double)nr / (double)M : 0.0;
        const bool fail = ratio < min_ratio || (n > 0 && n < min_inliers);
        isp_ok[p] = (st == 0 && !fail) ? 1 : 0;
    }
    if (st != 0) return;
    const int base = offsets[p];
    if (base + n > capacity) return;  // the host sized `capacity` from the same counts; never true in practice
    const uint2* src = match_idx + (size_t)p * mcap;
    const uint8_t* mk = mask + (size_t)p * mcap;
    int written = 0;
    for (int j0 = 0; j0 < M && written < n; j0 += 64) {
        const int j = j0 + lane;
        const bool keep = j < M && mk[j] != 0;
        const unsigned long long bal = __ballot(keep);
        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
        if (keep && written + r < n) v_corr[base + written + r] = src[j];
        written += __popcll(bal);
    }
}

}  // namespace

extern "C" {

int gtsfm_compact_verified(const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                           const uint8_t* d_inlier_mask, const int* d_status, const int* d_n_inliers,
                           const int* d_ratio_inliers, int n_pairs, int min_inliers, double min_inlier_ratio,
                           int* d_offsets, uint32_t* d_v_corr, int capacity, uint8_t* d_isp_ok, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs < 0 || mcap < 0 || capacity < 0) return GTSFM_ERR_ARG;
    if (!d_offsets) return GTSFM_ERR_ARG;
    if (n_pairs == 0) {
        GTSFM_CHECK_HIP(hipMemsetAsync(d_offsets, 0, sizeof(int), stream));
        return GTSFM_OK;
    }
    if (!d_match_idx || !d_match_count || !d_inlier_mask || !d_status || !d_n_inliers || !d_isp_ok ||
        (capacity > 0 && !d_v_corr))
        return GTSFM_ERR_ARG;
    hipLaunchKernelGGL(scan_rows_kernel, dim3(1), dim3(kScanThreads), 0, stream, d_status, d_n_inliers, n_pairs,
                       d_offsets);
    GTSFM_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(compact_rows_kernel, dim3((n_pairs + 3) / 4), dim3(256), 0, stream, (const uint2*)d_match_idx,
                       d_match_count, mcap, d_inlier_mask, d_status, d_n_inliers, d_ratio_inliers, n_pairs, min_inliers,
                       min_inlier_ratio, d_offsets, capacity, (uint2*)d_v_corr, d_isp_ok);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
