// NetVLAD global image descriptor on gfx950: the network of thirdparty/hloc/netvlad.py:160-191 as driven by
// gtsfm/frontend/global_descriptor/netvlad_global_descriptor.py:27-46, batched over same-sized RGB images.
//
//   u8 RGB -> x / 255 * 255, clamp [0, 255], - averageImage (netvlad.py:174-180)
//   -> VGG16 features[:-2]: 13 conv3x3 (ReLU after all but the last), 2x2 max-pool after conv 2, 4, 7, 10
//   -> per location L2 pre-normalisation over the 512 channels (:187)
//   -> NetVLADLayer (:56-71): soft assignment softmax(W_s x) over 64 clusters, residual sums
//      V[d][k] = sum_n s[n][k] (x[n][d] - c[d][k]), intra-normalisation over d, flatten (d-major), L2
//   -> whitening Linear 32768 -> 4096 + bias, L2 (:189-191).
//
// Kernels ("NetVLAD"):
// - nv_input_conv_kernel: the preprocessing fused into the first 3 -> 64 conv (27 fp32 FMAs per output, VALU);
// - conv3_kernel (conv3.hpp, shared with SuperPoint): the other 12 convolutions as implicit GEMMs on the bf16
//   matrix cores at fp32 accuracy (three-plane split), max-pool fused into the epilogue;
// - nv_prenorm_kernel: one wave per location, the normalised features with a trailing 1 (the assignment mass);
// - gemm_f32_kernel: strided, batched, split-K fp32 MFMA GEMM (v_mfma_f32_32x32x2f32) for the three products
//   (assignment logits, residual sums including the masses, whitening);
// - nv_softmax_kernel, nv_vlad_finalize_kernel, nv_white_finalize_kernel: row-wise epilogues, fixed summation order
//   (the split-K partials are summed in split order), so results do not depend on scheduling.
#include <float.h>

#include "common.hpp"

#pragma clang fp contract(off)

namespace {

#include "conv3.hpp"

struct VggConv {
    int cin, cout, pool;
};
constexpr int kNvConvs = 13;
constexpr VggConv kVgg[kNvConvs] = {
    {3, 64, 0},    {64, 64, 1},   {64, 128, 0},  {128, 128, 1}, {128, 256, 0}, {256, 256, 0}, {256, 256, 1},
    {256, 512, 0}, {512, 512, 0}, {512, 512, 1}, {512, 512, 0}, {512, 512, 0}, {512, 512, 0},
};
constexpr int kDim = 512, kClusters = 64, kWhite = 4096, kVlad = kDim * kClusters;
constexpr int kXaStride = 528;  // floats per location in the pre-normalised block: 512 features, the 1, zero pad
constexpr int kVRows = 576;     // residual-sum rows: 512 features + the mass row, padded to the GEMM tile

// ------------------------------------------------------------------ packed weight blob (include/gtsfm_hip.h)
__host__ __device__ constexpr size_t nv_conv_floats(int l) {
    return (size_t)9 * kVgg[l].cin * kVgg[l].cout + kVgg[l].cout;
}
__host__ __device__ constexpr size_t nv_conv_offset(int l) {
    size_t o = 4;  // preprocessing mean (3 + pad)
    for (int i = 0; i < l; ++i) o += nv_conv_floats(i);
    return o;
}
constexpr size_t kOffScore = nv_conv_offset(kNvConvs);          // [64][512]
constexpr size_t kOffCenters = kOffScore + (size_t)kClusters * kDim;  // [512][64]
constexpr size_t kOffWhiteW = kOffCenters + (size_t)kDim * kClusters;  // [4096][32768]
constexpr size_t kOffWhiteB = kOffWhiteW + (size_t)kWhite * kVlad;    // [4096]
constexpr size_t kBlobFloats = kOffWhiteB + kWhite;

__host__ __device__ constexpr size_t nv_w3_offset(int l) {  // bf16 planes of conv layers 1..12
    size_t o = 0;
    for (int i = 1; i < l; ++i) o += (size_t)3 * 9 * kVgg[i].cin * kVgg[i].cout;
    return o;
}

// ------------------------------------------------------------------ conv 1 with the preprocessing
// v = clamp(fl(fl(u / 255) * 255), 0, 255) - mean[c] exactly as the reference's two tensor ops (describe()'s / 255
// and forward()'s * 255, clamp, - mean, / 1); padding taps are 0 (conv2d pads the preprocessed tensor).
__global__ __launch_bounds__(256) void nv_input_conv_kernel(const uint8_t* __restrict__ imgs, int n, int H, int W,
                                                            const float* __restrict__ blob, float* __restrict__ out) {
    __shared__ float w[27 * 64 + 64];
    const float* wl = blob + nv_conv_offset(0);
    for (int i = threadIdx.x; i < 27 * 64 + 64; i += blockDim.x) w[i] = wl[i];
    __syncthreads();
    const size_t pix = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= (size_t)n * H * W) return;
    const int x = (int)(pix % W);
    const int y = (int)((pix / W) % H);
    const int img = (int)(pix / ((size_t)W * H));
    const uint8_t* im = imgs + (size_t)img * H * W * 3;
    const float mean[3] = {blob[0], blob[1], blob[2]};
    float v[27];  // [tap][channel]
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int yy = y + ky - 1, xx = x + kx - 1;
            const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
            const uint8_t* p = im + ((size_t)(in ? yy : 0) * W + (in ? xx : 0)) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float t = (float)p[c] / 255.0f;
                t = t * 255.0f;
                t = fminf(fmaxf(t, 0.0f), 255.0f);
                v[(ky * 3 + kx) * 3 + c] = in ? t - mean[c] : 0.0f;
            }
        }
    f32x4* o = (f32x4*)(out + pix * 64);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int co = 4 * q + e;
            float acc = 0.0f;
#pragma unroll
            for (int t = 0; t < 27; ++t) acc = __builtin_fmaf(v[t], w[t * 64 + co], acc);
            acc = acc + w[27 * 64 + co];
            r[e] = acc > 0.0f ? acc : 0.0f;
        }
        o[q] = r;
    }
}

// fp32 weights [tap][Cin][Cout] -> bf16 planes [tap][Cin / 16][plane][Cout][16] (conv3.hpp's staging layout)
__global__ void nv_split_weights_kernel(const float* __restrict__ w, int Cin, int Cout, __bf16* __restrict__ out) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (size_t)9 * Cin * Cout) return;
    const int co = (int)(e % Cout), ci = (int)((e / Cout) % Cin), kk = (int)(e / ((size_t)Cout * Cin));
    __bf16 pl[3];
    sp_split3(w[e], pl[0], pl[1], pl[2]);
#pragma unroll
    for (int p = 0; p < 3; ++p)
        out[((((size_t)kk * (Cin / kCinChunk) + ci / kCinChunk) * 3 + p) * Cout + co) * 16 + ci % kCinChunk] = pl[p];
}

// ------------------------------------------------------------------ pre-normalisation (netvlad.py:187)
// F.normalize(x, dim=1) = x / max(||x||_2, 1e-12), one wave per location (8 channels per lane); the output row is
// [x / n (512) | 1 | 0 x 15] so one GEMM forms the residual sums and the assignment masses together.
__global__ __launch_bounds__(256) void nv_prenorm_kernel(const float* __restrict__ F, long long n_loc,
                                                         float* __restrict__ xa) {
    const long long loc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (loc >= n_loc) return;
    const f32x4* src = (const f32x4*)(F + loc * kDim) + 2 * lane;
    const f32x4 a = src[0], b = src[1];
    float ss = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) ss = __builtin_fmaf(a[j], a[j], ss);
#pragma unroll
    for (int j = 0; j < 4; ++j) ss = __builtin_fmaf(b[j], b[j], ss);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    const float nrm = fmaxf(__builtin_sqrtf(ss), 1e-12f);
    f32x4* dst = (f32x4*)(xa + loc * kXaStride) + 2 * lane;
    f32x4 ra, rb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ra[j] = a[j] / nrm;
        rb[j] = b[j] / nrm;
    }
    dst[0] = ra;
    dst[1] = rb;
    if (lane < 4) {
        f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
        if (lane == 0) t[0] = 1.0f;
        *((f32x4*)(xa + loc * kXaStride + kDim) + lane) = t;
    }
}

// ------------------------------------------------------------------ strided batched split-K fp32 GEMM
// C[b][split][m][n] = sum_{k in split} A[b](m, k) B[b](k, n); element (m, k) of A at A + b*sab + m*sam + k*sak, etc.
// 64 x 64 tile per workgroup of four waves (32 x 32 each, v_mfma_f32_32x32x2f32: lane l supplies A(l % 32, k0 + l / 32)
// and B(k0 + l / 32, l % 32)), K staged in chunks of 16 through LDS, the next chunk prefetched in registers. Loads
// are coalesced along whichever of the operand's two strides is 1.
struct GemmArgs {
    const float* A;
    long long sam, sak, sab;
    const float* B;
    long long sbk, sbn, sbb;
    float* C;
    long long scm, scb, scs;  // C row stride (columns contiguous), batch stride, split stride
    int M, N, K, k_split, tiles_n;
};

constexpr int kGemmKC = 16, kGemmLd = 64 + 4;

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
    __shared__ float As[kGemmKC][kGemmLd], Bs[kGemmKC][kGemmLd];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tm = blockIdx.x / g.tiles_n, tn = blockIdx.x % g.tiles_n;
    const int split = blockIdx.y, b = blockIdx.z;
    const int m0 = 64 * tm, n0 = 64 * tn;
    const int k_beg = split * g.k_split, k_end = min(g.K, k_beg + g.k_split);
    const float* A = g.A + b * g.sab;
    const float* B = g.B + b * g.sbb;
    const bool a_kfast = g.sak == 1, b_nfast = g.sbn == 1;
    float ra[4], rb[4];
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            const int mm = a_kfast ? e / kGemmKC : e % 64, kk = a_kfast ? e % kGemmKC : e / 64;
            const int m = m0 + mm, k = k0 + kk;
            ra[u] = (m < g.M && k < k_end) ? A[m * g.sam + k * g.sak] : 0.0f;
            const int nn = b_nfast ? e % 64 : e / kGemmKC, kb = b_nfast ? e / 64 : e % kGemmKC;
            const int nc = n0 + nn, kq = k0 + kb;
            rb[u] = (nc < g.N && kq < k_end) ? B[kq * g.sbk + nc * g.sbn] : 0.0f;
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = tid + 256 * u;
            const int mm = a_kfast ? e / kGemmKC : e % 64, kk = a_kfast ? e % kGemmKC : e / 64;
            As[kk][mm] = ra[u];
            const int nn = b_nfast ? e % 64 : e / kGemmKC, kb = b_nfast ? e / 64 : e % kGemmKC;
            Bs[kb][nn] = rb[u];
        }
    };
    const int wm = wave & 1, wn = wave >> 1, i = lane & 31, kh = lane >> 5;
    f32x16 acc = {};
    if (k_beg < k_end) {
        load(k_beg);
        stash();
        __syncthreads();
        for (int k0 = k_beg; k0 < k_end; k0 += kGemmKC) {
            const bool more = k0 + kGemmKC < k_end;
            if (more) load(k0 + kGemmKC);
#pragma unroll
            for (int s = 0; s < kGemmKC / 2; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[2 * s + kh][32 * wm + i], Bs[2 * s + kh][32 * wn + i], acc,
                                                           0, 0, 0);
            if (!more) break;
            __syncthreads();
            stash();
            __syncthreads();
        }
    }
    float* C = g.C + b * g.scb + split * g.scs;
    const int n = n0 + 32 * wn + i;
    if (n >= g.N) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + 32 * wm + 4 * kh + (r & 3) + 8 * (r >> 2);
        if (m < g.M) C[(long long)m * g.scm + n] = acc[r];
    }
}

hipError_t launch_gemm(GemmArgs g, int batch, int splits, hipStream_t stream) {
    const int tiles_m = (g.M + 63) / 64;
    g.tiles_n = (g.N + 63) / 64;
    g.k_split = (g.K + splits - 1) / splits;
    g.k_split = (g.k_split + kGemmKC - 1) / kGemmKC * kGemmKC;
    if (tiles_m == 0 || g.tiles_n == 0 || batch == 0) return hipSuccess;
    hipLaunchKernelGGL(gemm_f32_kernel, dim3((unsigned)(tiles_m * g.tiles_n), (unsigned)splits, (unsigned)batch),
                       dim3(256), 0, stream, g);
    return hipGetLastError();
}

// ------------------------------------------------------------------ soft assignment (netvlad.py:61-62)
// F.softmax over the 64 clusters of a location's logits, in place: max, exp(l - max), sum, divide.
__global__ __launch_bounds__(256) void nv_softmax_kernel(float* __restrict__ s, long long n_loc) {
    const long long loc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (loc >= n_loc) return;
    float v = s[loc * kClusters + lane];
    float mx = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    const float e = expf(v - mx);
    float sum = e;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    s[loc * kClusters + lane] = e / sum;
}

// ------------------------------------------------------------------ VLAD epilogue (netvlad.py:63-70)
// Per image: V (kVRows x 64, rows 0..511 = sum_n s x, row 512 = sum_n s) summed over the split partials in split order;
// r[d][k] = V[d][k] - c[d][k] S[k]; each cluster column normalised over d (intra-norm), the flattened d-major 32768
// vector normalised again. 256 threads: column k = t % 64, rows d = t / 64 + 4 j; norms by a fixed LDS tree.
__global__ __launch_bounds__(256) void nv_vlad_finalize_kernel(const float* __restrict__ Vp, int splits,
                                                               const float* __restrict__ blob, float* __restrict__ vlad) {
    const int img = blockIdx.x, t = threadIdx.x, k = t & 63, q = t >> 6;
    const float* V = Vp + (size_t)img * splits * kVRows * kClusters;
    const float* cen = blob + kOffCenters;
    __shared__ float red[4][64];
    __shared__ float tot[4];
    float S = 0.0f;
    for (int sp = 0; sp < splits; ++sp) S += V[((size_t)sp * kVRows + kDim) * kClusters + k];
    // r[d][k], recomputed from the partials in each of the three passes (no per-thread array in scratch)
    auto resid = [&](int d) {
        float v = 0.0f;
        for (int sp = 0; sp < splits; ++sp) v += V[((size_t)sp * kVRows + d) * kClusters + k];
        return v - cen[d * kClusters + k] * S;
    };
    float ss = 0.0f;
    for (int j = 0; j < kDim / 4; ++j) {
        const float v = resid(q + 4 * j);
        ss = __builtin_fmaf(v, v, ss);
    }
    red[q][k] = ss;
    __syncthreads();
    const float col = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    const float cn = fmaxf(__builtin_sqrtf(col), 1e-12f);
    float s2 = 0.0f;
    for (int j = 0; j < kDim / 4; ++j) {
        const float v = resid(q + 4 * j) / cn;
        s2 = __builtin_fmaf(v, v, s2);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s2 += __shfl_xor(s2, off);
    if ((t & 63) == 0) tot[q] = s2;
    __syncthreads();
    const float gn = fmaxf(__builtin_sqrtf(((tot[0] + tot[1]) + tot[2]) + tot[3]), 1e-12f);
    float* out = vlad + (size_t)img * kVlad;
    for (int j = 0; j < kDim / 4; ++j) {
        const int d = q + 4 * j;
        out[d * kClusters + k] = (resid(d) / cn) / gn;
    }
}

// whitening epilogue (netvlad.py:189-191): y = sum of split partials (split order) + bias, then L2 normalised
__global__ __launch_bounds__(256) void nv_white_finalize_kernel(const float* __restrict__ Wp, int splits, int n,
                                                                const float* __restrict__ blob, float* __restrict__ desc) {
    const int img = blockIdx.x, t = threadIdx.x;
    const float* bias = blob + kOffWhiteB;
    __shared__ float tot[4];
    float y[kWhite / 256];
    float ss = 0.0f;
#pragma unroll
    for (int j = 0; j < kWhite / 256; ++j) {
        const int o = t + 256 * j;
        float v = 0.0f;
        for (int sp = 0; sp < splits; ++sp) v += Wp[((size_t)sp * n + img) * kWhite + o];
        v = v + bias[o];
        y[j] = v;
        ss = __builtin_fmaf(v, v, ss);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    if ((t & 63) == 0) tot[t >> 6] = ss;
    __syncthreads();
    const float nrm = fmaxf(__builtin_sqrtf(((tot[0] + tot[1]) + tot[2]) + tot[3]), 1e-12f);
#pragma unroll
    for (int j = 0; j < kWhite / 256; ++j) desc[(size_t)img * kWhite + t + 256 * j] = y[j] / nrm;
}

// ------------------------------------------------------------------ workspace
struct NvDims {
    int H[5], W[5];  // after 0..4 pools
};
NvDims nv_dims(int H, int W) {
    NvDims d;
    d.H[0] = H;
    d.W[0] = W;
    for (int i = 1; i < 5; ++i) {
        d.H[i] = d.H[i - 1] / 2;
        d.W[i] = d.W[i - 1] / 2;
    }
    return d;
}

constexpr int kVSplits = 8, kWSplits = 8;

struct NvLayout {
    size_t act0, act1, w3, xa, s, vpart, vlad, wpart, total;
};
NvLayout nv_layout(int n, const NvDims& d) {
    NvLayout L;
    size_t o = 0;
    const size_t px = (size_t)n * d.H[0] * d.W[0];
    const size_t loc = (size_t)n * d.H[4] * d.W[4];
    L.act0 = o; o += gtsfm_align_up(px * 64 * 4, 256);
    L.act1 = o; o += gtsfm_align_up(px * 16 * 4 + 16, 256);
    L.w3 = o; o += gtsfm_align_up(nv_w3_offset(kNvConvs) * sizeof(__bf16), 256);
    L.xa = o; o += gtsfm_align_up(loc * kXaStride * 4, 256);
    L.s = o; o += gtsfm_align_up(loc * kClusters * 4, 256);
    L.vpart = o; o += gtsfm_align_up((size_t)n * kVSplits * kVRows * kClusters * 4, 256);
    L.vlad = o; o += gtsfm_align_up((size_t)n * kVlad * 4, 256);
    L.wpart = o; o += gtsfm_align_up((size_t)kWSplits * n * kWhite * 4, 256);
    L.total = o;
    return L;
}

template <bool POOL>
hipError_t nv_conv(int n, const float* in, int Hi, int Wi, const float* blob, const __bf16* w3, int l, float* out,
                   int relu, hipStream_t stream) {
    ConvArgs a;
    a.in = in; a.Hi = Hi; a.Wi = Wi; a.in_cstride = kVgg[l].cin; a.in_c0 = 0; a.Cin = kVgg[l].cin;
    a.w = blob + nv_conv_offset(l);
    a.cout_pad = kVgg[l].cout;
    a.bias = a.w + (size_t)9 * kVgg[l].cin * kVgg[l].cout;
    a.out = out; a.out_cstride = kVgg[l].cout; a.out_c0 = 0; a.Cout = kVgg[l].cout; a.relu = relu;
    a.tiles_x = (Wi + 31) / 32;
    a.tiles_y = POOL ? (Hi / 2 + conv3_rp(3) - 1) / conv3_rp(3) : (Hi + conv3_rows(3) - 1) / conv3_rows(3);
    if (a.tiles_x == 0 || a.tiles_y == 0) return hipSuccess;
    const dim3 grid((unsigned)(a.tiles_x * a.tiles_y * n), (unsigned)(kVgg[l].cout / 64));
    hipLaunchKernelGGL((conv3_kernel<3, POOL>), grid, dim3(conv3_threads(3)), 0, stream, a, w3 + nv_w3_offset(l));
    return hipGetLastError();
}

}  // namespace

extern "C" {

size_t gtsfm_netvlad_weights_floats(void) { return kBlobFloats; }

size_t gtsfm_netvlad_workspace_bytes(int n, int H, int W) {
    if (n <= 0 || H <= 0 || W <= 0) return 0;
    return nv_layout(n, nv_dims(H, W)).total;
}

int gtsfm_netvlad_batched(const uint8_t* d_images, int n, int H, int W, int C, const float* d_weights, int whiten,
                          float* d_vlad, float* d_desc, void* d_workspace, size_t workspace_bytes, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n == 0) return GTSFM_OK;
    if (!d_images || !d_weights || !d_workspace || n < 0 || H <= 0 || W <= 0 || C != 3 || (whiten && !d_desc) ||
        (!whiten && !d_vlad))
        return GTSFM_ERR_ARG;
    const NvDims d = nv_dims(H, W);
    const NvLayout L = nv_layout(n, d);
    if (workspace_bytes < L.total) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    float* act0 = (float*)(ws + L.act0);
    float* act1 = (float*)(ws + L.act1);
    __bf16* w3 = (__bf16*)(ws + L.w3);
    float* xa = (float*)(ws + L.xa);
    float* s = (float*)(ws + L.s);
    float* vpart = (float*)(ws + L.vpart);
    float* vlad = d_vlad ? d_vlad : (float*)(ws + L.vlad);
    float* wpart = (float*)(ws + L.wpart);
    const float* blob = d_weights;
    for (int l = 1; l < kNvConvs; ++l) {
        const size_t e = (size_t)9 * kVgg[l].cin * kVgg[l].cout;
        hipLaunchKernelGGL(nv_split_weights_kernel, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, stream,
                           blob + nv_conv_offset(l), kVgg[l].cin, kVgg[l].cout, w3 + nv_w3_offset(l));
    }
    GTSFM_CHECK_HIP(hipGetLastError());
    // backbone (netvlad.py:183): ping-pong act0 / act1, pools after conv 2, 4, 7, 10; no ReLU after conv 13
    {
        const size_t pix = (size_t)n * H * W;
        hipLaunchKernelGGL(nv_input_conv_kernel, dim3((unsigned)((pix + 255) / 256)), dim3(256), 0, stream, d_images, n,
                           H, W, blob, act0);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    float* cur = act0;
    float* nxt = act1;
    int lvl = 0;
    for (int l = 1; l < kNvConvs; ++l) {
        const int relu = l + 1 < kNvConvs;
        if (kVgg[l].pool) {
            GTSFM_CHECK_HIP(nv_conv<true>(n, cur, d.H[lvl], d.W[lvl], blob, w3, l, nxt, relu, stream));
            ++lvl;
        } else {
            GTSFM_CHECK_HIP(nv_conv<false>(n, cur, d.H[lvl], d.W[lvl], blob, w3, l, nxt, relu, stream));
        }
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    const long long n_per = (long long)d.H[4] * d.W[4];
    const long long n_loc = (long long)n * n_per;
    if (n_loc > 0) {
        hipLaunchKernelGGL(nv_prenorm_kernel, dim3((unsigned)((n_loc + 3) / 4)), dim3(256), 0, stream,
                           (const float*)cur, n_loc, xa);
        GTSFM_CHECK_HIP(hipGetLastError());
        // logits[loc][k] = sum_d xa[loc][d] W_s[k][d] (score_proj, no bias: netvlad.py:45, 60)
        GemmArgs g{};
        g.A = xa; g.sam = kXaStride; g.sak = 1; g.sab = 0;
        g.B = blob + kOffScore; g.sbk = 1; g.sbn = kDim; g.sbb = 0;
        g.C = s; g.scm = kClusters; g.scb = 0; g.scs = 0;
        g.M = (int)n_loc; g.N = kClusters; g.K = kDim;
        GTSFM_CHECK_HIP(launch_gemm(g, 1, 1, stream));
        hipLaunchKernelGGL(nv_softmax_kernel, dim3((unsigned)((n_loc + 3) / 4)), dim3(256), 0, stream, s, n_loc);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    {
        // V[img][split][d][k] = sum_{loc in split} xa[loc][d] s[loc][k], d = 0..512 (512: the mass sum_n s)
        GemmArgs g{};
        g.A = xa; g.sam = 1; g.sak = kXaStride; g.sab = n_per * kXaStride;
        g.B = s; g.sbk = kClusters; g.sbn = 1; g.sbb = n_per * kClusters;
        g.C = vpart; g.scm = kClusters; g.scb = (long long)kVSplits * kVRows * kClusters;
        g.scs = (long long)kVRows * kClusters;
        g.M = kDim + 1; g.N = kClusters; g.K = (int)n_per;
        if (n_per == 0)
            GTSFM_CHECK_HIP(hipMemsetAsync(vpart, 0, (size_t)n * kVSplits * kVRows * kClusters * 4, stream));
        else
            GTSFM_CHECK_HIP(launch_gemm(g, n, kVSplits, stream));
        hipLaunchKernelGGL(nv_vlad_finalize_kernel, dim3((unsigned)n), dim3(256), 0, stream, (const float*)vpart,
                           kVSplits, blob, vlad);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    if (whiten) {
        // y[img][o] = sum_j vlad[img][j] Wt[o][j] (nn.Linear: x W^T + b)
        GemmArgs g{};
        g.A = vlad; g.sam = kVlad; g.sak = 1; g.sab = 0;
        g.B = blob + kOffWhiteW; g.sbk = 1; g.sbn = kVlad; g.sbb = 0;
        g.C = wpart; g.scm = kWhite; g.scb = 0; g.scs = (long long)n * kWhite;
        g.M = n; g.N = kWhite; g.K = kVlad;
        GTSFM_CHECK_HIP(launch_gemm(g, 1, kWSplits, stream));
        hipLaunchKernelGGL(nv_white_finalize_kernel, dim3((unsigned)n), dim3(256), 0, stream, (const float*)wpart,
                           kWSplits, n, blob, d_desc);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    return GTSFM_OK;
}

}  // extern "C"
