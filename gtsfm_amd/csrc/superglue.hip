// SuperGlue matcher on gfx950: thirdparty/SuperGluePretrainedNetwork/models/superglue.py:228-283 as driven by
// gtsfm/frontend/matcher/superglue_matcher.py:43-111 (20 Sinkhorn iterations, match threshold 0.2), batched over
// image pairs.
//
//   keypoint normalisation + MLP encoder (with eval BatchNorm) -> 18 x {self, cross} attentional propagation
//   (4-head attention d = 256, MLP 512 -> 512 -> 256, residual) -> final projection -> scores / 16
//   -> log-space optimal transport with a dustbin -> mutual argmax + threshold.
//
// Layout: every (pair, side) owns a kmax x C row-major (point-major) feature block, so each 1x1 Conv1d is a
// batched GEMM  Y[n][co] = sum_ci X[n][ci] W^T[ci][co]  on the bf16 matrix cores at near-fp32 accuracy (three-plane
// split, six products: sg_gemm3_kernel). Differences from the fp32 torch reference come from: summation order; the
// three dropped plane products (each below 2^-23 |a b|); exp taken as v_exp_f32 of x log2(e) in the attention and
// Sinkhorn kernels (the product's rounding gives a relative error of about |x| 2^-24). tests/test_superglue_gpu.py
// bounds the result: log-assignment within 2e-3 of the reference module, matches equal up to near-ties. Heads
// are stored head-major (channel h * 64 + d; the reference's view(b, 64, 4, n) interleaves them as 4 d + h — the
// host packs the q/k/v/merge weights accordingly). Attention is one fused kernel (online softmax on the same split
// products): the K1 x K2 probability matrix never reaches HBM. The Sinkhorn matrix (K1 + 1) x (K2 + 1) does, once
// per pair.
#include <float.h>

#include <type_traits>

#include "common.hpp"

#pragma clang fp contract(off)

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kD = 256;     // descriptor_dim
constexpr int kHeads = 4;
constexpr int kHd = 64;     // per-head dim

// ------------------------------------------------------------------ packed weights (include/gtsfm_hip.h)
// GEMM weights are W^T[cin][cout] row-major. Encoder layers: W^T (cin_pad x cout), bias, bn_scale, bn_shift
// (the last encoder layer has no BN). GNN layer: Wqkv^T (256 x 768, columns [q | k | v], head-major), bqkv,
// Wm^T (256 x 256, rows head-major), bm, W1^T (512 x 512: rows 0..255 act on x, 256..511 on the message), b1,
// bn1 scale, bn1 shift, W2^T (512 x 256), b2. Then final_proj W^T (256 x 256), bias, and bin_score (1 float).
constexpr int kEncIn[5] = {16, 32, 64, 128, 256};  // cin (the 3 encoder inputs zero-padded to 16)
constexpr int kEncOut[5] = {32, 64, 128, 256, 256};

__host__ __device__ constexpr size_t enc_floats(int i) {
    return (size_t)kEncIn[i] * kEncOut[i] + kEncOut[i] + (i < 4 ? 2 * kEncOut[i] : 0);
}
__host__ __device__ constexpr size_t enc_total() {
    size_t o = 0;
    for (int i = 0; i < 5; ++i) o += enc_floats(i);
    return o;
}
constexpr size_t kLayerFloats = (size_t)256 * 768 + 768 + 256 * 256 + 256 + 512 * 512 + 512 * 3 + 512 * 256 + 256;
__host__ __device__ constexpr size_t sg_weights_floats(int n_layers) {
    return enc_total() + (size_t)n_layers * kLayerFloats + 256 * 256 + 256 + 1;
}

// ------------------------------------------------------------------ batched GEMM on fp32 MFMA
constexpr int kGemmThreads = 256;
constexpr int kKc = 16;  // K chunk staged in LDS (a multiple of 16; chunks past K are zero-filled)
static_assert(kKc % 16 == 0, "K chunk");

struct GemmArgs {
    const float* A;   // A[z][m][k] (k < Ksplit), row stride lda, batch stride a_batch
    long lda, a_batch;
    const float* A2;  // A2[z][m][k - Ksplit] (k >= Ksplit)
    long lda2, a2_batch;
    int Ksplit;
    const float* B;   // b_trans = 0: B[z][k][n] (ldb); 1: B[z][n][k]
    long ldb, b_batch;
    int b_trans;
    const float* bias, *bn_scale, *bn_shift;  // per output column, may be null
    int relu;
    float alpha;      // applied last (before the residual add)
    float* C;         // C[z][m][n], row stride ldc
    long ldc, c_batch;
    int residual;     // C += result
    int M, N, K;
    const int* m_lim; // per-batch valid rows / columns (may be null)
    const int* n_lim;
    int lim_stride;   // index of batch z into m_lim / n_lim: z * lim_stride (+1 for n_lim)
};

// 64 x 64 output tile per workgroup; wave w computes rows 32 (w & 1) .., columns 32 (w >> 1) ..
__global__ __launch_bounds__(kGemmThreads) void sg_gemm_kernel(GemmArgs g) {
    __shared__ float As[64 * (kKc + 1)];
    __shared__ float Bs[kKc * 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int z = blockIdx.z;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    int Mv = g.M, Nv = g.N;
    if (g.m_lim) Mv = min(Mv, g.m_lim[z * g.lim_stride]);
    if (g.n_lim) Nv = min(Nv, g.n_lim[z * g.lim_stride + 1]);
    if (m0 >= Mv || n0 >= Nv) return;
    const float* A = g.A + z * g.a_batch;
    const float* A2 = g.A2 ? g.A2 + z * g.a2_batch : nullptr;
    const float* B = g.B + z * g.b_batch;
    const int wm = wave & 1, wn = wave >> 1;
    const int r = lane & 31, kh = lane >> 5;
    f32x16 acc = {};
    for (int k0 = 0; k0 < g.K; k0 += kKc) {
        // A tile: 64 rows x kKc k (float4 per thread and step)
#pragma unroll
        for (int it = 0; it < kKc / 16; ++it) {
            const int idx = tid + kGemmThreads * it;
            const int row = idx / (kKc / 4), q = idx % (kKc / 4);
            const int gm = m0 + row, gk = k0 + 4 * q;
            f32x4_t v = {0.0f, 0.0f, 0.0f, 0.0f};
            if (gm < g.M && gk < g.K) {
                if (gk < g.Ksplit) v = *(const f32x4_t*)(A + (long)gm * g.lda + gk);
                else v = *(const f32x4_t*)(A2 + (long)gm * g.lda2 + (gk - g.Ksplit));
            }
            float* d = As + row * (kKc + 1) + 4 * q;
            d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
        }
        // B tile: kKc k x 64 n
#pragma unroll
        for (int it = 0; it < kKc / 16; ++it) {
            const int idx = tid + kGemmThreads * it;
            if (!g.b_trans) {
                const int kk = idx >> 4, q = idx & 15;
                const int gn = n0 + 4 * q;
                f32x4_t v = {0.0f, 0.0f, 0.0f, 0.0f};
                if (gn < g.N && k0 + kk < g.K) v = *(const f32x4_t*)(B + (long)(k0 + kk) * g.ldb + gn);
                *(f32x4_t*)(Bs + kk * 64 + 4 * q) = v;
            } else {
                const int nn = idx / (kKc / 4), q = idx % (kKc / 4);
                const int gn = n0 + nn;
                f32x4_t v = {0.0f, 0.0f, 0.0f, 0.0f};
                if (gn < g.N && k0 + 4 * q < g.K) v = *(const f32x4_t*)(B + (long)gn * g.ldb + k0 + 4 * q);
                Bs[(4 * q + 0) * 64 + nn] = v[0];
                Bs[(4 * q + 1) * 64 + nn] = v[1];
                Bs[(4 * q + 2) * 64 + nn] = v[2];
                Bs[(4 * q + 3) * 64 + nn] = v[3];
            }
        }
        __syncthreads();
        const float* pa = As + (32 * wm + r) * (kKc + 1) + 8 * kh;
        const float* pb = Bs + (8 * kh) * 64 + 32 * wn + r;
#pragma unroll
        for (int g16 = 0; g16 < kKc / 16; ++g16)
#pragma unroll
            for (int s = 0; s < 8; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[16 * g16 + s], pb[(16 * g16 + s) * 64], acc, 0, 0, 0);
        __syncthreads();
    }
    const int n = n0 + 32 * wn + r;
    if (n >= Nv) return;
    const float b = g.bias ? g.bias[n] : 0.0f;
    const float sc = g.bn_scale ? g.bn_scale[n] : 1.0f;
    const float sh = g.bn_shift ? g.bn_shift[n] : 0.0f;
    float* C = g.C + z * g.c_batch + n;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int m = m0 + 32 * wm + 4 * kh + (e & 3) + 8 * (e >> 2);
        if (m >= Mv) continue;
        float v = acc[e] + b;
        if (g.bn_scale) v = v * sc + sh;
        if (g.relu) v = v > 0.0f ? v : 0.0f;
        if (g.alpha != 1.0f) v = v * g.alpha;
        float* c = C + (long)m * g.ldc;
        *c = g.residual ? *c + v : v;
    }
}

// XCD-aware workgroup order: the dispatcher deals workgroup L to XCD L % 8, so workgroup L takes logical tile
// (L % 8) * (T / 8) + L / 8 and every XCD runs a contiguous range of logical tiles, whose shared operands (one
// (side, head)'s key / value planes; one row block of A) then stay in that XCD's L2. Identity when 8 does not divide T.
__device__ __forceinline__ void xcd_tile(int& x, int& y, int& z) {
    const int nx = gridDim.x, ny = gridDim.y;
    const long T = (long)nx * ny * gridDim.z;
    const long L = blockIdx.x + (long)nx * (blockIdx.y + (long)ny * blockIdx.z);
    const long t = T % 8 == 0 ? (L % 8) * (T / 8) + L / 8 : L;
    x = (int)(t % nx);
    y = (int)((t / nx) % ny);
    z = (int)(t / ((long)nx * ny));
}

// ------------------------------------------------------------------ batched GEMM, fp32-accurate on bf16 MFMA
// Every fp32 operand x is split exactly into three bf16 planes, x = x_h + x_m + x_l (each plane the bf16 rounding of
// what the planes above it leave; the two subtractions are exact), and a product a b is formed from the six largest
// of its nine plane products: a_h b_h + a_h b_m + a_m b_h + a_m b_m + a_h b_l + a_l b_h. bf16 x bf16 products are
// exact in the fp32 accumulator, and the dropped terms (a_m b_l, a_l b_m, a_l b_l) are below 2^-23 |a b| together,
// so each product carries an fp32-level error; the sums are fp32 as on the fp32 matrix cores. Six
// v_mfma_f32_32x32x16_bf16 (16 k each) replace eight v_mfma_f32_32x32x2_f32 (2 k each): 2.7x the product rate.
// Weights are split once per layer into [plane][n][k] (sg_split_weights_kernel); activations are split as they are
// staged into LDS. TM x 128 output tile per workgroup of four waves (TM / 2 x 64 each, 32 x 32 accumulators),
// K in chunks of 16 held in LDS as [plane][row][16] bf16 (32-byte rows: a lane's 16-byte fragment read is
// conflict-free), the next chunk in flight in registers during the MFMAs.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kG3Tile = 128;

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

// eight consecutive fp32 -> three 16-byte planes
__device__ __forceinline__ void split3x8(const f32x4_t& a, const f32x4_t& b, bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 hh, mm, ll;
        split3(j < 4 ? a[j & 3] : b[j & 3], hh, mm, ll);
        h[j] = hh;
        m[j] = mm;
        l[j] = ll;
    }
}

struct Gemm3Args {
    const float* A;  // A[z][m][k] (k < Ksplit), A2[z][m][k - Ksplit] (k >= Ksplit); K a multiple of 16
    long lda, a_batch;
    const float* A2;
    long lda2, a2_batch;
    int Ksplit;
    const __bf16* Bp;  // weights: [3][N][K] bf16 planes (batch-invariant), or null
    const float* Bt;   // activations: Bt[z][n][k] fp32 (ldb, b_batch), split while staging
    long ldb, b_batch;
    const float *bias, *bn_scale, *bn_shift;
    int relu;
    float alpha;
    float* C;
    long ldc, c_batch;
    int residual;
    int M, N, K;
    const int* m_lim;
    const int* n_lim;
    int lim_stride;
    // q/k/v projection only: columns 256..511 (keys) and 512..767 (values) go to bf16 planes for the attention
    // kernel instead of C: K planes [z][3][head][m][64], then V^T planes [z][3][head][64][M] (kv_batch per z)
    __bf16* kv;
    long kv_batch;
};

// Two LDS staging buffers since round 6 (one barrier per chunk; a chunk's split and stores overlap the MFMAs of the
// chunk before): C5 slice match stage 826 -> 806 ms per step, TM = 128 launches 3.5 -> 3.27 ms (profiles/r06n_*).
// KC: K per LDS chunk (16 or 32; rows padded to 40 elements at 32 so the fragment reads stay conflict-free);
// SLOTS: chunks kept in flight in registers (round 5, single LDS buffer). Measured on the C5 slice (qkv / W1 / Wm+W2 launches of 992 sides):
// <16, 1> 7.05 / 7.57 / 3.45 ms (162 VGPRs, three waves per SIMD), <16, 2> 7.87 / 8.38 / 4.17, <32, 1> 7.40 / 7.76 /
// 4.04, <32, 2> 10.19 / 10.94 / 5.38: the kernel is bound by LDS fragment traffic (12 16-byte reads per 24 MFMAs per
// wave), so occupancy beats prefetch depth; <16, 1> is the one launched.
// TM: output rows per workgroup (128 or 256; waves 2 x 2, each TM / 2 x 64). Measured on the C5 slice (992 sides):
// TM = 256 runs the N = 768 / 512 launches (q/k/v, W1) at 7.21 / 7.02 ms against 7.53 / 7.42 for 128, the N = 256 ones
// (Wm, W2) at 3.69 against 3.53, so run_gemm3 takes 256 for N >= 512.
constexpr int kG3Kc = 16, kG3Slots = 1;
constexpr int kG3EpiRow = 72;  // epilogue tile row stride (floats): 4 rows apart = 32 banks apart
// dynamic LDS bytes of sg_gemm3_kernel<16, 1, TM>: two staging buffers, or the epilogue's four 32 x 72 fp32 tiles
constexpr int sg_gemm3_lds(int tm) {
    return (2 * 3 * (tm + kG3Tile) * 16 * 2) > 4 * 32 * kG3EpiRow * 4 ? 2 * 3 * (tm + kG3Tile) * 16 * 2
                                                                      : 4 * 32 * kG3EpiRow * 4;
}
// Epilogue of the split GEMMs through LDS, one 32-row accumulator tile at a time: the wave parks tile i (32 x 64 fp32,
// rows padded to 72 floats: conflict-free both ways) in the (free) staging LDS and walks it with lane = column, so no
// unrolled per-register epilogue sits beside the live accumulators. The caller has retired every staging access.
template <int TM>
__device__ __forceinline__ void g3_epilogue(const Gemm3Args& g, f32x16 (&acc)[TM / 64][2], float* smemf, int wave,
                                            int lane, int m0, int n0, int Mv, int Nv, int z) {
    constexpr int WI = TM / 64;
    const int wm = wave & 1, wn = wave >> 1;
    const int r = lane & 31, hk = lane >> 5;
    float* T = smemf + wave * 32 * kG3EpiRow;
    const int col = lane, n = n0 + 64 * wn + col;
    const bool n_ok = n < Nv;
    const float bb = n_ok && g.bias ? g.bias[n] : 0.0f;
    const float sc = n_ok && g.bn_scale ? g.bn_scale[n] : 1.0f;
    const float sh = n_ok && g.bn_shift ? g.bn_shift[n] : 0.0f;
    // values (q/k/v projection, n >= 512) go to the transposed planes [..][dim][key] (four consecutive keys per
    // 8-byte store); keys (256 <= n < 512) to [..][key][dim] (lanes along the dimension)
    const bool vt = g.kv && n >= 2 * kD, kt = g.kv && n >= kD && n < 2 * kD;
    auto post = [&](float v) {
        v = v + bb;
        if (g.bn_scale) v = v * sc + sh;
        if (g.relu) v = v > 0.0f ? v : 0.0f;
        if (g.alpha != 1.0f) v = v * g.alpha;
        return v;
    };
#pragma unroll
    for (int i = 0; i < WI; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 16; ++k) T[(8 * (k >> 2) + 4 * hk + (k & 3)) * kG3EpiRow + 32 * j + r] = acc[i][j][k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the tile's first row. M is a multiple of 64; Mv is M unless m_lim is set (the score GEMM), which kv mode
        // never sets (run_gemm3 rejects it): the V^T path's four-key stores below assume Mv == M
        const int mt = m0 + (TM / 2) * wm + 32 * i;
        if (n_ok && mt < Mv) {
            if (vt) {
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                const int d = n - 2 * kD, hh = d / kHd, dd = d % kHd;
                __bf16* base = g.kv + z * g.kv_batch + (long)3 * kD * g.M;
#pragma unroll 2
                for (int rg = 0; rg < 8; ++rg) {
                    const int mg = mt + 4 * rg;
                    if (mg >= Mv) break;
                    bf16x4 pl[3];
#pragma unroll
                    for (int e4 = 0; e4 < 4; ++e4) {
                        __bf16 h0, h1, h2;
                        split3(post(T[(4 * rg + e4) * kG3EpiRow + col]), h0, h1, h2);
                        pl[0][e4] = h0;
                        pl[1][e4] = h1;
                        pl[2][e4] = h2;
                    }
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        *(bf16x4*)(base + (((long)q * kHeads + hh) * kHd + dd) * g.M + mg) = pl[q];
                }
            } else if (kt) {
                const int d = n - kD, hh = d / kHd, dd = d % kHd;
                __bf16* base = g.kv + z * g.kv_batch;
#pragma unroll 4
                for (int row = 0; row < 32; ++row) {
                    const int m = mt + row;
                    if (m >= Mv) break;
                    __bf16 pl[3];
                    split3(post(T[row * kG3EpiRow + col]), pl[0], pl[1], pl[2]);
#pragma unroll
                    for (int q = 0; q < 3; ++q) base[(((long)q * kHeads + hh) * g.M + m) * kHd + dd] = pl[q];
                }
            } else {
                float* C = g.C + z * g.c_batch + n;
#pragma unroll 4
                for (int row = 0; row < 32; ++row) {
                    const int m = mt + row;
                    if (m >= Mv) break;
                    const float v = post(T[row * kG3EpiRow + col]);
                    float* c = C + (long)m * g.ldc;
                    *c = g.residual ? *c + v : v;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the tile is read before the next one overwrites it
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int KC, int SLOTS, int TM>
__global__ __launch_bounds__(256, 2) void sg_gemm3_kernel(Gemm3Args g) {
    constexpr int kRow = KC == 16 ? 16 : 40;
    constexpr int kU = KC / 16;   // 8-float A units / 16-byte B units per thread, plane and chunk
    constexpr int RA = TM / 128;  // A rows staged per thread
    constexpr int WI = TM / 64;   // 32-row accumulator tiles per wave (2 x 2 waves over TM x 128)
    // staging planes As [3][TM][kRow] | Bs [3][128][kRow], reused by the epilogue's per-wave 32 x 72 fp32 tiles
    // two staging buffers (chunk c in buffer c & 1): one barrier per chunk, and a chunk's split and LDS stores run
    // while the MFMAs of the chunk before it drain
    constexpr int kStage = 3 * (TM + kG3Tile) * kRow;
    extern __shared__ __attribute__((aligned(16))) __bf16 smem[];
    auto As_of = [&](int b) { return reinterpret_cast<__bf16(*)[TM][kRow]>(smem + b * kStage); };
    auto Bs_of = [&](int b) { return reinterpret_cast<__bf16(*)[kG3Tile][kRow]>(smem + b * kStage + 3 * TM * kRow); };
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bx, by, z;
    xcd_tile(bx, by, z);
    const int m0 = by * TM, n0 = bx * kG3Tile;
    int Mv = g.M, Nv = g.N;
    if (g.m_lim) Mv = min(Mv, g.m_lim[z * g.lim_stride]);
    if (g.n_lim) Nv = min(Nv, g.n_lim[z * g.lim_stride + 1]);
    if (m0 >= Mv || n0 >= Nv) return;
    const int wm = wave & 1, wn = wave >> 1;
    const int r = lane & 31, hk = lane >> 5;
    // staging roles: thread t stages A rows (t >> 1) + 128 ra and B column t >> 1, k offset (KC / 2) (t & 1)
    const int srow = tid >> 1, sk = (KC / 2) * (tid & 1);
    const bool b_ok = n0 + srow < g.N;
    bool a_ok[RA];
    const float *Arow[RA], *A2row[RA];
#pragma unroll
    for (int ra = 0; ra < RA; ++ra) {
        a_ok[ra] = m0 + srow + 128 * ra < g.M;
        Arow[ra] = g.A + z * g.a_batch + (long)(m0 + srow + 128 * ra) * g.lda + sk;
        A2row[ra] = g.A2 ? g.A2 + z * g.a2_batch + (long)(m0 + srow + 128 * ra) * g.lda2 + sk - g.Ksplit : nullptr;
    }
    f32x4_t pa[SLOTS][RA][2 * kU], pb[SLOTS][2 * kU];
    u32x4 pw[SLOTS][3][kU];
    auto load = [&](int k0, auto slot) {
        constexpr int q = decltype(slot)::value;
#pragma unroll
        for (int ra = 0; ra < RA; ++ra) {
#pragma unroll
            for (int u = 0; u < 2 * kU; ++u) pa[q][ra][u] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
            if (a_ok[ra]) {
                const float* src = k0 < g.Ksplit ? Arow[ra] + k0 : A2row[ra] + k0;
#pragma unroll
                for (int u = 0; u < 2 * kU; ++u) pa[q][ra][u] = *(const f32x4_t*)(src + 4 * u);
            }
        }
        if (g.Bp) {
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int u = 0; u < kU; ++u)
                    pw[q][p][u] = b_ok ? *(const u32x4*)(g.Bp + ((long)p * g.N + n0 + srow) * g.K + k0 + sk + 8 * u)
                                       : u32x4{0, 0, 0, 0};
        } else {
#pragma unroll
            for (int u = 0; u < 2 * kU; ++u) pb[q][u] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
            if (b_ok) {
                const float* src = g.Bt + z * g.b_batch + (long)(n0 + srow) * g.ldb + k0 + sk;
#pragma unroll
                for (int u = 0; u < 2 * kU; ++u) pb[q][u] = *(const f32x4_t*)(src + 4 * u);
            }
        }
    };
    auto store = [&](auto slot, int buf) {
        constexpr int q = decltype(slot)::value;
        __bf16(*As)[TM][kRow] = As_of(buf);
        __bf16(*Bs)[kG3Tile][kRow] = Bs_of(buf);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            bf16x8 h, m, l;
#pragma unroll
            for (int ra = 0; ra < RA; ++ra) {
                split3x8(pa[q][ra][2 * u], pa[q][ra][2 * u + 1], h, m, l);
                *(bf16x8*)&As[0][srow + 128 * ra][sk + 8 * u] = h;
                *(bf16x8*)&As[1][srow + 128 * ra][sk + 8 * u] = m;
                *(bf16x8*)&As[2][srow + 128 * ra][sk + 8 * u] = l;
            }
            if (g.Bp) {
#pragma unroll
                for (int p = 0; p < 3; ++p) *(u32x4*)&Bs[p][srow][sk + 8 * u] = pw[q][p][u];
            } else {
                split3x8(pb[q][2 * u], pb[q][2 * u + 1], h, m, l);
                *(bf16x8*)&Bs[0][srow][sk + 8 * u] = h;
                *(bf16x8*)&Bs[1][srow][sk + 8 * u] = m;
                *(bf16x8*)&Bs[2][srow][sk + 8 * u] = l;
            }
        }
    };
    f32x16 acc[WI][2];
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    auto compute = [&](int buf) {
        __bf16(*As)[TM][kRow] = As_of(buf);
        __bf16(*Bs)[kG3Tile][kRow] = Bs_of(buf);
#pragma unroll
        for (int ks = 0; ks < kU; ++ks) {
            // B fragments for the chunk, then A one row tile at a time (fewer fragments live beside the accumulators)
            bf16x8 b[3][2];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int s = 0; s < 2; ++s) b[p][s] = *(const bf16x8*)&Bs[p][64 * wn + 32 * s + r][16 * ks + 8 * hk];
#pragma unroll
            for (int i = 0; i < WI; ++i) {
                bf16x8 a[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) a[p] = *(const bf16x8*)&As[p][(TM / 2) * wm + 32 * i + r][16 * ks + 8 * hk];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x16 c = acc[i][j];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2][j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0][j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1][j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1][j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0][j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0][j], c, 0, 0, 0);
                    acc[i][j] = c;
                }
            }
        }
    };
    using S0 = std::integral_constant<int, 0>;
    static_assert(SLOTS == 1, "one chunk in flight in registers, two in LDS");
    load(0, S0{});
    store(S0{}, 0);
    if (KC < g.K) load(KC, S0{});
    __syncthreads();
    for (int k0 = 0, buf = 0; k0 < g.K; k0 += KC, buf ^= 1) {
        compute(buf);
        if (k0 + KC < g.K) {
            store(S0{}, buf ^ 1);  // chunk k0 + KC (buffer buf ^ 1 was last read by chunk k0 - KC's MFMAs)
            if (k0 + 2 * KC < g.K) load(k0 + 2 * KC, S0{});
        }
        __syncthreads();  // chunk k0 + KC staged; everyone done reading buffer buf
    }
    g3_epilogue<TM>(g, acc, (float*)smem, wave, lane, m0, n0, Mv, Nv, z);  // (the loop's last barrier: stages free)
}

// The same products with the operands staged by LDS-DMA (round 6), for the weight GEMMs (B = pre-split planes, A
// fp32 rows): per 16-deep K chunk every wave issues five global_load_lds_dwordx4 pieces of 1 KiB (A: 128 rows x 64 B in
// eight pieces of 16 rows; B: three planes x 128 columns x 32 B in twelve pieces of 32 columns), S chunks in flight in
// an S-buffer LDS ring, waits counted (every chunk issues its five pieces, past the last chunk the last one again into
// the free buffer) and a raw s_barrier per chunk (__syncthreads would drain the ring). A stays fp32 in LDS and is split
// into its three planes on the fragment read -- the split3x8 of the staged form, on the same eight consecutive values,
// so the planes, the MFMA sequence and every output are bit-identical to sg_gemm3_kernel. The LDS image is
// lane-linear per piece (the DMA's destination is base + 16 lane), so the conflict-free layouts come from the source
// addresses: A row r's 16-byte unit q sits at slot q ^ ((r >> 2) & 3) of its 64-byte row, B column c's half h at slot
// h ^ ((c >> 3) & 1) of its 32 bytes (ds_read_b128 serves lanes {0-3, 12-15, 20-27}, ... together: 16 distinct
// 4-bank groups either way).
__host__ __device__ constexpr int sg_gemm3d_pieces(int tm) { return tm / 64 + 3; }  // per wave per chunk (A, B)
__host__ __device__ constexpr int sg_gemm3d_lds(int tm, int stages) {
    return stages * (tm * 16 * 4 + 3 * kG3Tile * 16 * 2) > 4 * 32 * kG3EpiRow * 4
               ? stages * (tm * 16 * 4 + 3 * kG3Tile * 16 * 2)
               : 4 * 32 * kG3EpiRow * 4;
}

template <int TM, int S>
__global__ __launch_bounds__(256, 2) void sg_gemm3d_kernel(Gemm3Args g) {
    constexpr int WI = TM / 64, RA = TM / 64;  // accumulator row tiles per wave; A pieces per wave
    constexpr int kA = TM * 16 * 4, kB = 3 * kG3Tile * 16 * 2, kStage = kA + kB;  // bytes
    extern __shared__ __attribute__((aligned(16))) unsigned char smem8[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bx, by, z;
    xcd_tile(bx, by, z);
    const int m0 = by * TM, n0 = bx * kG3Tile;
    int Mv = g.M, Nv = g.N;
    if (g.m_lim) Mv = min(Mv, g.m_lim[z * g.lim_stride]);
    if (g.n_lim) Nv = min(Nv, g.n_lim[z * g.lim_stride + 1]);
    if (m0 >= Mv || n0 >= Nv) return;
    const int wm = wave & 1, wn = wave >> 1;
    const int r = lane & 31, hk = lane >> 5;
    const int nk = g.K / 16;
    // this lane's source in each of the wave's pieces: (row, unit) of A, (plane, column, half) of B, clamped into the
    // matrix (rows / columns past it are staged but never stored)
    int a_row[RA], a_q[RA], b_pl[3], b_col[3], b_h[3];
#pragma unroll
    for (int t = 0; t < RA; ++t) {
        const int row = 16 * (RA * wave + t) + (lane >> 2);
        a_row[t] = min(m0 + row, g.M - 1);
        a_q[t] = (lane & 3) ^ ((row >> 2) & 3);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int pc = 3 * wave + t;  // piece 0..11: plane pc / 4, columns 32 (pc % 4) ..
        const int col = 32 * (pc % 4) + (lane >> 1);
        b_pl[t] = pc / 4;
        b_col[t] = min(n0 + col, g.N - 1);
        b_h[t] = (lane & 1) ^ ((col >> 3) & 1);
    }
    const float* Az = g.A + z * g.a_batch;
    const float* A2z = g.A2 ? g.A2 + z * g.a2_batch : nullptr;
    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)smem8;
    auto issue = [&](int c, int buf) {
        const int k0 = 16 * c;
        const bool second = k0 >= g.Ksplit;
        const float* abase = second ? A2z : Az;
        const long alda = second ? g.lda2 : g.lda;
        const int ak = second ? k0 - g.Ksplit : k0;
        const uint32_t stage = lds_base + (uint32_t)(buf * kStage);
#pragma unroll
        for (int t = 0; t < RA; ++t) {
            const uint32_t off = (uint32_t)(((long)a_row[t] * alda + ak + 4 * a_q[t]) * 4);
            const uint32_t la = __builtin_amdgcn_readfirstlane(stage + 1024u * (RA * wave + t));
            asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(abase), "{m0}"(la) : "memory");
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const uint32_t off = (uint32_t)((((long)b_pl[t] * g.N + b_col[t]) * g.K + k0 + 8 * b_h[t]) * 2);
            const uint32_t la = __builtin_amdgcn_readfirstlane(stage + kA + 1024u * (3 * wave + t));
            asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(g.Bp), "{m0}"(la) : "memory");
        }
    };
    f32x16 acc[WI][2];
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    auto compute = [&](int buf) {
        const unsigned char* st = smem8 + buf * kStage;
        bf16x8 b[3][2];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int col = 64 * wn + 32 * s2 + r;  // piece 4 p + col / 32, slot 2 (col % 32) + half
                b[p][s2] = *(const bf16x8*)(st + kA + 1024 * (4 * p + (col >> 5)) +
                                            16 * (2 * (col & 31) + (hk ^ ((col >> 3) & 1))));
            }
#pragma unroll
        for (int i = 0; i < WI; ++i) {
            const int row = (TM / 2) * wm + 32 * i + r;
            const int f = (row >> 2) & 3;
            const f32x4_t lo = *(const f32x4_t*)(st + 64 * row + 16 * ((2 * hk) ^ f));
            const f32x4_t hi = *(const f32x4_t*)(st + 64 * row + 16 * ((2 * hk + 1) ^ f));
            bf16x8 a[3];
            split3x8(lo, hi, a[0], a[1], a[2]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x16 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2][j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0][j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1][j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1][j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0][j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0][j], c, 0, 0, 0);
                acc[i][j] = c;
            }
        }
    };
    // chunks 0 .. S - 2 in flight before the loop; chunk c + S - 1 issued at chunk c (the last chunk again past the end)
#pragma unroll
    for (int c = 0; c < S - 1; ++c) issue(min(c, nk - 1), c);
    for (int c = 0; c < nk; ++c) {
        const int buf = c % S;
        // this wave's pieces of chunk c landed: (S - 2) later chunks' pieces may stay in flight
        if constexpr (S == 2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(sg_gemm3d_pieces(TM) * (S - 2)) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk c landed; chunk c - 1's buffer is free
        asm volatile("" ::: "memory");
        issue(min(c + S - 1, nk - 1), (c + S - 1) % S);
        compute(buf);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads land before the LDS is reused
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    g3_epilogue<TM>(g, acc, (float*)smem8, wave, lane, m0, n0, Mv, Nv, z);
}

// W^T[K][N] fp32 (row-major, the packed layout) -> [3][N][K] bf16 planes for sg_gemm3_kernel; up to four matrices
// per launch (blockIdx.y), one thread per element
struct SplitJob {
    const float* W;
    __bf16* out;
    int K, N;
};
struct SplitJobs {
    SplitJob j[4];
};

__global__ void sg_split_weights_kernel(SplitJobs jobs) {
    const SplitJob jb = jobs.j[blockIdx.y];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (!jb.W || e >= (long)jb.K * jb.N) return;
    const int n = (int)(e / jb.K), k = (int)(e % jb.K);
    __bf16 h, m, l;
    split3(jb.W[(long)k * jb.N + n], h, m, l);
    const long plane = (long)jb.K * jb.N;
    jb.out[e] = h;
    jb.out[plane + e] = m;
    jb.out[2 * plane + e] = l;
}

// ------------------------------------------------------------------ fused multi-head attention
// superglue.py:84-103: prob = softmax(q k / sqrt(64)) over keys; out = prob v. One workgroup = 256 queries of one
// (pair, side, head); wave w owns queries 32 w .. +32 (two 16-query tiles) and streams the source side's keys in chunks
// of 64 (online softmax); the K1 x K2 probability matrix never reaches HBM.
constexpr int kAttnKeys = 64;
constexpr int kAttnQT = 2;                    // 16-query tiles per wave: each staged K / V fragment feeds both
// eight waves (256 queries) per workgroup share each staged key / value chunk: 21.5 ms per C5 launch against 22.1 for
// four (`profiles/r04o_c5_kernel_grid_aw*.txt`)
constexpr int kAttnWaves = 8;
constexpr int kAttnThreads = 64 * kAttnWaves;
constexpr int kAttnQ = kAttnWaves * 16 * kAttnQT;  // queries per workgroup

// On bf16 MFMA with the three-plane products of sg_gemm3_kernel (v_mfma_f32_16x16x32_bf16: A lane l = A[l % 16][8 (l /
// 16) + j], B lane l = B[8 (l / 16) + j][l % 16], C lane l, j = C[4 (l / 16) + j][l % 16]). Both products run
// transposed so that a lane keeps one query throughout:
// - S^T = K Q^T: lane (lr, lq) of key tile t holds S[query lr][key 16 t + 4 lq + j], so the softmax max / sum of a
//   query are lane-local plus two shuffles, and its running max / sum / rescale factor never leave the lane;
// - O^T = V^T P^T over 32-key slabs whose k index runs through the keys in the order the lane already holds them
//   (k = 8 lq + j' -> key 32 s + 4 lq + j' for j' < 4, 32 s + 16 + 4 lq + j' - 4 otherwise): P^T's operand is the
//   lane's own probabilities (no LDS round trip) and V^T's is read with that key order.
// Keys arrive as bf16 planes [key][64] and values transposed [64][key] (written by the q/k/v projection's epilogue),
// staged by 16-byte copies; Q is split once per wave, P per chunk. LDS rows are padded to 72 elements.
constexpr int kAttnPad = 72;

__global__ __launch_bounds__(kAttnThreads) void sg_attention3_kernel(const float* __restrict__ qkv /*q: (2P, kmax, 256)*/,
                                                             const __bf16* __restrict__ kvp, long kv_batch,
                                                             const int* __restrict__ side_counts, int kmax, int cross,
                                                             float* __restrict__ out /*(2P, kmax, 256)*/) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    // double-buffered: chunk c + 1 is stashed into the other buffer while chunk c is read (one barrier per chunk)
    __shared__ __attribute__((aligned(16))) __bf16 Ks[2][3][kAttnKeys][kAttnPad];
    __shared__ __attribute__((aligned(16))) __bf16 Vs[2][3][kHd][kAttnPad];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int qb, h, zs;
    xcd_tile(qb, h, zs);
    const int zsrc = cross ? (zs ^ 1) : zs;
    const int q0 = qb * kAttnQ + 16 * kAttnQT * wave;
    const int nkeys = side_counts[zsrc];
    const int nq = side_counts[zs];
    if (qb * kAttnQ >= nq) return;
    const int lr = lane & 15, lq = lane >> 4;
    // Q fragments (the B operand of S^T), per tile, plane and k-step: Q[q0 + 16 qt + lr][32 s + 8 lq + j]
    bf16x8 qf[kAttnQT][3][2];
#pragma unroll
    for (int qt = 0; qt < kAttnQT; ++qt) {
        const float* qrow = qkv + ((long)zs * kmax + min(q0 + 16 * qt + lr, kmax - 1)) * kD + h * kHd + 8 * lq;
#pragma unroll
        for (int s = 0; s < 2; ++s)
            split3x8(*(const f32x4_t*)(qrow + 32 * s) * 0.125f, *(const f32x4_t*)(qrow + 32 * s + 4) * 0.125f,
                     qf[qt][0][s], qf[qt][1][s], qf[qt][2][s]);  // q / sqrt(64): a power of two, exact before the split
    }
    // per tile: the lane's query's running max / sum; o[qt][u][j] = O[q0 + 16 qt + lr][16 u + 4 lq + j]
    float m_run[kAttnQT], l_run[kAttnQT];
    f32x4_t o[kAttnQT][4];
#pragma unroll
    for (int qt = 0; qt < kAttnQT; ++qt) {
        m_run[qt] = -INFINITY;
        l_run[qt] = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[qt][u] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const __bf16* kb = kvp + zsrc * kv_batch;                          // [3][head][kmax][64]
    const __bf16* vb = kvp + zsrc * kv_batch + (long)3 * kD * kmax;    // [3][head][64][kmax]
    // the next key chunk's planes are loaded into registers while the current one is processed
    constexpr int kUnits = 3 * kAttnKeys * 8 / kAttnThreads;  // 16-byte units per thread and chunk (keys, values each)
    u32x4 pk[kUnits], pv[kUnits];
    auto load = [&](int c0) {
#pragma unroll
        for (int u = 0; u < kUnits; ++u) {
            const int e = tid + kAttnThreads * u;
            const int p = e / (kAttnKeys * 8), row = (e / 8) % kAttnKeys, seg = e % 8;
            pk[u] = pv[u] = u32x4{0, 0, 0, 0};
            if (c0 + row < nkeys) pk[u] = *(const u32x4*)(kb + (((long)p * kHeads + h) * kmax + c0 + row) * kHd + 8 * seg);
            if (c0 + 8 * seg < nkeys)
                pv[u] = *(const u32x4*)(vb + (((long)p * kHeads + h) * kHd + row) * kmax + c0 + 8 * seg);
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int u = 0; u < kUnits; ++u) {
            const int e = tid + kAttnThreads * u;
            const int p = e / (kAttnKeys * 8), row = (e / 8) % kAttnKeys, seg = e % 8;
            *(u32x4*)&Ks[buf][p][row][8 * seg] = pk[u];
            *(u32x4*)&Vs[buf][p][row][8 * seg] = pv[u];
        }
    };
    load(0);
    stash(0);
    __syncthreads();
    for (int c0 = 0, buf = 0; c0 < nkeys; c0 += kAttnKeys, buf ^= 1) {
        const bool more = c0 + kAttnKeys < nkeys;
        if (more) load(c0 + kAttnKeys);
        // S^T = K Q^T / 8 for 64 keys (4 tiles of 16) x the wave's query tiles
        f32x4_t s4[kAttnQT][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int qt = 0; qt < kAttnQT; ++qt) s4[qt][t] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bf16x8 k0 = *(const bf16x8*)&Ks[buf][0][16 * t + lr][32 * s + 8 * lq];
                const bf16x8 k1 = *(const bf16x8*)&Ks[buf][1][16 * t + lr][32 * s + 8 * lq];
                const bf16x8 k2 = *(const bf16x8*)&Ks[buf][2][16 * t + lr][32 * s + 8 * lq];
#pragma unroll
                for (int qt = 0; qt < kAttnQT; ++qt) {
                    f32x4_t acc = s4[qt][t];
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k2, qf[qt][0][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qt][2][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[qt][1][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[qt][0][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qt][1][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qt][0][s], acc, 0, 0, 0);
                    s4[qt][t] = acc;
                }
            }
        }
        // online softmax per query (lane-local; the 4 lanes sharing lr hold the chunk's other keys), then P's planes
        bf16x8 pf[kAttnQT][3][2];
#pragma unroll
        for (int qt = 0; qt < kAttnQT; ++qt) {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = s4[qt][t][j];
                    if (c0 + 16 * t + 4 * lq + j >= nkeys) v = -INFINITY;
                    s4[qt][t][j] = v;
                    mx = fmaxf(mx, v);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            const float mnew = fmaxf(m_run[qt], mx);
            // exp(x) = 2^(x log2 e) on v_exp_f32 (1 ulp): x <= 0 here, so no range reduction is needed
            const float corr = __builtin_amdgcn_exp2f((m_run[qt] - mnew) * 1.44269504088896341f);
            float rs = 0.0f;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float p = __builtin_amdgcn_exp2f((s4[qt][t][j] - mnew) * 1.44269504088896341f);
                    rs = rs + p;
                    s4[qt][t][j] = p;
                }
            rs = rs + __shfl_xor(rs, 16);
            rs = rs + __shfl_xor(rs, 32);
            l_run[qt] = l_run[qt] * corr + rs;
            m_run[qt] = mnew;
#pragma unroll
            for (int u = 0; u < 4; ++u) o[qt][u] = o[qt][u] * corr;
#pragma unroll
            for (int s = 0; s < 2; ++s)
                split3x8(s4[qt][2 * s], s4[qt][2 * s + 1], pf[qt][0][s], pf[qt][1][s], pf[qt][2][s]);
        }
        // O^T += V^T P^T: A = V^T (16 dims x 32 keys of slab s, in the lane's key order), B = P^T
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 v[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    const bf16x4 a = *(const bf16x4*)&Vs[buf][pl][16 * u + lr][32 * s + 4 * lq];
                    const bf16x4 b = *(const bf16x4*)&Vs[buf][pl][16 * u + lr][32 * s + 16 + 4 * lq];
                    v[pl] = bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
                }
#pragma unroll
                for (int qt = 0; qt < kAttnQT; ++qt) {
                    f32x4_t acc = o[qt][u];
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[2], pf[qt][0][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[0], pf[qt][2][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[1], pf[qt][1][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[1], pf[qt][0][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[0], pf[qt][1][s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v[0], pf[qt][0][s], acc, 0, 0, 0);
                    o[qt][u] = acc;
                }
            }
        }
        if (more) stash(buf ^ 1);  // the other buffer's last readers passed the previous barrier
        __syncthreads();
    }
    float* ob = out + (long)zs * kmax * 256 + h * kHd;
#pragma unroll
    for (int qt = 0; qt < kAttnQT; ++qt) {
        const int q = q0 + 16 * qt + lr;
        if (q >= nq) continue;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            f32x4_t r = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
            if (l_run[qt] > 0.0f) r = o[qt][u] / l_run[qt];
            *(f32x4_t*)(ob + (long)q * 256 + 16 * u + 4 * lq) = r;
        }
    }
}

// ------------------------------------------------------------------ encoder input and descriptor init
// superglue.py:64-71 normalize_keypoints: (kpts - size / 2) / (max(W, H) * 0.7), size = (W, H); the encoder input is
// (x_n, y_n, score) (:79-81), zero-padded to 16 channels. X <- descriptors (rows >= count zeroed).
__global__ void sg_prepare_kernel(const float* __restrict__ kp, const float* __restrict__ scores,
                                  const float* __restrict__ desc, const int* __restrict__ counts,
                                  const int* __restrict__ hw, const int* __restrict__ pairs, int kmax,
                                  float* __restrict__ enc_in /*(2P, kmax, 16)*/, float* __restrict__ X,
                                  int* __restrict__ side_counts) {
    const int zs = blockIdx.y;
    const int img = pairs[zs];
    const int n = counts[img];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 && threadIdx.x == 0) side_counts[zs] = n;
    if (i >= kmax) return;
    float* e = enc_in + ((long)zs * kmax + i) * 16;
    float* x = X + ((long)zs * kmax + i) * kD;
    const float* d = desc + ((long)img * kmax + i) * kD;
    if (i < n) {
        const float W = (float)hw[2 * img + 1], H = (float)hw[2 * img];
        const float scaling = fmaxf(W, H) * 0.7f;
        e[0] = (kp[((long)img * kmax + i) * 2] - W / 2.0f) / scaling;
        e[1] = (kp[((long)img * kmax + i) * 2 + 1] - H / 2.0f) / scaling;
        e[2] = scores[(long)img * kmax + i];
        for (int c = 0; c < kD; ++c) x[c] = d[c];
    } else {
        e[0] = e[1] = e[2] = 0.0f;
        for (int c = 0; c < kD; ++c) x[c] = 0.0f;
    }
    for (int c = 3; c < 16; ++c) e[c] = 0.0f;
}

// ------------------------------------------------------------------ log-space optimal transport
// superglue.py:114-145 with iters = 20: couplings [[S, alpha], [alpha, alpha]], norm = -log(m + n),
// log_mu = [norm] * m + [log(n) + norm], log_nu = [norm] * n + [log(m) + norm],
// u = log_mu - logsumexp(Z + v, 2), v = log_nu - logsumexp(Z + u, 1); result Z + u + v - norm.
__global__ void sk_init_kernel(float* __restrict__ Z, const int* __restrict__ side_counts, int kmax,
                               const float* __restrict__ bin_score, float* __restrict__ u, float* __restrict__ v) {
    const int p = blockIdx.y;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const long ld = kmax + 1;
    float* Zp = Z + (long)p * ld * ld;
    const float alpha = bin_score[0];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m) Zp[(long)t * ld + n] = alpha;
    if (t < n) Zp[(long)m * ld + t] = alpha;
    if (t == 0) Zp[(long)m * ld + n] = alpha;
    if (t <= m) u[(long)p * ld + t] = 0.0f;
    if (t <= n) v[(long)p * ld + t] = 0.0f;
}

// exp(x) = 2^(x log2 e) on v_exp_f32 (1 ulp; arguments <= 0 here)
__device__ __forceinline__ float sk_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// online log-sum-exp over four values at a time: one running-max update and no divergent branch per element, and the
// four loads behind it are issued together (the passes stream Z from HBM: 8.3 GB each on the C5 slice)
__device__ __forceinline__ void lse_push4(const float (&x)[4], float& mx, float& s) {
    const float nm = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), mx);
    if (nm == -INFINITY) return;  // nothing seen yet (padding lanes)
    s = s * sk_exp(mx - nm) + ((sk_exp(x[0] - nm) + sk_exp(x[1] - nm)) + (sk_exp(x[2] - nm) + sk_exp(x[3] - nm)));
    mx = nm;
}

__device__ __forceinline__ void lse_merge(float& mx, float& s, float mo, float so) {
    if (mo > mx) {
        s = s * sk_exp(mx - mo) + so;
        mx = mo;
    } else if (so > 0.0f) {
        s = s + so * sk_exp(mo - mx);
    }
}

__device__ __forceinline__ float sk_norm(int m, int n) { return -logf((float)m + (float)n); }

// u[i] for rows 0..m: one wave per row
__global__ __launch_bounds__(256) void sk_rows_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                      int kmax, float* __restrict__ u, const float* __restrict__ v) {
    const int p = blockIdx.y;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i > m) return;
    const long ld = kmax + 1;
    const float* row = Z + (long)p * ld * ld + (long)i * ld;
    const float* vp = v + (long)p * ld;
    float mx = -INFINITY, s = 0.0f;
    for (int j0 = lane; j0 <= n; j0 += 256) {
        float x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = j0 + 64 * k;
            x[k] = j <= n ? row[j] + vp[j] : -INFINITY;
        }
        lse_push4(x, mx, s);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float mo = __shfl_xor(mx, o), so = __shfl_xor(s, o);
        lse_merge(mx, s, mo, so);
    }
    if (lane == 0) {
        const float norm = sk_norm(m, n);
        const float log_mu = i < m ? norm : logf((float)n) + norm;
        u[(long)p * ld + i] = log_mu - (logf(s) + mx);
    }
}

// v[j] for columns 0..n: 64 columns x 4 row groups per workgroup
__global__ __launch_bounds__(256) void sk_cols_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                      int kmax, const float* __restrict__ u, float* __restrict__ v) {
    __shared__ float pm[4][64], ps[4][64];
    const int p = blockIdx.y;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    if (blockIdx.x * 64 > n) return;
    const long ld = kmax + 1;
    const float* Zp = Z + (long)p * ld * ld;
    const float* up = u + (long)p * ld;
    float mx = -INFINITY, s = 0.0f;
    if (j <= n)
        for (int i0 = g; i0 <= m; i0 += 16) {
            float x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + 4 * k;
                x[k] = i <= m ? Zp[(long)i * ld + j] + up[i] : -INFINITY;
            }
            lse_push4(x, mx, s);
        }
    pm[g][c] = mx;
    ps[g][c] = s;
    __syncthreads();
    if (g == 0 && j <= n) {
        for (int o = 1; o < 4; ++o) lse_merge(mx, s, pm[o][c], ps[o][c]);
        const float norm = sk_norm(m, n);
        const float log_nu = j < n ? norm : logf((float)m) + norm;
        v[(long)p * ld + j] = log_nu - (logf(s) + mx);
    }
}

// One pass over Z per Sinkhorn iteration (kmax <= kSkFusedMaxK): a 64-lane workgroup takes kSkRows rows of one pair,
// lane l holding columns l + 64 k. Per row: u_i = log_mu - logsumexp_j(Z_ij + v_j) (sk_rows_kernel's grouping and
// order, so u is unchanged given v), then, from the same registers, each column's running log-sum-exp of Z_ij + u_i
// over the workgroup's rows; the partials (max, scaled sum) go to `part` and sk_vmerge_kernel turns them into v.
// Z is read once per iteration instead of twice; the column sums run in another order than sk_cols_kernel's, so v
// differs from the two-pass form in the last bits (the log-assignment tolerance of tests/test_superglue_gpu.py).
constexpr int kSkRows = 64, kSkNC = 33, kSkFusedMaxK = 64 * kSkNC - 1;
__host__ __device__ constexpr int sk_row_blocks(int kmax) { return (kmax + 1 + kSkRows - 1) / kSkRows; }

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void sk_pass_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                     int kmax, float* __restrict__ u, const float* __restrict__ v,
                                                     float2* __restrict__ part) {
    const int p = blockIdx.y, rb = blockIdx.x, lane = threadIdx.x;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int i0 = rb * kSkRows;
    const long ld = kmax + 1;
    float2* pp = part + ((long)p * sk_row_blocks(kmax) + rb) * ld;
    if (i0 > m) {  // a block wholly past the rows: an empty partial for every column
        for (int j = lane; j <= n; j += 64) pp[j] = make_float2(-INFINITY, 0.0f);
        return;
    }
    const float* Zp = Z + (long)p * ld * ld;
    __shared__ float vj[kSkNC * 64];  // v of the lane's columns (LDS: registers hold the row, its prefetch and partials)
    float cm[kSkNC], cs[kSkNC];
#pragma unroll
    for (int k = 0; k < kSkNC; ++k) {
        const int j = lane + 64 * k;
        vj[64 * k + lane] = j <= n ? v[(long)p * ld + j] : 0.0f;
        cm[k] = -INFINITY;
        cs[k] = 0.0f;
    }
    const float norm = sk_norm(m, n);
    const int i1 = min(m, i0 + kSkRows - 1);
    // row i + 1's loads are issued before row i is reduced (a wave's rows are a dependent sequence otherwise)
    float xn[kSkNC];
    auto load_row = [&](int i) {
        const float* row = Zp + (long)min(i, i1) * ld;
#pragma unroll
        for (int k = 0; k < kSkNC; ++k) {
            const int j = lane + 64 * k;
            xn[k] = j <= n ? row[j] : -INFINITY;
        }
    };
    load_row(i0);
    for (int i = i0; i <= i1; ++i) {
        float x[kSkNC];
#pragma unroll
        for (int k = 0; k < kSkNC; ++k) x[k] = xn[k];
        load_row(i + 1);
        float mx = -INFINITY, s = 0.0f;
#pragma unroll
        for (int k0 = 0; k0 < kSkNC; k0 += 4) {
            float y[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) y[q] = k0 + q < kSkNC ? x[k0 + q] + vj[64 * (k0 + q) + lane] : -INFINITY;
            lse_push4(y, mx, s);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float mo = __shfl_xor(mx, o), so = __shfl_xor(s, o);
            lse_merge(mx, s, mo, so);
        }
        const float log_mu = i < m ? norm : logf((float)n) + norm;
        const float ui = log_mu - (logf(s) + mx);
        if (lane == 0) u[(long)p * ld + i] = ui;
#pragma unroll
        for (int k = 0; k < kSkNC; ++k) {
            const float y = x[k] + ui;
            const float nm = fmaxf(cm[k], y);
            if (nm != -INFINITY) {
                cs[k] = cs[k] * sk_exp(cm[k] - nm) + sk_exp(y - nm);
                cm[k] = nm;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kSkNC; ++k) {
        const int j = lane + 64 * k;
        if (j <= n) pp[j] = make_float2(cm[k], cs[k]);
    }
}

// v_j = log_nu - logsumexp over the row blocks' partials of column j (sk_pass_kernel)
__global__ __launch_bounds__(256) void sk_vmerge_kernel(const float2* __restrict__ part,
                                                        const int* __restrict__ side_counts, int kmax,
                                                        float* __restrict__ v) {
    const int p = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    if (j > n) return;
    const long ld = kmax + 1;
    const int nrb = sk_row_blocks(kmax), used = m / kSkRows + 1;
    const float2* pp = part + (long)p * nrb * ld + j;
    float mx = -INFINITY, s = 0.0f;
    for (int r = 0; r < used; ++r) {
        const float2 q = pp[(long)r * ld];
        lse_merge(mx, s, q.x, q.y);
    }
    const float norm = sk_norm(m, n);
    const float log_nu = j < n ? norm : logf((float)m) + norm;
    v[(long)p * ld + j] = log_nu - (logf(s) + mx);
}

// row-wise max / argmax of the final scores ((Z + u) + v) - norm over the first n columns (first index on ties)
__global__ __launch_bounds__(256) void sk_rowmax_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                        int kmax, const float* __restrict__ u,
                                                        const float* __restrict__ v, float* __restrict__ max0,
                                                        int* __restrict__ idx0) {
    const int p = blockIdx.y;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= m) return;
    const long ld = kmax + 1;
    const float* row = Z + (long)p * ld * ld + (long)i * ld;
    const float ui = u[(long)p * ld + i];
    const float* vp = v + (long)p * ld;
    const float norm = sk_norm(m, n);
    float best = -INFINITY;
    int bj = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
        const float z = ((row[j] + ui) + vp[j]) - norm;
        if (z > best) { best = z; bj = j; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oj = __shfl_xor(bj, o);
        if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
    }
    if (lane == 0) {
        max0[(long)p * kmax + i] = best;
        idx0[(long)p * kmax + i] = bj;
    }
}

__global__ __launch_bounds__(256) void sk_colmax_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                        int kmax, const float* __restrict__ u,
                                                        const float* __restrict__ v, int* __restrict__ idx1) {
    __shared__ float pb[4][64];
    __shared__ int pi[4][64];
    const int p = blockIdx.y;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    if (blockIdx.x * 64 >= n) return;
    const long ld = kmax + 1;
    const float* Zp = Z + (long)p * ld * ld;
    const float* up = u + (long)p * ld;
    const float norm = sk_norm(m, n);
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if (j < n) {
        const float vj = v[(long)p * ld + j];
        for (int i = g; i < m; i += 4) {
            const float z = ((Zp[(long)i * ld + j] + up[i]) + vj) - norm;
            if (z > best) { best = z; bi = i; }
        }
    }
    pb[g][c] = best;
    pi[g][c] = bi;
    __syncthreads();
    if (g == 0 && j < n) {
        for (int o = 1; o < 4; ++o)
            if (pb[o][c] > best || (pb[o][c] == best && pi[o][c] < bi)) { best = pb[o][c]; bi = pi[o][c]; }
        idx1[(long)p * kmax + j] = bi;
    }
}

// mutual check + threshold (superglue.py:268-276), matches in ascending i (superglue_matcher.py:104-109)
__global__ __launch_bounds__(256) void sg_emit_kernel(const int* __restrict__ side_counts, int kmax,
                                                      const float* __restrict__ max0, const int* __restrict__ idx0,
                                                      const int* __restrict__ idx1, float threshold,
                                                      uint32_t* __restrict__ out_idx, int* __restrict__ out_count,
                                                      float* __restrict__ out_mscore) {
    __shared__ int sh[4];
    const int p = blockIdx.x;
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int base = 0;
    for (int i0 = 0; i0 < kmax; i0 += 256) {
        const int i = i0 + threadIdx.x;
        int valid = 0;
        float ms = 0.0f;
        int j = -1;
        if (i < m && n > 0) {
            j = idx0[(long)p * kmax + i];
            const bool mutual = idx1[(long)p * kmax + j] == i;
            ms = mutual ? expf(max0[(long)p * kmax + i]) : 0.0f;
            valid = (mutual && ms > threshold) ? 1 : 0;
        }
        if (out_mscore && i < kmax) out_mscore[(long)p * kmax + i] = i < m ? ms : 0.0f;
        int x = valid;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) sh[wave] = x;
        __syncthreads();
        int off = base;
        for (int w = 0; w < wave; ++w) off += sh[w];
        const int total = sh[0] + sh[1] + sh[2] + sh[3];
        if (valid) {
            const int o = off + x - 1;
            out_idx[((long)p * kmax + o) * 2] = (uint32_t)i;
            out_idx[((long)p * kmax + o) * 2 + 1] = (uint32_t)j;
        }
        base += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) out_count[p] = base;
}

// final log-assignment of one pair ((Z + u) + v) - norm, rows 0..m, columns 0..n (ld = kmax + 1), NaN elsewhere
__global__ __launch_bounds__(256) void sk_final_kernel(const float* __restrict__ Z, const int* __restrict__ side_counts,
                                                       int kmax, const float* __restrict__ u,
                                                       const float* __restrict__ v, int p, float* __restrict__ out) {
    const int m = side_counts[2 * p], n = side_counts[2 * p + 1];
    const long ld = kmax + 1;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= ld * ld) return;
    const int i = (int)(e / ld), j = (int)(e % ld);
    out[e] = (i <= m && j <= n) ? ((Z[(long)p * ld * ld + e] + u[(long)p * ld + i]) + v[(long)p * ld + j]) -
                                      sk_norm(m, n)
                                : __builtin_nanf("");
}

// ------------------------------------------------------------------ host-side orchestration
struct SgLayout {
    size_t enc_in, X, T1, T2, qkv, kvp, att, msg, hid, Z, u, v, part, max0, idx0, idx1, cnt, wsplit, total;
};

// bf16 planes of one GNN layer's four weight matrices (Wqkv, Wm, W1, W2), reused by the final projection
constexpr size_t kSplitElems = (size_t)256 * 768 + 256 * 256 + 512 * 512 + 512 * 256;

__host__ SgLayout sg_layout(int P, int kmax) {
    SgLayout L{};
    const size_t S = (size_t)2 * P * kmax;
    const size_t ld = (size_t)kmax + 1;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += gtsfm_align_up(bytes, 256); return r; };
    L.enc_in = take(S * 16 * 4);
    L.X = take(S * kD * 4);
    L.T1 = take(S * kD * 4);
    L.T2 = take(S * kD * 4);
    L.qkv = take(S * kD * 4);  // q only: keys and values go straight to the bf16 planes (kvp)
    L.kvp = take(S * 2 * kD * 3 * sizeof(__bf16));  // key and value planes of the current layer
    L.att = take(S * kD * 4);
    L.msg = take(S * kD * 4);
    L.hid = take(S * 512 * 4);
    L.Z = take((size_t)P * ld * ld * 4);
    L.u = take((size_t)P * ld * 4);
    L.v = take((size_t)P * ld * 4);
    L.part = take((size_t)P * sk_row_blocks(kmax) * ld * sizeof(float2));  // Sinkhorn column partials
    L.max0 = take((size_t)P * kmax * 4);
    L.idx0 = take((size_t)P * kmax * 4);
    L.idx1 = take((size_t)P * kmax * 4);
    L.cnt = take((size_t)2 * P * 4);
    L.wsplit = take(kSplitElems * 3 * sizeof(__bf16));
    L.total = o;
    return L;
}

hipError_t run_gemm(const GemmArgs& g, int batches, hipStream_t stream) {
    const dim3 grid((unsigned)((g.N + 63) / 64), (unsigned)((g.M + 63) / 64), (unsigned)batches);
    hipLaunchKernelGGL(sg_gemm_kernel, grid, dim3(kGemmThreads), 0, stream, g);
    return hipGetLastError();
}

hipError_t run_gemm3(const Gemm3Args& g, int batches, hipStream_t stream) {
    if (g.kv && (g.m_lim || g.M % 64 != 0)) return hipErrorInvalidValue;  // kv stores write whole 4-key groups
    // LDS-DMA staging (sg_gemm3d_kernel) for the weight GEMMs whose A rows are 16-byte aligned: 256-row tiles for N >=
    // 512, else 128, two chunks in flight. C5 slice, same box (profiles/r06p_*): q/k/v + W1 7.20 -> 6.58 ms, Wm + W2
    // 3.35 -> 2.72 ms per launch, 551 -> 574 pairs/s (128-row tiles throughout: 563; three chunks in flight: 542).
    // GTSFM_SG_GEMM_DMA (test and A/B hooks): 0 the register-staged kernel, 2 / 3 128-row tiles with 2 / 3 chunks.
    // Measured and not kept (profiles/r06q_*): the GNN's A operands pre-split into bf16 planes by their producers
    // (attention / GEMM epilogues) and staged as planes, no split in the loop: bit-identical but 7.54 / 3.82 ms per
    // launch against 6.39 / 2.70 -- 1.5x the operand bytes and a third more LDS-DMA pieces cost more than the split.
    const char* dma_env = getenv("GTSFM_SG_GEMM_DMA");
    const char dma_mode = dma_env && dma_env[0] ? dma_env[0] : '4';
    const bool aligned = g.lda % 4 == 0 && ((uintptr_t)g.A & 15) == 0 &&
                         (!g.A2 || (g.lda2 % 4 == 0 && ((uintptr_t)g.A2 & 15) == 0)) && g.Ksplit % 16 == 0;
    if (dma_mode != '0' && g.Bp && aligned && g.K % 16 == 0) {
        // '2' / '3': 128-row tiles, 2 / 3 chunks in flight; '4': 256-row tiles for N >= 512, 2 chunks
        const bool wide = dma_mode == '4' && g.N >= 512;
        const int tm = wide ? 256 : 128, stages = dma_mode == '3' ? 3 : 2;
        const dim3 grid((unsigned)((g.N + kG3Tile - 1) / kG3Tile), (unsigned)((g.M + tm - 1) / tm), (unsigned)batches);
        const void* fn = wide ? (const void*)sg_gemm3d_kernel<256, 2>
                              : (stages == 2 ? (const void*)sg_gemm3d_kernel<128, 2> : (const void*)sg_gemm3d_kernel<128, 3>);
        const int lds = sg_gemm3d_lds(tm, stages);
        if (gtsfm_set_dynamic_lds(fn, lds) != hipSuccess) return hipErrorInvalidValue;
        if (wide)
            hipLaunchKernelGGL((sg_gemm3d_kernel<256, 2>), grid, dim3(256), lds, stream, g);
        else if (stages == 2)
            hipLaunchKernelGGL((sg_gemm3d_kernel<128, 2>), grid, dim3(256), lds, stream, g);
        else
            hipLaunchKernelGGL((sg_gemm3d_kernel<128, 3>), grid, dim3(256), lds, stream, g);
        return hipGetLastError();
    }
    if (g.N >= 512) {
        const void* fn = (const void*)sg_gemm3_kernel<kG3Kc, kG3Slots, 256>;
        const int lds = sg_gemm3_lds(256);
        if (gtsfm_set_dynamic_lds(fn, lds) != hipSuccess) return hipErrorInvalidValue;
        const dim3 grid((unsigned)((g.N + kG3Tile - 1) / kG3Tile), (unsigned)((g.M + 255) / 256), (unsigned)batches);
        hipLaunchKernelGGL((sg_gemm3_kernel<kG3Kc, kG3Slots, 256>), grid, dim3(256), lds, stream, g);
    } else {
        const void* fn = (const void*)sg_gemm3_kernel<kG3Kc, kG3Slots, 128>;
        const int lds = sg_gemm3_lds(128);
        if (gtsfm_set_dynamic_lds(fn, lds) != hipSuccess) return hipErrorInvalidValue;
        const dim3 grid((unsigned)((g.N + kG3Tile - 1) / kG3Tile), (unsigned)((g.M + 127) / 128), (unsigned)batches);
        hipLaunchKernelGGL((sg_gemm3_kernel<kG3Kc, kG3Slots, 128>), grid, dim3(256), lds, stream, g);
    }
    return hipGetLastError();
}

// Y[z] = A[z] W (+ bias) with W's planes Wp ([3][N][K]) for every (pair, side) block
Gemm3Args side_gemm3(const float* A, int lda, const __bf16* Wp, int K, int N, const float* bias, float* C, int ldc,
                     int kmax) {
    Gemm3Args g{};
    g.A = A; g.lda = lda; g.a_batch = (long)kmax * lda;
    g.A2 = nullptr; g.Ksplit = K;
    g.Bp = Wp;
    g.bias = bias; g.alpha = 1.0f;
    g.C = C; g.ldc = ldc; g.c_batch = (long)kmax * ldc;
    g.M = kmax; g.N = N; g.K = K;
    return g;
}

hipError_t split_weights(const SplitJobs& jobs, hipStream_t stream) {
    long most = 0;
    for (int i = 0; i < 4; ++i)
        if (jobs.j[i].W) most = std::max(most, (long)jobs.j[i].K * jobs.j[i].N);
    hipLaunchKernelGGL(sg_split_weights_kernel, dim3((unsigned)((most + 255) / 256), 4), dim3(256), 0, stream, jobs);
    return hipGetLastError();
}

GemmArgs side_gemm(const float* A, int lda, const float* W, int K, int N, const float* bias, float* C, int ldc,
                   int kmax) {
    GemmArgs g{};
    g.A = A; g.lda = lda; g.a_batch = (long)kmax * lda;
    g.A2 = nullptr; g.Ksplit = K;
    g.B = W; g.ldb = N; g.b_batch = 0; g.b_trans = 0;
    g.bias = bias; g.alpha = 1.0f;
    g.C = C; g.ldc = ldc; g.c_batch = (long)kmax * ldc;
    g.M = kmax; g.N = N; g.K = K;
    return g;
}

}  // namespace

extern "C" {

size_t gtsfm_superglue_weights_floats(int n_layers) { return n_layers > 0 ? sg_weights_floats(n_layers) : 0; }

size_t gtsfm_superglue_workspace_bytes(int n_pairs, int kmax) {
    if (n_pairs <= 0 || kmax <= 0) return 0;
    return sg_layout(n_pairs, (kmax + 63) / 64 * 64).total;
}

int gtsfm_superglue_batched(const float* d_kp, const float* d_scores, const float* d_desc, const int* d_counts,
                            const int* d_image_hw, int n_img, int kmax, const int* d_pairs, int n_pairs,
                            const float* d_weights, int n_layers, int sinkhorn_iters, float match_threshold,
                            void* d_workspace, size_t workspace_bytes, uint32_t* d_out_idx, int* d_out_count,
                            float* d_out_mscores, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_kp || !d_scores || !d_desc || !d_counts || !d_image_hw || !d_pairs || !d_weights || !d_workspace ||
        !d_out_idx || !d_out_count || n_img <= 0 || kmax <= 0 || n_pairs < 0 || n_layers <= 0 || sinkhorn_iters < 0 ||
        kmax % 64 != 0)
        return GTSFM_ERR_ARG;
    const SgLayout L = sg_layout(n_pairs, kmax);
    if (workspace_bytes < L.total) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    float* enc_in = (float*)(ws + L.enc_in);
    float* X = (float*)(ws + L.X);
    float* T1 = (float*)(ws + L.T1);
    float* T2 = (float*)(ws + L.T2);
    float* qkv = (float*)(ws + L.qkv);
    __bf16* kvp = (__bf16*)(ws + L.kvp);
    const long kv_batch = (long)2 * 3 * kD * kmax;
    float* att = (float*)(ws + L.att);
    float* msg = (float*)(ws + L.msg);
    float* hid = (float*)(ws + L.hid);
    float* Z = (float*)(ws + L.Z);
    float* u = (float*)(ws + L.u);
    float* v = (float*)(ws + L.v);
    float* max0 = (float*)(ws + L.max0);
    int* idx0 = (int*)(ws + L.idx0);
    int* idx1 = (int*)(ws + L.idx1);
    int* side_counts = (int*)(ws + L.cnt);
    __bf16* wsp = (__bf16*)(ws + L.wsplit);
    __bf16* Pqkv = wsp;                        // [3][768][256]
    __bf16* Pm = Pqkv + 3 * (size_t)768 * 256;  // [3][256][256]
    __bf16* P1 = Pm + 3 * (size_t)256 * 256;    // [3][512][512]
    __bf16* P2 = P1 + 3 * (size_t)512 * 512;    // [3][256][512]
    const int S = 2 * n_pairs;
    hipLaunchKernelGGL(sg_prepare_kernel, dim3((kmax + 255) / 256, S), dim3(256), 0, stream, d_kp, d_scores, d_desc,
                       d_counts, d_image_hw, d_pairs, kmax, enc_in, X, side_counts);
    GTSFM_CHECK_HIP(hipGetLastError());
    // keypoint encoder (superglue.py:74-81): MLP [3, 32, 64, 128, 256, 256], BN + ReLU between layers; desc += enc
    const float* w = d_weights;
    {
        const float* in = enc_in;
        int cin = 16;
        float* bufs[2] = {T1, T2};
        for (int i = 0; i < 5; ++i) {
            const float* W = w;
            const float* bias = W + (size_t)kEncIn[i] * kEncOut[i];
            const int co = kEncOut[i];
            GemmArgs g = side_gemm(in, cin, W, kEncIn[i], co, bias, i < 4 ? bufs[i & 1] : X, i < 4 ? co : kD, kmax);
            if (i < 4) {
                g.bn_scale = bias + co;
                g.bn_shift = bias + 2 * co;
                g.relu = 1;
            } else {
                g.residual = 1;  // desc0 + kenc(...)
            }
            GTSFM_CHECK_HIP(run_gemm(g, S, stream));
            in = bufs[i & 1];
            cin = co;
            w += enc_floats(i);
        }
    }
    // attentional GNN (superglue.py:104-121): layer l is 'self' for even l, 'cross' for odd l
    for (int l = 0; l < n_layers; ++l) {
        const float* Wqkv = w;
        const float* bqkv = Wqkv + 256 * 768;
        const float* Wm = bqkv + 768;
        const float* bm = Wm + 256 * 256;
        const float* W1 = bm + 256;
        const float* b1 = W1 + 512 * 512;
        const float* s1 = b1 + 512;
        const float* h1 = s1 + 512;
        const float* W2 = h1 + 512;
        const float* b2 = W2 + 512 * 256;
        w += kLayerFloats;
        GTSFM_CHECK_HIP(split_weights(SplitJobs{{{Wqkv, Pqkv, kD, 768}, {Wm, Pm, kD, kD}, {W1, P1, 512, 512},
                                                 {W2, P2, 512, kD}}},
                                      stream));
        Gemm3Args gq = side_gemm3(X, kD, Pqkv, kD, 768, bqkv, qkv, kD, kmax);  // C = q (columns < 256), ldc 256
        gq.kv = kvp;
        gq.kv_batch = kv_batch;
        GTSFM_CHECK_HIP(run_gemm3(gq, S, stream));
        hipLaunchKernelGGL(sg_attention3_kernel, dim3((kmax + kAttnQ - 1) / kAttnQ, kHeads, S), dim3(kAttnThreads), 0,
                           stream, qkv, kvp, kv_batch, side_counts, kmax, l & 1, att);
        GTSFM_CHECK_HIP(hipGetLastError());
        GTSFM_CHECK_HIP(run_gemm3(side_gemm3(att, kD, Pm, kD, kD, bm, msg, kD, kmax), S, stream));
        Gemm3Args g1 = side_gemm3(X, kD, P1, 512, 512, b1, hid, 512, kmax);
        g1.Ksplit = kD;  // cat([x, message])
        g1.A2 = msg;
        g1.lda2 = kD;
        g1.a2_batch = (long)kmax * kD;
        g1.bn_scale = s1;
        g1.bn_shift = h1;
        g1.relu = 1;
        GTSFM_CHECK_HIP(run_gemm3(g1, S, stream));
        Gemm3Args g2 = side_gemm3(hid, 512, P2, 512, kD, b2, X, kD, kmax);
        g2.residual = 1;  // desc + delta
        GTSFM_CHECK_HIP(run_gemm3(g2, S, stream));
    }
    // final projection, scores = mdesc0^T mdesc1 / 16 into the coupling matrix interior
    const float* Wf = w;
    const float* bf = Wf + 256 * 256;
    const float* bin = bf + 256;
    GTSFM_CHECK_HIP(split_weights(SplitJobs{{{Wf, Pm, kD, kD}, {}, {}, {}}}, stream));
    GTSFM_CHECK_HIP(run_gemm3(side_gemm3(X, kD, Pm, kD, kD, bf, T1, kD, kmax), S, stream));
    const long ld = kmax + 1;
    {
        Gemm3Args g{};
        g.A = T1; g.lda = kD; g.a_batch = (long)2 * kmax * kD;
        g.Ksplit = kD;
        g.Bt = T1 + (long)kmax * kD; g.ldb = kD; g.b_batch = (long)2 * kmax * kD;
        g.alpha = 1.0f / 16.0f;
        g.C = Z; g.ldc = ld; g.c_batch = ld * ld;
        g.M = kmax; g.N = kmax; g.K = kD;
        g.m_lim = side_counts; g.n_lim = side_counts; g.lim_stride = 2;
        GTSFM_CHECK_HIP(run_gemm3(g, n_pairs, stream));
    }
    hipLaunchKernelGGL(sk_init_kernel, dim3((kmax + 256) / 256, n_pairs), dim3(256), 0, stream, Z, side_counts, kmax,
                       bin, u, v);
    // Sinkhorn: one pass over Z per iteration (sk_pass_kernel + sk_vmerge_kernel) for kmax <= 2048 (33 columns per
    // lane), else two passes (sk_rows_kernel, sk_cols_kernel). C5 slice match stage 860 -> 826 ms per step, 532
    // -> 555 pairs/s (profiles/r06m_*). Round 5's one-pass form (a workgroup's 8 rows of Z in LDS, 65 KB, phases in
    // series) ran 7.35 ms per iteration against 2.09 + 2.01 ms for the two passes; this one keeps the rows and the
    // column partials in registers (one 64-lane wave per 64 rows, the next row prefetched) and needs no LDS for Z.
    const char* sk_env = getenv("GTSFM_SG_SINKHORN_TWO_PASS");  // test hook: the two-pass form below
    if (kmax <= kSkFusedMaxK && !(sk_env && sk_env[0] == '1')) {
        float2* part = (float2*)(ws + L.part);
        for (int it = 0; it < sinkhorn_iters; ++it) {
            hipLaunchKernelGGL(sk_pass_kernel, dim3(sk_row_blocks(kmax), n_pairs), dim3(64), 0, stream, Z,
                               side_counts, kmax, u, (const float*)v, part);
            hipLaunchKernelGGL(sk_vmerge_kernel, dim3((kmax + 256) / 256, n_pairs), dim3(256), 0, stream,
                               (const float2*)part, side_counts, kmax, v);
        }
    } else {
        for (int it = 0; it < sinkhorn_iters; ++it) {
            hipLaunchKernelGGL(sk_rows_kernel, dim3((kmax + 4) / 4, n_pairs), dim3(256), 0, stream, Z, side_counts,
                               kmax, u, (const float*)v);
            hipLaunchKernelGGL(sk_cols_kernel, dim3((kmax + 64) / 64, n_pairs), dim3(256), 0, stream, Z, side_counts,
                               kmax, (const float*)u, v);
        }
    }
    hipLaunchKernelGGL(sk_rowmax_kernel, dim3(kmax / 4, n_pairs), dim3(256), 0, stream, Z, side_counts, kmax, u, v,
                       max0, idx0);
    hipLaunchKernelGGL(sk_colmax_kernel, dim3(kmax / 64, n_pairs), dim3(256), 0, stream, Z, side_counts, kmax, u, v,
                       idx1);
    hipLaunchKernelGGL(sg_emit_kernel, dim3(n_pairs), dim3(256), 0, stream, side_counts, kmax, max0, idx0, idx1,
                       match_threshold, d_out_idx, d_out_count, d_out_mscores);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

int gtsfm_superglue_log_assignment(const void* d_workspace, size_t workspace_bytes, int n_pairs, int kmax, int pair,
                                   float* d_out, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (!d_workspace || !d_out || n_pairs <= 0 || pair < 0 || pair >= n_pairs || kmax <= 0 || kmax % 64 != 0)
        return GTSFM_ERR_ARG;
    const SgLayout L = sg_layout(n_pairs, kmax);
    if (workspace_bytes < L.total) return GTSFM_ERR_CAPACITY;
    const unsigned char* ws = (const unsigned char*)d_workspace;
    const long ld = kmax + 1;
    hipLaunchKernelGGL(sk_final_kernel, dim3((unsigned)((ld * ld + 255) / 256)), dim3(256), 0, stream,
                       (const float*)(ws + L.Z), (const int*)(ws + L.cnt), kmax, (const float*)(ws + L.u),
                       (const float*)(ws + L.v), pair, d_out);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
