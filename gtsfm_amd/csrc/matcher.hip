// Mutual-nearest-neighbour + ratio-test matcher for batches of image pairs (gfx950).
//
// Replaces gtsfm/frontend/matcher/twoway_matcher.py:42-144 (TwoWayMatcher.match): two one-way
// cv.BFMatcher(NORM_L2).knnMatch(k=2) passes (:102, :136), the ratio test `m1.distance <= r*m2.distance`
// (:137), the stable sort by distance (:141), the query->train dict (:142) and the mutual filter in
// 1->2 order (:117-120).
//
// Fast path (GTSFM_MATCH_INT_F16): one K1 x K2 distance GEMM per pair on fp16 MFMA
// (v_mfma_f32_32x32x16_f16). The squared norms are folded into 4 extra K columns, so the accumulator
// IS the squared L2 distance:   A'_r = [a, |a|^2 mod 2048, |a|^2 div 2048, 1, 2048, 2048]
//                               B'_c = [-2b, 1, 2048, |b|^2 mod 2048, |b|^2 div 2048, 4096]
// (the last column adds 2^23, see the epilogue)
// Every factor is an integer exactly representable in fp16 and every partial sum is an integer < 2^24,
// so the fp32 accumulation is exact in any order: d2 = |a|^2 + |b|^2 - 2 a.b exactly.
// The epilogue keeps a running top-2 per row in registers and per column through LDS; the K1 x K2 matrix is never
// written to HBM. Columns (image i1) track packed keys d2 << ib | row (ib = max(11, ceil log2 kmax)); rows (image i2)
// track distance VALUES only, with no key build. Both insert two values at a time (v_min3 + v_med3 + v_min per pair):
// 3.8 VALU per distance. In finalize, i1's keypoint i with nearest j is mutual iff j's best distance equals d(i, j) and
// j has no tie at its minimum; tied j are recomputed exactly (rare). Lexicographic (d2, index) order == OpenCV's
// strict-'<' scan order, and for d2 < 2^22 ordering by d2 equals ordering by sqrtf(d2), so results are bit-identical
// to the oracle.
//
// Exact path (GTSFM_MATCH_EXACT_F32): float descriptors, per-row sequential fp32 sums (no FMA
// contraction), top-2 on sqrtf distances — the oracle's arithmetic, for tests and non-SIFT data.
//
// Both paths end in match_finalize_kernel: ratio test in double on float32 distances, mutual check,
// LDS compaction and a bitonic sort on (distance, i1) — the reference's output order.
#include "common.hpp"

#include <type_traits>

namespace {

// Packed key = (d2 << ib) | index with ib = ceil(log2(kmax)) (>= 11) index bits and 32-ib distance bits.
// d2 saturates at 2^(32-ib)-1; finalize recomputes any row/column whose top-2 touched the saturated value.
constexpr uint32_t kNoKey = 0xFFFFFFFFu;
constexpr int kMaxKmaxPacked = 8192;   // fast path
// Correctly rounded fp32 square root, as the oracle's sqrtf (HIP's __fsqrt_rn is the ~1-ulp native sqrt).
__device__ __forceinline__ float sqrt_cr(float x) { return __builtin_sqrtf(x); }

constexpr int kMaxKmax = 65535;        // exact path (16-bit indices in the sort key)

inline int index_bits(int kmax) {
    int b = 11;
    while ((1 << b) < kmax) ++b;
    return b;
}

// ---------------------------------------------------------------------------------------------
// Pack float descriptors into the two fp16 MFMA operand forms (norm digits folded into K).
// A form: row-major [img][kpad][da]. B form: fragment-major per 32-row chunk, [img][chunk][s][h][r][8] with
// k = 16 s + 8 h + e: the 64 16-B granules one MFMA k-step reads (rows r = 0..31 x halves h) are one contiguous
// KiB, so a linear LDS-DMA copy of the chunk gives conflict-free ds_read_b128 at lane * 16.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ size_t b_form_index(int img, int row, int k, int kpad, int da) {
    const size_t chunk = (size_t)img * kpad + (row & ~31);
    return chunk * da + (size_t)(k >> 4) * 512 + ((k >> 3) & 1) * 256 + (row & 31) * 8 + (k & 7);
}

__global__ void pack_desc_kernel(const float* __restrict__ desc, const int* __restrict__ counts, int kmax, int dim,
                                 int kpad, int da, _Float16* __restrict__ a_form, _Float16* __restrict__ b_form) {
    const int img = blockIdx.y;
    const int row = blockIdx.x * blockDim.y + threadIdx.y;  // one 64-lane wave per descriptor row
    if (row >= kpad) return;
    const int lane = threadIdx.x;
    const int n = counts[img];
    _Float16* ar = a_form + ((size_t)img * kpad + row) * da;
    if (row >= n) {  // padding rows: all-zero operands (masked in the epilogue)
        for (int k = lane; k < da; k += 64) {
            ar[k] = (_Float16)0.f;
            b_form[b_form_index(img, row, k, kpad, da)] = (_Float16)0.f;
        }
        return;
    }
    const float* src = desc + ((size_t)img * kmax + row) * dim;
    float sq = 0.f;
    for (int k = lane; k < dim; k += 64) {
        float v = src[k];
        sq += v * v;  // integer-valued: exact
        ar[k] = (_Float16)v;
        b_form[b_form_index(img, row, k, kpad, da)] = (_Float16)(-2.f * v);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
    const uint32_t nsq = (uint32_t)sq;
    const float lo = (float)(nsq & 2047u), hi = (float)(nsq >> 11);
    for (int k = dim + lane; k < da; k += 64) {
        const int e = k - dim;
        float av = 0.f, bv = 0.f;
        if (e == 0) { av = lo; bv = 1.f; }
        else if (e == 1) { av = hi; bv = 2048.f; }
        else if (e == 2) { av = 1.f; bv = lo; }
        else if (e == 3) { av = 2048.f; bv = hi; }
        else if (e == 4) { av = 2048.f; bv = 4096.f; }  // + 2^23: accumulator bits = 0x4B000000 | d2
        ar[k] = (_Float16)av;
        b_form[b_form_index(img, row, k, kpad, da)] = (_Float16)bv;
    }
}

// ---------------------------------------------------------------------------------------------
// Fused distance GEMM + row/column top-2. One workgroup (4 waves) per pair.
// Each wave owns 64 rows (two 32-row MFMA tiles) of a 256-row pass; B streams through LDS in
// 32-column chunks (double buffered, 304-B padded rows: conflict-free ds_read_b128).
// ---------------------------------------------------------------------------------------------
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kRowsPerPass = kWaves * 64;
constexpr int kChunk = 32;

template <int NK>  // NK = da / 16 k-steps
struct MnnCfg {
    static constexpr int kDa = NK * 16;
    static constexpr int kRowBytes = kDa * 2;                      // 288 B at dim 128 (B-form row)
    static constexpr int kBufBytes = kChunk * kRowBytes;           // one B chunk, contiguous in HBM
    static constexpr int kGlds = kBufBytes / 1024;                 // 1-KiB LDS-DMA wave-instructions
    static_assert(kBufBytes % 1024 == 0, "chunk must be whole 1-KiB LDS-DMA pieces");
};

// Async HBM -> LDS copy of one 1-KiB piece by one wave (lane l moves bytes [16l, 16l+16)).
__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                     (__attribute__((address_space(3))) void*)ldst, 16, 0, 0);
}

// A fifth folded K column (A' = 2048, B' = 4096) adds 2^23 to every accumulator, so each holds 2^23 + d2 exactly
// (d2 < 2^20 for non-negative integer descriptors with |a|^2 < 2^19) and its bit pattern is 0x4B000000 | d2.
// kFast (ib <= 12, i.e. kmax <= 4096): the packed key is one v_lshl_or_b32 of the raw accumulator bits (the shift
// drops exponent and sign), no conversion and no saturation. ib = 13 converts, subtracts 2^23 and saturates.
// B streams through LDS in super-chunks of kSub x 32 columns per barrier; the column partials of a super-chunk are
// merged by one wave with all 64 lanes busy.
constexpr int kSub = 2;
constexpr int kSuper = kSub * kChunk;

// Orientation: the GEMM's rows (A operand, held in registers) are image i2's keypoints and its columns (B operand,
// streamed through LDS) are image i1's. Pairs arrive in lexicographic (i1, i2) order, so consecutive pairs share the
// streamed image; the XCD-aware block remap below hands every XCD a contiguous run of pairs, so the workgroups
// resident on one XCD stream the same B image out of that XCD's L2 instead of re-reading it from HBM.
//   rowres[p][j2] = top-2 of image i2's keypoint j2 (distance values in kFast, packed keys otherwise)
//   colres[p][j1] = top-2 packed keys of image i1's keypoint j1 (index = keypoint of i2)
template <int NK, bool kFast>
__global__ __launch_bounds__(kThreads, 2) void mnn_mfma_kernel(const _Float16* __restrict__ a_form,
                                                               const _Float16* __restrict__ b_form,
                                                               const int* __restrict__ counts,
                                                               const int* __restrict__ pairs, int n_pairs,
                                                               int kpad, int kmax, int ib,
                                                               uint2* __restrict__ rowres,
                                                               uint2* __restrict__ colres) {
    using Cfg = MnnCfg<NK>;
    constexpr int kSupBytes = kSub * Cfg::kBufBytes;
    const uint32_t dsat = (1u << (32 - ib)) - 1u;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* bbuf = smem;                                      // [2][kSuper][kRowBytes]
    uint32_t* partial = (uint32_t*)(smem + 2 * kSupBytes);           // [2][kWaves][kSuper][2]
    uint2* colstate = (uint2*)(partial + 2 * kWaves * kSuper * 2);   // [kmax]

    // bijective XCD remap (blocks b, b + 8, ... share an XCD and take consecutive pairs)
    const int blk = blockIdx.x, xcd = blk & 7, q8 = n_pairs >> 3, r8 = n_pairs & 7;
    const int p = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blk >> 3);
    const int img_a = pairs[2 * p + 1], img_b = pairs[2 * p];
    const int n1 = counts[img_a], n2 = counts[img_b];  // n1 rows (A), n2 columns (B)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lrow = lane & 31, half = lane >> 5;
    if (n1 <= 0 || n2 <= 0) return;  // nothing to match; finalize reads zero rows

    const _Float16* A = a_form + (size_t)img_a * kpad * Cfg::kDa;
    const unsigned char* Bbytes = (const unsigned char*)(b_form + (size_t)img_b * kpad * Cfg::kDa);
    uint2* rres = rowres + (size_t)p * kmax;
    uint2* cres = colres + (size_t)p * kmax;

    for (int c = tid; c < n2; c += kThreads) colstate[c] = make_uint2(kNoKey, kNoKey);
    const int nsup = (n2 + kSuper - 1) / kSuper;

    // Super-chunk `sc` of B (kSuper consecutive B-form rows, contiguous in HBM; B-form rows are padded to kpad,
    // a multiple of 256, so a whole super-chunk is always in bounds) -> LDS buffer `buf`.
    auto issue_super = [&](int sc, int buf) {
        const unsigned char* src = Bbytes + (size_t)sc * kSupBytes + lane * 16;
        unsigned char* dst = bbuf + buf * kSupBytes;
        for (int q = wave; q < kSub * Cfg::kGlds; q += kWaves) glds16(src + q * 1024, dst + q * 1024);
    };
    // Merge the 4 waves' column partials of super-chunk `sc` (buffer pb) into colstate (one wave, lane = column).
    auto merge_partials = [&](int sc, int pb) {
        if (wave == (sc & (kWaves - 1))) {
            const int col = sc * kSuper + lane;
            if (col < n2) {
                uint2 s = colstate[col];
                uint32_t s1 = s.x, s2 = s.y;
#pragma unroll
                for (int w = 0; w < kWaves; ++w) {
                    const uint32_t* pp = partial + ((pb * kWaves + w) * kSuper + lane) * 2;
                    top2_merge(s1, s2, pp[0], pp[1]);
                }
                colstate[col] = make_uint2(s1, s2);
            }
        }
    };

    for (int rp = 0; rp < n1; rp += kRowsPerPass) {
        const int r0w = rp + wave * 64;
        // A fragments for this wave's two row tiles: lane holds A[row = lrow][k = 16s + 8*half .. +8].
        half8 afrag[2][NK];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const _Float16* arow = A + (size_t)(r0w + 32 * t + lrow) * Cfg::kDa + 8 * half;
#pragma unroll
            for (int s = 0; s < NK; ++s) afrag[t][s] = *(const half8*)(arow + 16 * s);
        }
        uint32_t rb1[2][16], rb2[2][16];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 16; ++g) rb1[t][g] = rb2[t][g] = kNoKey;
        const bool rows_partial1 = (r0w + 64 > n1);  // either row tile of this wave is partial

        issue_super(0, 0);
        __syncthreads();  // vmcnt(0) + barrier: super-chunk 0 landed, colstate initialised

        for (int sc = 0; sc < nsup; ++sc) {
            const int buf = sc & 1;
            if (sc + 1 < nsup) issue_super(sc + 1, buf ^ 1);  // lands during this super-chunk's MFMAs
            // Both 32-column chunks of the super-chunk against both row tiles (acc[sub][t]), so every row sees two
            // new distances per epilogue and takes them with one paired top-2 insert (3 VALU per 2 distances).
            // B fragments: lane holds B[k = 16s + 8*half .. +8][col = lrow]; 2-way bank conflict on 288-B rows.
            const unsigned char* bb = bbuf + buf * kSupBytes + lane * 16;
            f32x16 acc[kSub][2];
#pragma unroll
            for (int sub = 0; sub < kSub; ++sub) acc[sub][0] = acc[sub][1] = f32x16{};
#pragma unroll
            for (int s = 0; s < NK; ++s) {
#pragma unroll
                for (int sub = 0; sub < kSub; ++sub) {
                    const half8 bf = *(const half8*)(bb + sub * Cfg::kBufBytes + 1024 * s);
                    acc[sub][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(afrag[0][s], bf, acc[sub][0], 0, 0, 0);
                    acc[sub][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(afrag[1][s], bf, acc[sub][1], 0, 0, 0);
                }
            }

            const int c0 = sc * kSuper;
            const bool cols_partial = (c0 + kSuper > n2);
            uint32_t cb1[kSub], cb2[kSub];
            // Epilogue. kFast: rows keep value-only top-2s of the raw accumulator bits (0x4B000000 | d2, monotone in
            // d2), columns keep packed keys with the row index (one v_lshl_or), both inserted two at a time. Partial
            // tiles (last row tile / column chunk) take a separate masked copy so the full-tile path has no selects.
            auto epilogue = [&](auto masked) {
                constexpr bool kMasked = decltype(masked)::value;
#pragma unroll
                for (int sub = 0; sub < kSub; ++sub) cb1[sub] = cb2[sub] = kNoKey;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const uint32_t rowbase = (uint32_t)(r0w + 32 * t + 4 * half);
#pragma unroll
                    for (int g0 = 0; g0 < 16; g0 += 2) {  // two rows at a time: column keys go in as a pair
                        uint32_t ck[kSub][2];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int g = g0 + h;
                            const uint32_t grow = rowbase + (uint32_t)((g & 3) + 8 * (g >> 2));
                            uint32_t rv[kSub];
#pragma unroll
                            for (int sub = 0; sub < kSub; ++sub) {
                                const uint32_t gcol = (uint32_t)(c0 + sub * kChunk + lrow);
                                const uint32_t bits = __float_as_uint(acc[sub][t][g]);
                                if constexpr (kFast) {
                                    rv[sub] = bits;
                                    ck[sub][h] = lshl_or(bits, (uint32_t)ib, grow);
                                } else {
                                    const uint32_t d2 = umin((uint32_t)acc[sub][t][g] - (1u << 23), dsat);
                                    rv[sub] = (d2 << ib) | gcol;
                                    ck[sub][h] = (d2 << ib) | grow;
                                }
                                if constexpr (kMasked) {
                                    if ((int)gcol >= n2) rv[sub] = kNoKey;
                                    if ((int)grow >= n1) ck[sub][h] = kNoKey;
                                }
                            }
                            top2_insert2(rb1[t][g], rb2[t][g], rv[0], rv[1]);
                        }
#pragma unroll
                        for (int sub = 0; sub < kSub; ++sub) top2_insert2(cb1[sub], cb2[sub], ck[sub][0], ck[sub][1]);
                    }
                }
            };
            static_assert(kSub == 2, "paired row insert takes exactly two chunks");
            if (cols_partial || rows_partial1)
                epilogue(std::true_type{});
            else
                epilogue(std::false_type{});
            // combine the two half-waves (same column, rows +0/+4) and publish the wave's column partials
#pragma unroll
            for (int sub = 0; sub < kSub; ++sub) {
                uint32_t a1 = cb1[sub], a2 = cb2[sub];
                const uint32_t o1 = __shfl_xor(a1, 32), o2 = __shfl_xor(a2, 32);
                top2_merge(a1, a2, o1, o2);
                partial[((buf * kWaves + wave) * kSuper + sub * kChunk + lrow) * 2 + half] = half ? a2 : a1;
            }
            if (sc > 0) merge_partials(sc - 1, buf ^ 1);
            __syncthreads();  // next super-chunk landed (vmcnt(0)); partials of this one visible
        }
        merge_partials(nsup - 1, (nsup - 1) & 1);

        // reduce each row's top-2 across the 32 lanes of its half-wave and store it
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                uint32_t b1 = rb1[t][g], b2 = rb2[t][g];
#pragma unroll
                for (int m = 1; m < 32; m <<= 1) {
                    const uint32_t o1 = __shfl_xor(b1, m), o2 = __shfl_xor(b2, m);
                    top2_merge(b1, b2, o1, o2);
                }
                const int grow = r0w + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
                if (lrow == g && grow < n1) rres[grow] = make_uint2(b1, b2);
            }
        }
        __syncthreads();
    }
    for (int c = tid; c < n2; c += kThreads) cres[c] = colstate[c];
}

// ---------------------------------------------------------------------------------------------
// Exact fp32 path: one thread per query row, sequential-k sums (FMA contraction disabled for this
// translation unit), top-2 on sqrtf distance with OpenCV's strict '<' insertion.
// Result per row: (d1, d2) float distances and j1.
// ---------------------------------------------------------------------------------------------
struct ExactTop2 {
    float d1, d2;
    int j1, pad;
};

__global__ void exact_top2_kernel(const float* __restrict__ desc, const int* __restrict__ counts, int kmax, int dim,
                                  const int* __restrict__ pairs, int swap, ExactTop2* __restrict__ out) {
#pragma clang fp contract(off)  // sequential, unfused (a-b)^2 sums: the oracle's arithmetic (oracle/twoway.c)
    const int p = blockIdx.y;
    const int iq = pairs[2 * p + (swap ? 1 : 0)], it = pairs[2 * p + (swap ? 0 : 1)];
    const int nq = counts[iq], nt = counts[it];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const float* q = desc + ((size_t)iq * kmax + i) * dim;
    const float* T = desc + (size_t)it * kmax * dim;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int j1 = -1;
    for (int j = 0; j < nt; ++j) {
        const float* t = T + (size_t)j * dim;
        float acc = 0.f;
        for (int k = 0; k < dim; ++k) {
            const float df = q[k] - t[k];
            acc = acc + df * df;  // unfused: contract(off) above
        }
        const float d = sqrt_cr(acc);
        if (d < b2) {
            if (d < b1) {
                b2 = b1;
                b1 = d;
                j1 = j;
            } else {
                b2 = d;
            }
        }
    }
    out[(size_t)p * kmax + i] = ExactTop2{b1, b2, j1, 0};
}

// ---------------------------------------------------------------------------------------------
// Finalize: ratio test + mutual check + compaction + bitonic sort by (distance, i1).
// ---------------------------------------------------------------------------------------------
constexpr int kFinThreads = 256;

__device__ __forceinline__ bool ratio_ok(float d1, float d2, double ratio) {
    if (ratio < 0.0) return true;
    return (double)d1 <= ratio * (double)d2;  // twoway_matcher.py:137 (Python float compare)
}

// Exact top-2 of one query row against nt train rows, computed by the whole block (rare path: only for
// rows/columns whose packed keys saturated). Same arithmetic as exact_top2_kernel.
__device__ void block_exact_top2(const float* __restrict__ q, const float* __restrict__ T, int nt, int dim,
                                 float* red_d, int* red_j, float& d1, float& d2, int& j1) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int bj = -1;
    for (int j = tid; j < nt; j += kFinThreads) {  // each thread scans its own j in increasing order
        const float* t = T + (size_t)j * dim;
        float acc = 0.f;
        for (int k = 0; k < dim; ++k) {
            const float df = q[k] - t[k];
            acc = acc + df * df;  // unfused: contract(off) above
        }
        const float d = sqrt_cr(acc);
        if (d < b2) {
            if (d < b1) { b2 = b1; b1 = d; bj = j; } else { b2 = d; }
        }
    }
    // lexicographic (distance, index) merge across threads: thread t's second best has index > its best
    red_d[2 * tid] = b1;
    red_d[2 * tid + 1] = b2;
    red_j[tid] = bj;
    __syncthreads();
    if (tid == 0) {
        // best = lexicographic min of (b1, j) over threads; second distance = min(best thread's b2,
        // every other thread's b1) — its index never matters, only its distance (ratio test)
        int bt = -1;
        for (int t = 0; t < kFinThreads; ++t) {
            const int cj = red_j[t];
            if (cj < 0) continue;
            if (bt < 0 || red_d[2 * t] < red_d[2 * bt] || (red_d[2 * t] == red_d[2 * bt] && cj < red_j[bt])) bt = t;
        }
        float m1 = __builtin_inff(), m2 = __builtin_inff();
        int mj = -1;
        if (bt >= 0) {
            m1 = red_d[2 * bt];
            mj = red_j[bt];
            m2 = red_d[2 * bt + 1];
            for (int t = 0; t < kFinThreads; ++t)
                if (t != bt && red_j[t] >= 0) m2 = fminf(m2, red_d[2 * t]);
        }
        red_d[0] = m1;
        red_d[1] = m2;
        red_j[0] = mj;
    }
    __syncthreads();
    d1 = red_d[0];
    d2 = red_d[1];
    j1 = red_j[0];
    __syncthreads();
}

// Per-keypoint top-2 encodings consumed by finalize. side1 = image i1's keypoints (best in i2), side2 = image i2's.
//   kResExact:  ExactTop2 on both sides (exact fp32 path)
//   kResKeys:   packed (d2 << ib | index) keys on both sides (ib = 13)
//   kResValues: side1 packed keys, side2 raw accumulator bits 0x4B000000 | d2 without an index (ib <= 12)
constexpr int kResExact = 0, kResKeys = 1, kResValues = 2;

template <int kRes>
__global__ __launch_bounds__(kFinThreads) void match_finalize_kernel(const void* __restrict__ rowres_v,
                                                                     const void* __restrict__ colres_v,
                                                                     const float* __restrict__ desc,
                                                                     const int* __restrict__ counts,
                                                                     const int* __restrict__ pairs, int kmax,
                                                                     int dim, int ib, double ratio,
                                                                     uint32_t* __restrict__ out_idx,
                                                                     int* __restrict__ out_count) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int* hdr = (int*)smem;                                           // [0] matches, [1] redo rows
    float* red_d = (float*)(smem + 16);                               // [2*kFinThreads]
    int* red_j = (int*)(smem + 16 + 8 * kFinThreads);                 // [kFinThreads]
    int* redo = (int*)(smem + 16 + 12 * kFinThreads);                 // [kmax]
    unsigned long long* keys =
        (unsigned long long*)(smem + 16 + 12 * kFinThreads + gtsfm_align_up((size_t)kmax * 4, 16));
    const int p = blockIdx.x;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const int n1 = counts[i1], n2 = counts[i2];
    const int tid = threadIdx.x;
    if (tid == 0) { hdr[0] = 0; hdr[1] = 0; }
    __syncthreads();
    const uint32_t imask = (1u << ib) - 1u, dsat = (1u << (32 - ib)) - 1u;
    auto push = [&](int i, int j, float d1r) {
        const int slot = atomicAdd(&hdr[0], 1);
        keys[slot] = ((unsigned long long)__float_as_uint(d1r) << 32) | ((unsigned long long)i << 16) | (uint32_t)j;
    };

    constexpr bool kPacked = kRes == kResKeys;
    const float* D1 = desc + (size_t)i1 * kmax * dim;
    const float* D2 = desc + (size_t)i2 * kmax * dim;
    if constexpr (kRes == kResValues) {
        // side2 carries distances only. Keypoint i's nearest j (from its key) is mutual iff j's best distance equals
        // d(i, j) and j has no tie at its minimum (then i, reaching that minimum, is j's unique nearest). A tied j
        // whose own ratio test can pass is recomputed exactly below; one that cannot is in no match.
        constexpr uint32_t kMant = 0x7FFFFFu;
        const uint2* s1 = (const uint2*)rowres_v + (size_t)p * kmax;
        const uint2* s2 = (const uint2*)colres_v + (size_t)p * kmax;
        for (int j = tid; j < n2 && n1 > 0; j += kFinThreads) {
            const uint2 v = s2[j];
            if (v.x == kNoKey || v.x != v.y) continue;
            const float d = sqrt_cr((float)(v.x & kMant));
            if (ratio_ok(d, d, ratio)) redo[atomicAdd(&hdr[1], 1)] = j;
        }
        for (int i = tid; i < n1 && n2 > 0; i += kFinThreads) {
            const uint2 k = s1[i];
            if (k.x == kNoKey) continue;
            const int j = (int)(k.x & imask);
            const uint32_t d = k.x >> ib;
            const uint2 v = s2[j];
            if (v.x == v.y || (v.x & kMant) != d) continue;  // j tied (redo) or j's nearest is not i
            const float d1r = sqrt_cr((float)d);
            const float d2r = (k.y == kNoKey) ? __builtin_inff() : sqrt_cr((float)(k.y >> ib));
            const float d2c = (v.y == kNoKey) ? __builtin_inff() : sqrt_cr((float)(v.y & kMant));
            if (ratio_ok(d1r, d2r, ratio) && ratio_ok(d1r, d2c, ratio)) push(i, j, d1r);
        }
        __syncthreads();
        const int nredo = hdr[1];
        for (int r = 0; r < nredo; ++r) {
            const int j = redo[r];
            float d1r, d2r, d1c, d2c;
            int i, jj;
            block_exact_top2(D2 + (size_t)j * dim, D1, n1, dim, red_d, red_j, d1c, d2c, i);
            if (i < 0) continue;
            block_exact_top2(D1 + (size_t)i * dim, D2, n2, dim, red_d, red_j, d1r, d2r, jj);
            if (tid == 0 && jj == j && ratio_ok(d1r, d2r, ratio) && ratio_ok(d1c, d2c, ratio)) push(i, j, d1r);
            __syncthreads();
        }
    }
    for (int i = tid; i < n1 && n2 > 0 && kRes != kResValues; i += kFinThreads) {
        float d1r, d2r, d1c, d2c;
        int j, ic;
        if (kPacked) {
            const uint2 r = ((const uint2*)rowres_v)[(size_t)p * kmax + i];
            if (r.x == kNoKey) continue;
            j = (int)(r.x & imask);
            const uint2 c = ((const uint2*)colres_v)[(size_t)p * kmax + j];
            const bool sat = (r.x >> ib) == dsat || (r.y != kNoKey && (r.y >> ib) == dsat) || (c.x >> ib) == dsat ||
                             (c.y != kNoKey && (c.y >> ib) == dsat);
            if (sat) {
                redo[atomicAdd(&hdr[1], 1)] = i;
                continue;
            }
            d1r = sqrt_cr((float)(r.x >> ib));
            d2r = (r.y == kNoKey) ? __builtin_inff() : sqrt_cr((float)(r.y >> ib));
            ic = (int)(c.x & imask);
            d1c = sqrt_cr((float)(c.x >> ib));
            d2c = (c.y == kNoKey) ? __builtin_inff() : sqrt_cr((float)(c.y >> ib));
        } else {
            const ExactTop2 r = ((const ExactTop2*)rowres_v)[(size_t)p * kmax + i];
            if (r.j1 < 0) continue;
            j = r.j1;
            d1r = r.d1;
            d2r = r.d2;
            const ExactTop2 c = ((const ExactTop2*)colres_v)[(size_t)p * kmax + j];
            ic = c.j1;
            d1c = c.d1;
            d2c = c.d2;
        }
        if (ic == i && ratio_ok(d1r, d2r, ratio) && ratio_ok(d1c, d2c, ratio)) push(i, j, d1r);
    }
    __syncthreads();
    if (kPacked) {  // rare: saturated keys -> exact block-wide recomputation of that row and its column
        const int nredo = hdr[1];
        for (int r = 0; r < nredo; ++r) {
            const int i = redo[r];
            float d1r, d2r, d1c, d2c;
            int j, ic;
            block_exact_top2(D1 + (size_t)i * dim, D2, n2, dim, red_d, red_j, d1r, d2r, j);
            if (j < 0) continue;
            block_exact_top2(D2 + (size_t)j * dim, D1, n1, dim, red_d, red_j, d1c, d2c, ic);
            if (tid == 0 && ic == i && ratio_ok(d1r, d2r, ratio) && ratio_ok(d1c, d2c, ratio)) push(i, j, d1r);
            __syncthreads();
        }
    }
    __syncthreads();
    const int m = hdr[0];
    int np2 = 1;
    while (np2 < m) np2 <<= 1;
    for (int k = m + tid; k < np2; k += kFinThreads) keys[k] = ~0ull;
    __syncthreads();
    // bitonic sort (ascending) of np2 keys: (distance bits, i1, i2) == the reference's stable sort order
    for (int size = 2; size <= np2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int k = tid; k < np2; k += kFinThreads) {
                const int o = k ^ stride;
                if (o > k) {
                    const unsigned long long a = keys[k], b = keys[o];
                    const bool up = ((k & size) == 0);
                    if ((a > b) == up) {
                        keys[k] = b;
                        keys[o] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    uint32_t* dst = out_idx + (size_t)p * kmax * 2;
    for (int k = tid; k < m; k += kFinThreads) {
        const unsigned long long key = keys[k];
        dst[2 * k] = (uint32_t)((key >> 16) & 0xFFFFu);
        dst[2 * k + 1] = (uint32_t)(key & 0xFFFFu);
    }
    if (tid == 0) out_count[p] = m;
}

inline int next_pow2(int x) {
    int n = 1;
    while (n < x) n <<= 1;
    return n;
}

// K width of the packed forms: dim + 5 folded columns, rounded up to an instantiated MFMA depth (NK in {2, 5, 9})
inline int pack_da(int dim) {
    const int nk = (dim + 5 + 15) / 16;
    return 16 * (nk <= 2 ? 2 : nk <= 5 ? 5 : nk <= 9 ? 9 : nk);
}
inline int pack_kpad(int kmax) { return (int)gtsfm_align_up((size_t)kmax, kRowsPerPass); }

template <int NK, bool kFast>
int launch_mnn_t(const _Float16* a_form, const _Float16* b_form, const int* counts, const int* pairs, int n_pairs,
                 int kpad, int kmax, int ib, uint2* rowres, uint2* colres, hipStream_t stream) {
    using Cfg = MnnCfg<NK>;
    const size_t lds = 2 * kSub * Cfg::kBufBytes + 2 * kWaves * kSuper * 2 * sizeof(uint32_t) +
                       (size_t)kmax * sizeof(uint2);
    if (lds > 160 * 1024) return GTSFM_ERR_ARG;
    if (lds > 65536)
        GTSFM_CHECK_HIP(hipFuncSetAttribute((const void*)mnn_mfma_kernel<NK, kFast>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((mnn_mfma_kernel<NK, kFast>), dim3(n_pairs), dim3(kThreads), lds, stream, a_form, b_form,
                       counts, pairs, n_pairs, kpad, kmax, ib, rowres, colres);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

template <int NK>
int launch_mnn(const _Float16* a_form, const _Float16* b_form, const int* counts, const int* pairs, int n_pairs,
               int kpad, int kmax, int ib, uint2* rowres, uint2* colres, hipStream_t stream) {
    if (ib <= 12)
        return launch_mnn_t<NK, true>(a_form, b_form, counts, pairs, n_pairs, kpad, kmax, ib, rowres, colres, stream);
    return launch_mnn_t<NK, false>(a_form, b_form, counts, pairs, n_pairs, kpad, kmax, ib, rowres, colres, stream);
}

// side1 / side2: per-keypoint top-2 of image i1 / image i2 of each pair (encoding kRes)
template <int kRes>
int launch_finalize(const void* side1, const void* side2, const float* desc, const int* counts, const int* pairs,
                    int n_pairs, int kmax, int dim, int ib, double ratio, uint32_t* out_idx, int* out_count,
                    hipStream_t stream) {
    const size_t lds = 16 + 12 * kFinThreads + gtsfm_align_up((size_t)kmax * 4, 16) +
                       (size_t)next_pow2(kmax) * sizeof(unsigned long long);
    if (lds > 160 * 1024) return GTSFM_ERR_ARG;
    if (lds > 65536)
        GTSFM_CHECK_HIP(hipFuncSetAttribute((const void*)match_finalize_kernel<kRes>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(match_finalize_kernel<kRes>, dim3(n_pairs), dim3(kFinThreads), lds, stream, side1, side2,
                       desc, counts, pairs, kmax, dim, ib, ratio, out_idx, out_count);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

hipEvent_t g_mnn_events[2] = {nullptr, nullptr};  // gtsfm_match_set_kernel_events

// ---------------------------------------------------------------------------------------------
// Float-descriptor path (GTSFM_MATCH_F16_RERANK, e.g. SuperPoint's 256-D unit vectors). An fp16 MFMA distance GEMM
// shortlists each keypoint's kFlCand nearest candidates on the other side (approximate keys |b|^2 - 2 a.b, fp32
// accumulation); fl_rerank_kernel recomputes the shortlist with exact_top2_kernel's arithmetic, in index order, and
// certifies it: with eps a bound on |approx - exact| squared distance (fp16 rounding of both operands, fp32
// accumulation and norms), every keypoint outside the shortlist has approx key >= the shortlist's last, so once
// (last + |a|^2) - eps clears the shortlist's exact second distance by a relative margin no outside keypoint can enter
// the top 2 or tie it. Rows without the certificate (or on an image with values outside the fp16 range) are rescanned
// exactly. The (d1, d2, j1) per keypoint, and so the matches, are bit-identical to GTSFM_MATCH_EXACT_F32.
// ---------------------------------------------------------------------------------------------
constexpr int kFlCand = 8;
constexpr int kFlRows = 64;   // train rows per LDS chunk (two 32-row MFMA tiles)
constexpr int kFlQ = 128;     // queries per workgroup: 4 waves x 32
constexpr int kFlMaxDim = 256;

__host__ __device__ inline int fl_dpad(int dim) { return dim <= 64 ? 64 : dim <= 128 ? 128 : 256; }
__host__ __device__ inline int fl_kpad(int kmax) { return (kmax + kFlQ - 1) / kFlQ * kFlQ; }

// One wave per descriptor row: fp16 form (zero-padded to dpad), fp32 squared norm (+inf for padding rows), the
// image's largest norm and an "unsafe" flag for values fp16 cannot hold within the error bound.
__global__ __launch_bounds__(256) void fl_prep_kernel(const float* __restrict__ desc, const int* __restrict__ counts,
                                                      int kmax, int dim, int kpad, int dpad,
                                                      _Float16* __restrict__ form, float* __restrict__ norm2,
                                                      unsigned* __restrict__ img_maxnorm, unsigned* __restrict__ img_unsafe) {
    const int img = blockIdx.y, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = counts[img];
    const bool valid = row < n && row < kmax;
    const float* d = desc + ((size_t)img * kmax + row) * dim;
    _Float16* f = form + ((size_t)img * kpad + row) * dpad;
    float sq = 0.f;
    bool bad = false;
    for (int k = lane; k < dpad; k += 64) {
        const float v = (valid && k < dim) ? d[k] : 0.f;
        bad |= !(fabsf(v) <= 60000.f);
        sq = fmaf(v, v, sq);
        f[k] = (_Float16)v;
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) sq += __shfl_xor(sq, m);
    const bool any_bad = __ballot(bad) != 0ull;
    if (lane == 0) {
        norm2[(size_t)img * kpad + row] = valid ? sq : __builtin_inff();
        if (valid) {
            atomicMax(&img_maxnorm[img], __float_as_uint(sqrtf(sq)));
            if (any_bad || !(sq <= 3.0e38f)) atomicOr(&img_unsafe[img], 1u);
        }
    }
}

typedef _Float16 fl_half8 __attribute__((ext_vector_type(8)));
typedef unsigned fl_u32x4 __attribute__((ext_vector_type(4)));
typedef float fl_float16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void fl_insert(float x, int j, float (&v)[kFlCand], int (&id)[kFlCand]) {
    // v sorted ascending and x < v[kFlCand - 1]: branch-free insertion (each slot takes its left neighbour, x or itself)
#pragma unroll
    for (int m = kFlCand - 1; m > 0; --m) {
        const bool sh = x < v[m - 1], here = x < v[m];
        v[m] = sh ? v[m - 1] : (here ? x : v[m]);
        id[m] = sh ? id[m - 1] : (here ? j : id[m]);
    }
    if (x < v[0]) { v[0] = x; id[0] = j; }
}

template <int NV, int DP>
__device__ __forceinline__ void fl_fetch(fl_u32x4 (&pre)[NV], float& pn, const _Float16* __restrict__ tbase,
                                         const float* __restrict__ nbase, int c0, int tid) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int vid = tid + 256 * k, row = vid / (DP / 8), c8 = vid % (DP / 8);
        pre[k] = *(const fl_u32x4*)(tbase + (size_t)(c0 + row) * DP + 8 * c8);
    }
    if (tid < kFlRows) pn = nbase[c0 + tid];
}

template <int NV, int DP>
__device__ __forceinline__ void fl_stash(const fl_u32x4 (&pre)[NV], float pn, _Float16* tl, float* nbl, int buf, int tid) {
    constexpr int RS = DP + 8;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int vid = tid + 256 * k, row = vid / (DP / 8), c8 = vid % (DP / 8);
        *(fl_u32x4*)(tl + buf * kFlRows * RS + row * RS + 8 * c8) = pre[k];
    }
    if (tid < kFlRows) nbl[buf * kFlRows + tid] = pn;
}

// grid (kpad / 128, P, 2 sides). Queries (image pairs[2p + side]) sit on the MFMA's N axis: lane l keeps the
// shortlist of query l & 31 over the train rows of its half (l >> 5) of every 32-row tile; the halves merge at the end.
// Train rows stream through LDS in double-buffered 64-row chunks (row stride dpad + 8 halfs: conflict-free b128 reads).
template <int NS>
__global__ __launch_bounds__(256, 2) void fl_shortlist_kernel(const _Float16* __restrict__ form,
                                                              const float* __restrict__ norm2,
                                                              const int* __restrict__ counts,
                                                              const int* __restrict__ pairs, int n_pairs, int kpad,
                                                              int kmax, int* __restrict__ cand,
                                                              float* __restrict__ tkey) {
    constexpr int DP = NS * 16, RS = DP + 8, NV = DP / 32;  // NV: 16-byte loads per thread per chunk
    extern __shared__ __attribute__((aligned(16))) unsigned char fl_smem[];
    _Float16* tl = (_Float16*)fl_smem;                                  // [2][kFlRows * RS]
    float* nbl = (float*)(fl_smem + 2 * kFlRows * RS * sizeof(_Float16));  // [2][kFlRows]
    const int p = blockIdx.y, side = blockIdx.z, tid = threadIdx.x, w = tid >> 6, l = tid & 63, h = l >> 5;
    const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
    const int nq = counts[iq], nt = counts[it];
    const int q0 = blockIdx.x * kFlQ;
    if (q0 >= nq) return;
    const int qn = q0 + w * 32 + (l & 31);
    fl_half8 bq[NS];
    const _Float16* qrow = form + ((size_t)iq * kpad + qn) * DP + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) bq[s] = *(const fl_half8*)(qrow + 16 * s);
    float v[kFlCand];
    int id[kFlCand];
#pragma unroll
    for (int c = 0; c < kFlCand; ++c) { v[c] = __builtin_inff(); id[c] = -1; }
    const _Float16* tbase = form + (size_t)it * kpad * DP;
    const float* nbase = norm2 + (size_t)it * kpad;
    fl_u32x4 pre[NV];
    float pn = 0.f;
    const int n_chunks = (nt + kFlRows - 1) / kFlRows;
    if (n_chunks > 0) {
        fl_fetch<NV, DP>(pre, pn, tbase, nbase, 0, tid);
        fl_stash<NV, DP>(pre, pn, tl, nbl, 0, tid);
    }
    __syncthreads();
    for (int c = 0; c < n_chunks; ++c) {
        const int buf = c & 1, c0 = c * kFlRows;
        if (c + 1 < n_chunks) {
            fl_fetch<NV, DP>(pre, pn, tbase, nbase, c0 + kFlRows, tid);
        }
        const _Float16* tb = tl + buf * kFlRows * RS;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            fl_float16 acc = {};
            const _Float16* arow = tb + (t * 32 + (l & 31)) * RS + 8 * h;
#pragma unroll
            for (int s = 0; s < NS; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const fl_half8*)(arow + 16 * s), bq[s], acc, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 nb = *(const float4*)(nbl + buf * kFlRows + t * 32 + 8 * g + 4 * h);
                const float k0 = fmaf(-2.f, acc[4 * g], nb.x), k1 = fmaf(-2.f, acc[4 * g + 1], nb.y);
                const float k2 = fmaf(-2.f, acc[4 * g + 2], nb.z), k3 = fmaf(-2.f, acc[4 * g + 3], nb.w);
                const float kmin = fminf(fminf(k0, k1), fminf(k2, k3));
                if (__ballot(kmin < v[kFlCand - 1]) == 0ull) continue;
                const int jb = c0 + t * 32 + 8 * g + 4 * h;
                if (k0 < v[kFlCand - 1]) fl_insert(k0, jb, v, id);
                if (k1 < v[kFlCand - 1]) fl_insert(k1, jb + 1, v, id);
                if (k2 < v[kFlCand - 1]) fl_insert(k2, jb + 2, v, id);
                if (k3 < v[kFlCand - 1]) fl_insert(k3, jb + 3, v, id);
            }
        }
        if (c + 1 < n_chunks) {
            fl_stash<NV, DP>(pre, pn, tl, nbl, buf ^ 1, tid);
        }
        __syncthreads();
    }
    // merge the two halves of each query's shortlist
#pragma unroll
    for (int c = 0; c < kFlCand; ++c) {
        const float pv = __shfl_xor(v[c], 32);
        const int pj = __shfl_xor(id[c], 32);
        if (h == 0 && pv < v[kFlCand - 1]) fl_insert(pv, pj, v, id);
    }
    if (h == 0 && qn < nq) {
        const size_t o = ((size_t)side * n_pairs + p) * kmax + qn;
#pragma unroll
        for (int c = 0; c < kFlCand; ++c) cand[o * kFlCand + c] = id[c];
        tkey[o] = v[kFlCand - 1];
    }
}

// grid (kpad / 32, P, 2 sides), 256 threads: thread (r, c) = (tid / 8, tid % 8) sums keypoint i0 + r's distance to
// its c-th shortlisted candidate straight from HBM/L2 (float4 row walks, many loads in flight), sequentially and
// unfused: exact_top2_kernel's arithmetic. Then one thread per keypoint scans its 8 candidates in index order (the
// exact scan's b1 / j1 / b2 updates) and checks the certificate; uncertified keypoints go to `redo`.
constexpr int kFlRerankRows = 256 / kFlCand;
__global__ __launch_bounds__(256) void fl_rerank_kernel(const float* __restrict__ desc, const int* __restrict__ counts,
                                                        int kmax, int dim, const int* __restrict__ pairs, int n_pairs,
                                                        int kpad, const float* __restrict__ norm2,
                                                        const unsigned* __restrict__ img_maxnorm,
                                                        const unsigned* __restrict__ img_unsafe,
                                                        const int* __restrict__ cand, const float* __restrict__ tkey,
                                                        ExactTop2* __restrict__ rowres, ExactTop2* __restrict__ colres,
                                                        int* __restrict__ redo_count, int4* __restrict__ redo) {
#pragma clang fp contract(off)
    __shared__ float sacc[kFlRerankRows][kFlCand];
    __shared__ int sj[kFlRerankRows][kFlCand];
    const int p = blockIdx.y, side = blockIdx.z, tid = threadIdx.x;
    const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
    const int nq = counts[iq], nt = counts[it];
    const int i0 = blockIdx.x * kFlRerankRows;
    if (i0 >= nq) return;
    const int r = tid / kFlCand, c = tid % kFlCand, i = i0 + r;
    int j = -1;
    float acc = __builtin_inff();
    if (i < nq) {
        j = cand[(((size_t)side * n_pairs + p) * kmax + i) * kFlCand + c];
        if (j >= nt) j = -1;
        if (j >= 0) {
            const float* q = desc + ((size_t)iq * kmax + i) * dim;
            const float* t = desc + ((size_t)it * kmax + j) * dim;
            acc = 0.f;
            if ((dim & 3) == 0) {
                const float4* q4 = (const float4*)q;
                const float4* t4 = (const float4*)t;
#pragma unroll 8
                for (int k = 0; k < dim / 4; ++k) {
                    const float4 a = q4[k], b = t4[k];
                    const float e0 = a.x - b.x, e1 = a.y - b.y, e2 = a.z - b.z, e3 = a.w - b.w;
                    acc = acc + e0 * e0;  // unfused, in index order: contract(off) above
                    acc = acc + e1 * e1;
                    acc = acc + e2 * e2;
                    acc = acc + e3 * e3;
                }
            } else {
                for (int k = 0; k < dim; ++k) {
                    const float df = q[k] - t[k];
                    acc = acc + df * df;
                }
            }
        }
    }
    sacc[r][c] = acc;
    sj[r][c] = j;
    __syncthreads();
    if (tid >= kFlRerankRows) return;
    const int ii = i0 + tid;
    if (ii >= nq) return;
    // the shortlist in index order (insertion sort of 8 (j, acc) records; -1 = empty goes last)
    int js[kFlCand];
    float as[kFlCand];
#pragma unroll
    for (int m = 0; m < kFlCand; ++m) { js[m] = sj[tid][m]; as[m] = sacc[tid][m]; }
#pragma unroll
    for (int a = 0; a < kFlCand; ++a)
#pragma unroll
        for (int b = 0; b + 1 < kFlCand - a; ++b)
            if ((unsigned)js[b] > (unsigned)js[b + 1]) {
                const int x = js[b]; js[b] = js[b + 1]; js[b + 1] = x;
                const float y = as[b]; as[b] = as[b + 1]; as[b + 1] = y;
            }
    float b1 = __builtin_inff(), b2 = __builtin_inff(), a1 = __builtin_inff(), a2 = __builtin_inff();
    int j1 = -1;
#pragma unroll
    for (int m = 0; m < kFlCand; ++m) {
        if (js[m] < 0) continue;
        const float d = sqrt_cr(as[m]);
        if (d < b2) {
            if (d < b1) { b2 = b1; a2 = a1; b1 = d; a1 = as[m]; j1 = js[m]; }
            else { b2 = d; a2 = as[m]; }
        }
    }
    bool certified = nt <= kFlCand;
    if (!certified && img_unsafe[iq] == 0u && img_unsafe[it] == 0u) {
        const float na = norm2[(size_t)iq * kpad + ii];
        const float an = sqrtf(na), bn = __uint_as_float(img_maxnorm[it]);
        const float u = 1.f / 2048.f, eta = 1.f / 33554432.f, D = (float)dim;
        const float e_dot = (2.f * u + u * u + D * 1.01f / 16777216.f) * an * bn + eta * sqrtf(D) * (an + bn) +
                            D * eta * eta;
        const float eps = 1.5f * (2.f * e_dot + (D + 4.f) * 2.f / 16777216.f * (na + bn * bn));
        certified = (na + tkey[((size_t)side * n_pairs + p) * kmax + ii]) - eps > a2 * (1.f + 1e-4f) + eps;
    }
    if (!certified) redo[atomicAdd(redo_count, 1)] = make_int4(side, p, ii, 0);
    (side ? colres : rowres)[(size_t)p * kmax + ii] = ExactTop2{b1, b2, j1, certified ? 0 : 1};
}

// Exact rescan of the uncertified keypoints: one 256-thread block per keypoint (block_exact_top2).
__global__ __launch_bounds__(kFinThreads) void fl_rescan_kernel(const float* __restrict__ desc,
                                                                const int* __restrict__ counts, int kmax, int dim,
                                                                const int* __restrict__ pairs,
                                                                const int* __restrict__ redo_count,
                                                                const int4* __restrict__ redo,
                                                                ExactTop2* __restrict__ rowres,
                                                                ExactTop2* __restrict__ colres) {
    __shared__ float red_d[2 * kFinThreads];
    __shared__ int red_j[kFinThreads];
    const int n = *redo_count;
    for (int e = blockIdx.x; e < n; e += gridDim.x) {
        const int4 r = redo[e];
        const int side = r.x, p = r.y, i = r.z;
        const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
        float d1, d2;
        int j1;
        block_exact_top2(desc + ((size_t)iq * kmax + i) * dim, desc + (size_t)it * kmax * dim, counts[it], dim, red_d,
                         red_j, d1, d2, j1);
        if (threadIdx.x == 0) (side ? colres : rowres)[(size_t)p * kmax + i] = ExactTop2{d1, d2, j1, 1};
    }
}

size_t fl_layout(int n_img, int kmax, int dim, int n_pairs, size_t* off) {
    const int kpad = fl_kpad(kmax), dpad = fl_dpad(dim);
    size_t o = 0;
    off[0] = o; o += gtsfm_align_up((size_t)n_img * kpad * dpad * sizeof(_Float16), 256);  // form
    off[1] = o; o += gtsfm_align_up((size_t)n_img * kpad * sizeof(float), 256);             // norm2
    off[2] = o; o += gtsfm_align_up((size_t)2 * n_img * sizeof(unsigned), 256);             // maxnorm, unsafe
    off[3] = o; o += gtsfm_align_up((size_t)2 * n_pairs * kmax * kFlCand * sizeof(int), 256);  // cand
    off[4] = o; o += gtsfm_align_up((size_t)2 * n_pairs * kmax * sizeof(float), 256);       // tkey
    off[5] = o; o += gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);       // rowres
    off[6] = o; o += gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);       // colres
    off[7] = o; o += 256;                                                                     // redo count
    off[8] = o; o += gtsfm_align_up((size_t)2 * n_pairs * kmax * sizeof(int4), 256);        // redo list
    return o;
}

template <int NS>
int launch_fl_shortlist(const _Float16* form, const float* norm2, const int* counts, const int* pairs, int n_pairs,
                        int kpad, int kmax, int* cand, float* tkey, hipStream_t stream) {
    const size_t lds = 2 * kFlRows * (NS * 16 + 8) * sizeof(_Float16) + 2 * kFlRows * sizeof(float);
    GTSFM_CHECK_HIP(gtsfm_set_dynamic_lds((const void*)fl_shortlist_kernel<NS>, (int)lds));
    hipLaunchKernelGGL(fl_shortlist_kernel<NS>, dim3(kpad / kFlQ, n_pairs, 2), dim3(256), lds, stream, form, norm2,
                       counts, pairs, n_pairs, kpad, kmax, cand, tkey);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

int run_fl_match(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim, const int* d_pairs,
                 int n_pairs, double ratio, unsigned char* ws, uint32_t* d_out_idx, int* d_out_count,
                 hipStream_t stream) {
    size_t off[9];
    fl_layout(n_img, kmax, dim, n_pairs, off);
    const int kpad = fl_kpad(kmax), dpad = fl_dpad(dim);
    _Float16* form = (_Float16*)(ws + off[0]);
    float* norm2 = (float*)(ws + off[1]);
    unsigned* maxnorm = (unsigned*)(ws + off[2]);
    unsigned* unsafe = maxnorm + n_img;
    int* cand = (int*)(ws + off[3]);
    float* tkey = (float*)(ws + off[4]);
    ExactTop2* rowres = (ExactTop2*)(ws + off[5]);
    ExactTop2* colres = (ExactTop2*)(ws + off[6]);
    int* redo_count = (int*)(ws + off[7]);
    int4* redo = (int4*)(ws + off[8]);
    GTSFM_CHECK_HIP(hipMemsetAsync(maxnorm, 0, 2 * (size_t)n_img * sizeof(unsigned), stream));
    GTSFM_CHECK_HIP(hipMemsetAsync(redo_count, 0, sizeof(int), stream));
    hipLaunchKernelGGL(fl_prep_kernel, dim3(kpad / 4, n_img), dim3(256), 0, stream, d_desc, d_counts, kmax, dim, kpad,
                       dpad, form, norm2, maxnorm, unsafe);
    GTSFM_CHECK_HIP(hipGetLastError());
    int rc;
    if (g_mnn_events[0]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[0], stream));
    switch (dpad) {
        case 64: rc = launch_fl_shortlist<4>(form, norm2, d_counts, d_pairs, n_pairs, kpad, kmax, cand, tkey, stream); break;
        case 128: rc = launch_fl_shortlist<8>(form, norm2, d_counts, d_pairs, n_pairs, kpad, kmax, cand, tkey, stream); break;
        default: rc = launch_fl_shortlist<16>(form, norm2, d_counts, d_pairs, n_pairs, kpad, kmax, cand, tkey, stream); break;
    }
    if (rc != GTSFM_OK) return rc;
    if (g_mnn_events[1]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[1], stream));
    hipLaunchKernelGGL(fl_rerank_kernel, dim3((kmax + kFlRerankRows - 1) / kFlRerankRows, n_pairs, 2), dim3(256), 0,
                       stream, d_desc, d_counts, kmax, dim, d_pairs, n_pairs, kpad, norm2, maxnorm, unsafe, cand, tkey,
                       rowres, colres, redo_count, redo);
    GTSFM_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(fl_rescan_kernel, dim3(2048), dim3(kFinThreads), 0, stream, d_desc, d_counts, kmax, dim,
                       d_pairs, redo_count, redo, rowres, colres);
    GTSFM_CHECK_HIP(hipGetLastError());
    return launch_finalize<kResExact>(rowres, colres, d_desc, d_counts, d_pairs, n_pairs, kmax, dim, 0, ratio,
                                      d_out_idx, d_out_count, stream);
}



}  // namespace

extern "C" {

int gtsfm_match_set_kernel_events(void* hip_event_start, void* hip_event_stop) {
    g_mnn_events[0] = (hipEvent_t)hip_event_start;
    g_mnn_events[1] = (hipEvent_t)hip_event_stop;
    return GTSFM_OK;
}

size_t gtsfm_match_workspace_bytes(int n_img, int kmax, int dim, int n_pairs, int mode) {
    if (n_img <= 0 || kmax <= 0 || dim <= 0 || n_pairs < 0) return 0;
    if (mode == GTSFM_MATCH_INT_F16) {
        const size_t forms = 2 * gtsfm_align_up((size_t)n_img * pack_kpad(kmax) * pack_da(dim) * sizeof(_Float16), 256);
        const size_t res = 2 * gtsfm_align_up((size_t)n_pairs * kmax * sizeof(uint2), 256);
        return forms + res;
    }
    if (mode == GTSFM_MATCH_F16_RERANK && dim <= kFlMaxDim) {
        size_t off[9];
        return fl_layout(n_img, kmax, dim, n_pairs, off);
    }
    return 2 * gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);
}

int gtsfm_match_batched(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim, const int* d_pairs,
                        int n_pairs, double ratio, int mode, void* d_workspace, size_t workspace_bytes,
                        uint32_t* d_out_idx, int* d_out_count, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_desc || !d_counts || !d_pairs || !d_out_idx || !d_out_count || n_img <= 0 || kmax <= 0 || dim <= 0 ||
        n_pairs < 0 || kmax > kMaxKmax)
        return GTSFM_ERR_ARG;
    if (workspace_bytes < gtsfm_match_workspace_bytes(n_img, kmax, dim, n_pairs, mode)) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;

    if (mode == GTSFM_MATCH_INT_F16) {
        const int da = pack_da(dim), kpad = pack_kpad(kmax), nk = da / 16, ib = index_bits(kmax);
        if (dim > 139 || kmax > kMaxKmaxPacked) return GTSFM_ERR_ARG;
        const size_t form_bytes = gtsfm_align_up((size_t)n_img * kpad * da * sizeof(_Float16), 256);
        _Float16* a_form = (_Float16*)ws;
        _Float16* b_form = (_Float16*)(ws + form_bytes);
        const size_t res_bytes = gtsfm_align_up((size_t)n_pairs * kmax * sizeof(uint2), 256);
        uint2* rowres = (uint2*)(ws + 2 * form_bytes);
        uint2* colres = (uint2*)(ws + 2 * form_bytes + res_bytes);
        hipLaunchKernelGGL(pack_desc_kernel, dim3(kpad / 4, n_img), dim3(64, 4), 0, stream, d_desc, d_counts, kmax,
                           dim, kpad, da, a_form, b_form);
        GTSFM_CHECK_HIP(hipGetLastError());
        int rc;
        if (g_mnn_events[0]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[0], stream));
        switch (nk) {
            case 2: rc = launch_mnn<2>(a_form, b_form, d_counts, d_pairs, n_pairs, kpad, kmax, ib, rowres, colres, stream); break;
            case 5: rc = launch_mnn<5>(a_form, b_form, d_counts, d_pairs, n_pairs, kpad, kmax, ib, rowres, colres, stream); break;
            case 9: rc = launch_mnn<9>(a_form, b_form, d_counts, d_pairs, n_pairs, kpad, kmax, ib, rowres, colres, stream); break;
            default: return GTSFM_ERR_ARG;
        }
        if (rc != GTSFM_OK) return rc;
        if (g_mnn_events[1]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[1], stream));
        // the GEMM's columns are image i1's keypoints (side1), its rows image i2's (side2)
        if (ib <= 12)
            return launch_finalize<kResValues>(colres, rowres, d_desc, d_counts, d_pairs, n_pairs, kmax, dim, ib,
                                               ratio, d_out_idx, d_out_count, stream);
        return launch_finalize<kResKeys>(colres, rowres, d_desc, d_counts, d_pairs, n_pairs, kmax, dim, ib, ratio,
                                         d_out_idx, d_out_count, stream);
    }
    if (mode == GTSFM_MATCH_F16_RERANK && dim <= kFlMaxDim)
        return run_fl_match(d_desc, d_counts, n_img, kmax, dim, d_pairs, n_pairs, ratio, ws, d_out_idx, d_out_count,
                            stream);
    if (mode != GTSFM_MATCH_EXACT_F32 && mode != GTSFM_MATCH_F16_RERANK) return GTSFM_ERR_ARG;
    const size_t res_bytes = gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);
    ExactTop2* rowres = (ExactTop2*)ws;
    ExactTop2* colres = (ExactTop2*)(ws + res_bytes);
    const dim3 grid((kmax + 127) / 128, n_pairs);
    hipLaunchKernelGGL(exact_top2_kernel, grid, dim3(128), 0, stream, d_desc, d_counts, kmax, dim, d_pairs, 0, rowres);
    GTSFM_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(exact_top2_kernel, grid, dim3(128), 0, stream, d_desc, d_counts, kmax, dim, d_pairs, 1, colres);
    GTSFM_CHECK_HIP(hipGetLastError());
    return launch_finalize<kResExact>(rowres, colres, d_desc, d_counts, d_pairs, n_pairs, kmax, dim, 0, ratio,
                                      d_out_idx, d_out_count, stream);
}

}  // extern "C"
