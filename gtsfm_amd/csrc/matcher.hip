// Mutual-nearest-neighbour + ratio-test matcher for batches of image pairs (gfx950).
//
// Replaces gtsfm/frontend/matcher/twoway_matcher.py:42-144 (TwoWayMatcher.match): two one-way
// cv.BFMatcher(NORM_L2).knnMatch(k=2) passes (:102, :136), the ratio test `m1.distance <= r*m2.distance`
// (:137), the stable sort by distance (:141), the query->train dict (:142) and the mutual filter in
// 1->2 order (:117-120).
//
// Fast path (GTSFM_MATCH_INT_F16): one K1 x K2 distance GEMM per pair on fp16 MFMA (v_mfma_f32_32x32x16_f16), rows =
// image i1's keypoints (A operand, held in registers), columns = image i2's (B operand, streamed through LDS). The
// squared norms and a 4-bit row code are folded into 5 extra K columns, so every accumulator IS
//      d2(i, j) + (i mod 16) / 16
// exactly (pack_code_kernel). The epilogue never converts: rows keep a value-only top-2 of the raw accumulator bits
// (their code is constant per row, so the order is d2's), columns keep a value-only top-2 over each lane's 16 rows of
// a tile (the code breaks ties in row order) and turn it into packed keys d2 << ib | row only once per tile. Three
// VALU per distance in total (two v_min3/v_med3/v_min inserts per two values, one per direction).
// The K1 x K2 matrix is never written to HBM. In finalize, i2's keypoint j with nearest i (from its key) is mutual iff
// i's best distance equals d(i, j) and i has no tie at its minimum; tied i are recomputed exactly (rare).
// Lexicographic (d2, index) order == OpenCV's strict-'<' scan order, and for d2 < 2^22 ordering by d2 equals ordering
// by sqrtf(d2), so results are bit-identical to the oracle.
//
// Exact path (GTSFM_MATCH_EXACT_F32): float descriptors, per-row sequential fp32 sums (no FMA
// contraction), top-2 on sqrtf distances — the oracle's arithmetic, for tests and non-SIFT data.
//
// Both paths end in match_finalize_kernel: ratio test in double on float32 distances, mutual check,
// LDS compaction and a bitonic sort on (distance, i1) — the reference's output order.
#include "common.hpp"

#include <atomic>
#include <type_traits>

namespace {

// Packed key = (d2 << ib) | index with ib = ceil(log2(kmax)) (>= 11) index bits and 32-ib distance bits.
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

// Poison distance of padding keypoints (the saturated key field when ib <= 12; 2^20 > every real d2 otherwise).
// A real value never reaches it: |a|^2, |b|^2 < 2^19 bound d2 <= 2^20 - 2.
inline uint32_t code_poison(int ib) { return ib <= 12 ? (1u << (32 - ib)) - 1u : (1u << 20); }
constexpr uint32_t kRowPoisonD2 = (1u << 20) - 1u;  // trunc(row value) >= this: poison (no such neighbour)

// ---------------------------------------------------------------------------------------------
// Pack float descriptors into the two fp16 MFMA operand forms of the INT_F16 distance GEMM. K columns
// (da = dim + 5 rounded up to 16 NK):
//   A'_i = [a_i, |a_i|^2 mod 2048, |a_i|^2 div 2048, 1, 2048, (i mod 16) / 16, 0 ...]      (image in registers)
//   B'_j = [-2 b_j, 1, 2048, |b_j|^2 mod 2048, |b_j|^2 div 2048, 1, 0 ...]                  (image streamed)
// Exactness: descriptors are integers in [0, 1023] with |a|^2 < 2^19, so every product is an exact integer (or the
// code) and EVERY partial sum of any subset of a row-column's K products lies in [-2 a.b, |a|^2 + |b|^2 + 1), inside
// +-2^20 where fp32 still holds 4 fraction bits: no accumulation order (inside an MFMA or across k-steps) rounds.
// Padding keypoints (>= count) are poison rows: exactly P = code_poison(ib) against every real keypoint of the other
// image (their norm columns carry P, their dims are zero), so they never enter a real keypoint's top-2 unless it has
// fewer than two real neighbours, where they read as "no neighbour".
// A form: row-major [img][kpad][da] with rows permuted inside each 32-row tile: MFMA tile row r' = (g & 3) + 8 (g >> 2)
//   + 4 h holds keypoint 16 h + g, so output lane-half h holds the tile's keypoints 16 h .. 16 h + 15 in register
//   order g, and the 4-bit code i mod 16 is the keypoint's offset inside its lane's 16 rows.
// B form: fragment-major per 32-row chunk, [img][chunk][s][h][r][8] with k = 16 s + 8 h + e: the 64 16-B granules one
//   MFMA k-step reads (rows r = 0..31 x halves h) are one contiguous KiB, so a linear LDS-DMA copy of the chunk gives
//   conflict-free ds_read_b128 at lane * 16.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ size_t b_form_index(int img, int row, int k, int kpad, int da) {
    const size_t chunk = (size_t)img * kpad + (row & ~31);
    return chunk * da + (size_t)(k >> 4) * 512 + ((k >> 3) & 1) * 256 + (row & 31) * 8 + (k & 7);
}

__global__ void pack_code_kernel(const float* __restrict__ desc, const int* __restrict__ counts, int kmax, int dim,
                                 int kpad, int da, uint32_t poison, _Float16* __restrict__ a_form,
                                 _Float16* __restrict__ b_form) {
    const int img = blockIdx.y;
    const int row = blockIdx.x * blockDim.y + threadIdx.y;  // keypoint; one 64-lane wave per descriptor row
    if (row >= kpad) return;
    const int lane = threadIdx.x;
    const bool real = row < counts[img];
    const int j = row & 31, g = j & 15;
    const int apos = (row & ~31) + (g & 3) + 8 * (g >> 2) + 4 * (j >> 4);
    _Float16* ar = a_form + ((size_t)img * kpad + apos) * da;
    float sq = 0.f;
    const float* src = desc + ((size_t)img * kmax + row) * dim;
    for (int k = lane; k < dim; k += 64) {
        const float v = real ? src[k] : 0.f;
        sq += v * v;  // integer-valued: exact
        ar[k] = (_Float16)v;
        b_form[b_form_index(img, row, k, kpad, da)] = (_Float16)(-2.f * v);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
    const uint32_t nrm = real ? (uint32_t)sq : poison;
    const float lo = (float)(nrm & 2047u), hi = (float)(nrm >> 11);
    for (int k = dim + lane; k < da; k += 64) {
        const int e = k - dim;
        float av = 0.f, bv = 0.f;
        if (e == 0) { av = lo; bv = real ? 1.f : 0.f; }
        else if (e == 1) { av = hi; bv = real ? 2048.f : 0.f; }
        else if (e == 2) { av = real ? 1.f : 0.f; bv = lo; }
        else if (e == 3) { av = real ? 2048.f : 0.f; bv = hi; }
        else if (e == 4 && real) { av = (float)(row & 15) * 0.0625f; bv = 1.f; }
        ar[k] = (_Float16)av;
        b_form[b_form_index(img, row, k, kpad, da)] = (_Float16)bv;
    }
}

// ---------------------------------------------------------------------------------------------
// Fused distance GEMM + row/column top-2, ping-pong over two wave groups.
//
// A workgroup = 8 waves, two groups of 4; waves w and w + 4 share a SIMD. Each wave holds 64 rows (two 32-row MFMA
// tiles) of A in registers, so a pass covers 512 rows. B streams through a 2-deep LDS ring in units of 64 columns
// (18 KiB at K = 144, one LDS-DMA burst issued a phase ahead). Every unit is one MFMA segment M (36 MFMAs per wave)
// and one epilogue segment E (~230 VALU per wave); group 1 runs one phase behind group 0, so in every phase each
// SIMD has one wave in M beside one wave in E: the matrix pipe and the VALU issue of a SIMD are both busy.
//   phase 2k:     group 0 M(unit k)        group 1 E(unit k-1)      (LDS-DMA of unit k+1 issued)
//   phase 2k+1:   group 0 E(unit k)        group 1 M(unit k)
// A workgroup takes a GROUP of up to kMaxGroup pairs that share image i1 (the register operand): per pass it loads
// its A rows once and streams each pair's B image in turn (unit order: pass, slot, column unit). Groups are laid out
// by the caller (gtsfm_match_batched_grouped) so that the ~32 workgroups resident on one XCD stream the same few B
// images out of that XCD's L2 while each reads its own A image once.
// B copies are staged through VGPRs (global_load_dwordx4 at the start of an even phase, ds_write_b128 at its end):
// no LDS-DMA, whose per-instruction issue cost and LDS-alias waits showed up as whole-phase stalls.
// Columns: per (column tile, row tile) a value-only top-2 over the lane's 16 rows (the four chains advance together,
// four inserts per asm statement); the two row tiles merge on the raw values (ties to the first tile) and become one
// packed key (d2 << ib) | row per column tile; a permlane32 swap hands lane L both halves of unit column L, and one
// returning LDS atomicMin on C1 plus one on C2 (min(max(old, k1), k2): the exact top-2 in any arrival order) fold the
// wave's 64 rows into the pair's column state. The C2 atomic is issued in the NEXT unit's epilogue (C2 is a plain
// min, so its timing does not matter), by when the C1 return has long arrived.
// Rows: value-only top-2 in registers across a pass; at the pass's last unit one 5-step halving exchange leaves lane
// l of each half-wave with row l's top-2, stored to rowres.
// Pass split (n_split > 1): a group's passes are cut into n_split contiguous ranges, one workgroup each, when there
// are too few groups to fill the CUs (e.g. one rank's share of C2 at 8 GPUs: 619 pairs, ~155 groups of 4). Rows are
// per pass, so they need nothing; each workgroup's column state then folds into colres (preset to kNoKey) with the
// same pair of returning atomics as inside the workgroup, on global memory: min on C1, min(max(old, k1), k2) on C2.
// ---------------------------------------------------------------------------------------------
constexpr int kPpGroupWaves = 4;
constexpr int kPpWaves = 2 * kPpGroupWaves;
constexpr int kPpThreads = kPpWaves * 64;
constexpr int kPpRowsPerPass = kPpWaves * 64;  // 512
constexpr int kUnitCols = 64;
constexpr int kMaxGroup = 4;
constexpr int kPpLdsBudget = 160 * 1024;
constexpr int kRowAlign = 256;                 // kpad granularity of the packed forms

template <int NK>
struct PpCfg {
    static constexpr int kDa = NK * 16;
    static constexpr int kChunkBytes = 32 * kDa * 2;    // one 32-column MFMA tile of B (9 KiB at NK = 9)
    static constexpr int kUnitBytes = 2 * kChunkBytes;  // 64 columns
    static constexpr int kPieces = kUnitBytes / 1024;   // 1-KiB wave copies (lane l: bytes [16l, 16l+16)) per unit
    static constexpr int kPiecesPerWave = (kPieces + 7) / 8;
    static_assert(kUnitBytes % 1024 == 0, "unit must be whole 1-KiB pieces");
};
typedef unsigned pp_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// x from lane (l ^ d) within each 32-lane half (ds_swizzle bit mode: and 0x1F, xor d; no address VGPR)
__device__ __forceinline__ uint32_t xor_swizzle(uint32_t x, int d) {
    switch (d) {
        case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (16 << 10));
        case 8: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (8 << 10));
        case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (4 << 10));
        case 2: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (2 << 10));
        default: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (1 << 10));
    }
}

// one v_med3_u32 / v_min3_u32 / v_and_or_b32, free to schedule
__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t min3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// running top-2 insert of two values, updated IN PLACE (tied asm operands): the loop-carried row state keeps its
// registers instead of rotating through copies
__device__ __forceinline__ void ins2(uint32_t& b1, uint32_t& b2, uint32_t a, uint32_t b) {
    uint32_t m;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m) : "v"(b1), "v"(a), "v"(b));
    asm("v_min3_u32 %0, %0, %1, %2" : "+v"(b1) : "v"(a), "v"(b));
    asm("v_min_u32 %0, %0, %1" : "+v"(b2) : "v"(m));
}
// four independent inserts in ONE asm statement, interleaved (each dependent pair three instructions apart). The
// compiler puts an s_nop after every inline-asm statement that is followed by another, so fewer, larger statements
// issue fewer of them.
__device__ __forceinline__ void ins2x4(uint32_t& b10, uint32_t& b20, uint32_t a0, uint32_t c0,
                                       uint32_t& b11, uint32_t& b21, uint32_t a1, uint32_t c1,
                                       uint32_t& b12, uint32_t& b22, uint32_t a2, uint32_t c2,
                                       uint32_t& b13, uint32_t& b23, uint32_t a3, uint32_t c3) {
    uint32_t m0, m1, m2, m3;
    asm("v_med3_u32 %8, %0, %12, %13\n\t"
        "v_med3_u32 %9, %2, %14, %15\n\t"
        "v_med3_u32 %10, %4, %16, %17\n\t"
        "v_med3_u32 %11, %6, %18, %19\n\t"
        "v_min3_u32 %0, %0, %12, %13\n\t"
        "v_min3_u32 %2, %2, %14, %15\n\t"
        "v_min3_u32 %4, %4, %16, %17\n\t"
        "v_min3_u32 %6, %6, %18, %19\n\t"
        "v_min_u32 %1, %1, %8\n\t"
        "v_min_u32 %3, %3, %9\n\t"
        "v_min_u32 %5, %5, %10\n\t"
        "v_min_u32 %7, %7, %11"
        : "+v"(b10), "+v"(b20), "+v"(b11), "+v"(b21), "+v"(b12), "+v"(b22), "+v"(b13), "+v"(b23),
          "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3)
        : "v"(a0), "v"(c0), "v"(a1), "v"(c1), "v"(a2), "v"(c2), "v"(a3), "v"(c3));
}


// Per-slot (pair) description, wave-uniform.
struct PpSlot {
    int pair, img_a, img_b, na, nb, nsup;
};

// Unit iterator over (pass, slot, column unit), skipping slots with no rows left in the pass; `cur` caches the
// slot's description so that stepping within a slot touches no memory. Wave-uniform.
struct PpIter {
    int pass, slot, sc, seq;  // seq: running unit number (LDS ring parity)
    bool valid;
    PpSlot cur;
};

#define PP_STAMP(v)

template <int NK, bool kClamp>
__global__ __launch_bounds__(kPpThreads, 1) void mnn_pp_kernel(const _Float16* __restrict__ a_form,
                                                               const _Float16* __restrict__ b_form,
                                                               const int* __restrict__ counts,
                                                               const int* __restrict__ pairs, int n_pairs,
                                                               const int* __restrict__ groups, int n_groups,
                                                               int group_size, int n_split, int kpad, int kmax,
                                                               int kmax64, int ib, uint2* __restrict__ rowres,
                                                               uint2* __restrict__ colres) {
    using Cfg = PpCfg<NK>;
    __shared__ __attribute__((aligned(1024))) unsigned char ring[2 * Cfg::kUnitBytes];
    __shared__ int sinfo[kMaxGroup * 8];
    extern __shared__ __attribute__((aligned(16))) uint32_t colstate[];  // [G][2][kmax64]

    const int tid = threadIdx.x, wave = uniform(tid >> 6), lane = tid & 63;
    const int lrow = lane & 31, half = lane >> 5, grp = wave >> 2;
    // bijective XCD remap (blocks b, b + 8, ... share an XCD and take consecutive (group, split) units: the splits
    // of one group stream the same B images through that XCD's L2)
    const int n_blk = n_groups * n_split;
    const int blk = blockIdx.x, xcd = blk & 7, q8 = n_blk >> 3, r8 = n_blk & 7;
    const int flat = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blk >> 3);
    const int grp_idx = flat / n_split, split = flat - grp_idx * n_split;
    const int G = groups ? group_size : 1;

    if (tid < kMaxGroup) {
        int p = -1;
        if (tid < G) p = groups ? groups[(size_t)grp_idx * group_size + tid] : grp_idx;
        if (p >= n_pairs) p = -1;
        int ia = 0, ibm = 0, na = 0, nb = 0;
        if (p >= 0) {
            ia = pairs[2 * p];
            ibm = pairs[2 * p + 1];
            na = counts[ia];
            nb = counts[ibm];
            if (na <= 0 || nb <= 0) na = nb = 0;
        }
        int* si = sinfo + tid * 8;
        si[0] = p; si[1] = ia; si[2] = ibm; si[3] = na; si[4] = nb; si[5] = (nb + kUnitCols - 1) / kUnitCols;
    }
    for (int c = tid; c < G * 2 * kmax64; c += kPpThreads) colstate[c] = kNoKey;
    __syncthreads();

    auto slot_info = [&](int s) {  // LDS broadcast read (slot changes only)
        const int* si = sinfo + s * 8;
        PpSlot r;
        r.pair = uniform(si[0]); r.img_a = uniform(si[1]); r.img_b = uniform(si[2]);
        r.na = uniform(si[3]); r.nb = uniform(si[4]); r.nsup = uniform(si[5]);
        return r;
    };
    int npass_all = 0;
    for (int s = 0; s < G; ++s) npass_all = max(npass_all, (slot_info(s).na + kPpRowsPerPass - 1) / kPpRowsPerPass);
    // this workgroup's passes [pass_lo, npass)
    const int pass_per = (npass_all + n_split - 1) / n_split;
    const int pass_lo = min(npass_all, split * pass_per), npass = min(npass_all, pass_lo + pass_per);
    auto seek = [&](PpIter& it) {  // from (pass, slot) onwards to the first active (pass, slot)
        while (it.pass < npass) {
            it.cur = slot_info(it.slot);
            if (it.cur.pair >= 0 && it.cur.nsup > 0 && it.pass * kPpRowsPerPass < it.cur.na) break;
            if (++it.slot == G) { it.slot = 0; ++it.pass; }
        }
        it.valid = it.pass < npass;
    };
    auto advance = [&](PpIter& it) {
        ++it.seq;
        if (++it.sc < it.cur.nsup) return;
        it.sc = 0;
        if (++it.slot == G) { it.slot = 0; ++it.pass; }
        seek(it);
    };
    PpIter first;
    first.slot = first.sc = first.seq = 0;
    first.pass = pass_lo;
    seek(first);
    int n_units = 0;
    for (PpIter it = first; it.valid; ) {  // whole slots at a time
        n_units += it.cur.nsup;
        it.seq += it.cur.nsup - 1;
        it.sc = it.cur.nsup - 1;
        advance(it);
    }

    // B unit copy, staged through VGPRs: this wave's kPiecesPerWave 1-KiB pieces (surplus pieces repeat one).
    pp_u32x4 stage[Cfg::kPiecesPerWave];
    auto stage_load = [&](const PpIter& it) {
        const unsigned char* src =
            (const unsigned char*)(b_form + ((size_t)it.cur.img_b * kpad + it.sc * kUnitCols) * Cfg::kDa) + lane * 16;
#pragma unroll
        for (int i = 0; i < Cfg::kPiecesPerWave; ++i)
            stage[i] = *(const pp_u32x4*)(src + ((wave + kPpWaves * i) % Cfg::kPieces) * 1024);
    };
    auto stage_store = [&](const PpIter& it) {
        unsigned char* dst = ring + (it.seq & 1) * Cfg::kUnitBytes + lane * 16;
#pragma unroll
        for (int i = 0; i < Cfg::kPiecesPerWave; ++i)
            *(pp_u32x4*)(dst + ((wave + kPpWaves * i) % Cfg::kPieces) * 1024) = stage[i];
    };

    half8 afrag[2][NK];
    int a_loaded_img = -1, a_loaded_pass = -1;
    // A fragments of this wave's 64 rows of pass `pass` (lane holds A[row = lrow][k = 16 s + 8 half .. +8])
    auto load_a = [&](int img, int pass) {
        if (img == a_loaded_img && pass == a_loaded_pass) return;
        a_loaded_img = img;
        a_loaded_pass = pass;
        const int r0w = pass * kPpRowsPerPass + wave * 64;
        if (r0w >= kpad) return;
        const _Float16* A = a_form + (size_t)img * kpad * Cfg::kDa;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const _Float16* arow = A + (size_t)(r0w + 32 * t + lrow) * Cfg::kDa + 8 * half;
#pragma unroll
            for (int s = 0; s < NK; ++s) afrag[t][s] = *(const half8*)(arow + 16 * s);
        }
        __builtin_amdgcn_s_waitcnt(0x0070);  // here: the MFMA stream after the join carries no A-load waits
    };

    const uint32_t dsat = (1u << (32 - ib)) - 1u;
    uint32_t rb1[2][16], rb2[2][16];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) rb1[t][g] = rb2[t][g] = kNoKey;
    f32x16 acc[2][2];  // [sub (32-column tile)][t (32-row tile)]
    uint32_t dold = 0, dm1 = 0, dm2 = 0;  // the pending C2 update of the previous unit
    uint32_t* dptr = colstate;
    bool dpend = false;

    PpIter work = first, cpy = first;
    if (first.valid) {  // unit 0 -> ring[0]
        stage_load(cpy);
        stage_store(cpy);
        advance(cpy);
    }
    __syncthreads();

    // Phases (one barrier each): group 0 runs M(k) in phase 2k and E(k) in phase 2k+1, group 1 one phase later. Every
    // wave loads its share of unit k+1 into VGPRs at the start of phase 2k and stores it at the end of phase 2k+1
    // into the ring buffer unit k-1 held (free since phase 2k-1): two phases of latency cover an HBM miss.
    PpIter cpy_pending;
    bool pending = false;
    auto copy_begin = [&]() {
        pending = cpy.valid;
        if (pending) {
            cpy_pending = cpy;
            stage_load(cpy);
            advance(cpy);
        }
    };
    auto copy_end = [&]() {
        if (pending) stage_store(cpy_pending);
        pending = false;
    };
    if (grp == 1 && n_units > 0) copy_begin();  // group 1's leading phase 0: the load of unit 1
    if (grp == 1 && n_units > 0) __syncthreads();
    for (int k = 0; k < n_units; ++k) {
        PP_STAMP(t0);
        const PpSlot si = work.cur;
        const int r0w = work.pass * kPpRowsPerPass + wave * 64;
        const bool rows_here = r0w < si.na;
        // ---- phase A of this iteration: group 0 -> phase 2k (copy of unit k+1), group 1 -> phase 2k+1 (merge k-1)
        // M: 2 x 2 tiles of 32 x 32, K = 16 NK. A new (pass, A image) reloads the A fragments first (once per pass:
        // a short stall the partner wave's E covers).
        load_a(si.img_a, work.pass);
        if (grp == 0) copy_begin();  // after the A loads, so the MFMAs never wait for the staged copy
        __builtin_amdgcn_s_setprio(2);  // the MFMA stream outranks the partner wave's VALU epilogue
        if (rows_here) {
            const unsigned char* bb = ring + (work.seq & 1) * Cfg::kUnitBytes + lane * 16;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) acc[sub][0] = acc[sub][1] = f32x16{};
            half8 bf[2][2];  // [k-step parity][sub]: the next k-step's B fragments are read ahead
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) bf[0][sub] = *(const half8*)(bb + sub * Cfg::kChunkBytes);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int s = 0; s < NK; ++s) {
                if (s + 1 < NK) {
#pragma unroll
                    for (int sub = 0; sub < 2; ++sub)
                        bf[(s + 1) & 1][sub] = *(const half8*)(bb + sub * Cfg::kChunkBytes + 1024 * (s + 1));
                }
#pragma unroll
                for (int sub = 0; sub < 2; ++sub) {
                    acc[sub][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(afrag[0][s], bf[s & 1][sub], acc[sub][0], 0, 0, 0);
                    acc[sub][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(afrag[1][s], bf[s & 1][sub], acc[sub][1], 0, 0, 0);
                }
                if (s + 1 < NK) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            }
        }
        if (grp == 1) copy_end();  // loaded at the start of phase 2k
        PP_STAMP(t1);
        __syncthreads();
        PP_STAMP(t2);
        // ---- phase B: group 0 -> phase 2k+1, group 1 -> phase 2k+2 (load of unit k+2)
        __builtin_amdgcn_s_setprio(0);
        if (grp == 1) copy_begin();
        if (rows_here) {
            // columns: value-only top-2 over the lane's 16 rows of each (column tile, row tile) -> keys
            // (d2 << ib) | row with row = rowbase | code; the two row tiles merged; a permlane32 swap then gives lane L
            // both halves' top-2 of column tile L >> 5, column L & 31, so lane L owns unit column L: one returning
            // atomic min on C1 and one on C2 per lane (min(max(old, k1), k2) keeps the exact top-2 in any order)
            uint32_t s1[2], s2[2];
            uint32_t cv1[2][2], cv2[2][2];  // the four (sub, t) column chains, advanced together
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    cv1[sub][t] = umin(__float_as_uint(acc[sub][t][0]), __float_as_uint(acc[sub][t][1]));
                    cv2[sub][t] = umax(__float_as_uint(acc[sub][t][0]), __float_as_uint(acc[sub][t][1]));
                }
#define PPU(sub, t, g) __float_as_uint(acc[sub][t][g])
#pragma unroll
            for (int g = 2; g < 16; g += 2)
                ins2x4(cv1[0][0], cv2[0][0], PPU(0, 0, g), PPU(0, 0, g + 1), cv1[0][1], cv2[0][1], PPU(0, 1, g),
                       PPU(0, 1, g + 1), cv1[1][0], cv2[1][0], PPU(1, 0, g), PPU(1, 0, g + 1), cv1[1][1], cv2[1][1],
                       PPU(1, 1, g), PPU(1, 1, g + 1));
            // the two row tiles of a column merge on the raw values (ties to t = 0: its rows come first), so one key
            // is built per column tile instead of two
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) {
                const uint32_t a0 = cv1[sub][0], a1 = cv1[sub][1];
                const bool take1 = a1 < a0;
                const uint32_t v1 = take1 ? a1 : a0;
                const uint32_t v2 = med3u(a0, a1, umin(cv2[sub][0], cv2[sub][1]));
                const uint32_t u = (uint32_t)(__uint_as_float(v1) * 16.f);
                uint32_t d1 = u >> 4, d2 = (uint32_t)__uint_as_float(v2);
                if constexpr (kClamp) { d1 = umin(d1, dsat); d2 = umin(d2, dsat); }
                const uint32_t rowbase = (uint32_t)(r0w + 16 * half) + (take1 ? 32u : 0u);
                s1[sub] = (d1 << ib) | rowbase | (u & 15u);
                s2[sub] = d2 << ib;
            }
            const auto x1 = __builtin_amdgcn_permlane32_swap(s1[0], s1[1], false, false);
            const auto x2 = __builtin_amdgcn_permlane32_swap(s2[0], s2[1], false, false);
            const uint32_t m1 = umin(x1[0], x1[1]), m2 = med3u(x1[0], x1[1], umin(x2[0], x2[1]));
            uint32_t* c1s = colstate + work.slot * 2 * kmax64 + work.sc * kUnitCols + lane;
            if (dpend) __hip_atomic_fetch_min(dptr + kmax64, umin(umax(dold, dm1), dm2), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
            dold = __hip_atomic_fetch_min(c1s, m1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            dm1 = m1; dm2 = m2; dptr = c1s; dpend = true;
            // the row inserts run while the returning atomic is in flight
            __builtin_amdgcn_sched_barrier(0);
            // rows: both column tiles' values of row (t, g) in one paired insert
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int g = 0; g < 16; g += 4)
                    ins2x4(rb1[t][g], rb2[t][g], PPU(0, t, g), PPU(1, t, g), rb1[t][g + 1], rb2[t][g + 1],
                           PPU(0, t, g + 1), PPU(1, t, g + 1), rb1[t][g + 2], rb2[t][g + 2], PPU(0, t, g + 2),
                           PPU(1, t, g + 2), rb1[t][g + 3], rb2[t][g + 3], PPU(0, t, g + 3), PPU(1, t, g + 3));
#undef PPU
            __builtin_amdgcn_sched_barrier(0);
            if (work.sc == si.nsup - 1) {
                // the pass is over for this pair: halving exchange across each half-wave's 32 lanes, then lane
                // (lrow, half) holds register j = lrow = 16 t + g, i.e. keypoint r0w + 32 t + 16 half + g
                uint32_t* x1 = &rb1[0][0];  // in place: the row state restarts after the store
                uint32_t* x2 = &rb2[0][0];
#pragma unroll
                for (int d = 16; d >= 1; d >>= 1) {
                    const bool up = (lrow & d) != 0;
#pragma unroll
                    for (int j = 0; j < d; ++j) {
                        const uint32_t s1 = up ? x1[j] : x1[j + d], s2 = up ? x2[j] : x2[j + d];
                        const uint32_t q1 = up ? x1[j + d] : x1[j], q2 = up ? x2[j + d] : x2[j];
                        const uint32_t o1 = xor_swizzle(s1, d), o2 = xor_swizzle(s2, d);
                        x1[j] = umin(q1, o1);
                        x2[j] = med3u(q1, o1, umin(q2, o2));
                        if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound the temporaries
                    }
                }
                const int key = r0w + 32 * (lrow >> 4) + 16 * half + (lrow & 15);
                if (key < si.na) rowres[(size_t)si.pair * kmax + key] = make_uint2(x1[0], x2[0]);
#pragma unroll
                for (int j = 0; j < 32; ++j) x1[j] = x2[j] = kNoKey;
            }
        }
        if (grp == 0) copy_end();  // loaded in phase 2k
        advance(work);
        PP_STAMP(t3);
        __syncthreads();
        PP_STAMP(t4);
    }
    if (dpend) __hip_atomic_fetch_min(dptr + kmax64, umin(umax(dold, dm1), dm2), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    if (grp == 0 && n_units > 0) __syncthreads();  // group 0's trailing phase 2U (group 1's E of the last unit)
    __syncthreads();
    for (int s = 0; s < G; ++s) {
        const PpSlot si = slot_info(s);
        if (si.pair < 0 || si.na == 0) continue;
        const uint32_t* c1s = colstate + s * 2 * kmax64;
        const uint32_t* c2s = c1s + kmax64;
        if (n_split == 1) {
            for (int c = tid; c < si.nb; c += kPpThreads)
                colres[(size_t)si.pair * kmax + c] = make_uint2(c1s[c], c2s[c]);
        } else if (pass_lo * kPpRowsPerPass < si.na) {  // this workgroup saw rows of the pair
            for (int c = tid; c < si.nb; c += kPpThreads) {
                uint32_t* g = (uint32_t*)(colres + (size_t)si.pair * kmax + c);
                const uint32_t k1 = c1s[c], k2 = c2s[c];
                const uint32_t old = __hip_atomic_fetch_min(g, k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_min(g + 1, umin(umax(old, k1), k2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
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

// Per-keypoint top-2 encodings consumed by finalize.
//   kResExact: ExactTop2 on both sides (exact fp32 path); rowres = image i1's keypoints, colres = image i2's.
//   kResCodes: mnn_pp_kernel. rowres = image i1's keypoints: raw accumulator bits (d2 + code/16, value-only);
//              colres = image i2's keypoints: packed keys (d2 << ib) | i1 index (second: distance only).
constexpr int kResExact = 0, kResCodes = 1;
template <int kRes> constexpr int kRedoIntsOf = kRes == kResCodes ? 2 : 1;  // redo list length / kmax

template <int kRes>
__global__ __launch_bounds__(kFinThreads) void match_finalize_kernel(const void* __restrict__ rowres_v,
                                                                     const void* __restrict__ colres_v,
                                                                     const float* __restrict__ desc,
                                                                     const int* __restrict__ counts,
                                                                     const int* __restrict__ pairs, int kmax,
                                                                     int dim, int ib, double ratio,
                                                                     uint32_t* __restrict__ out_idx,
                                                                     int* __restrict__ out_count) {
    constexpr int kRedoInts = kRedoIntsOf<kRes>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int* hdr = (int*)smem;                                           // [0] matches, [1] redo rows, [2] redo keys
    float* red_d = (float*)(smem + 16);                               // [2*kFinThreads]
    int* red_j = (int*)(smem + 16 + 8 * kFinThreads);                 // [kFinThreads]
    int* redo = (int*)(smem + 16 + 12 * kFinThreads);                 // [2 kmax]: rows from the front, keys from the back
    unsigned long long* keys =
        (unsigned long long*)(smem + 16 + 12 * kFinThreads + gtsfm_align_up((size_t)kmax * kRedoInts * 4, 16));
    const int p = blockIdx.x;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const int n1 = counts[i1], n2 = counts[i2];
    const int tid = threadIdx.x;
    if (tid == 0) { hdr[0] = 0; hdr[1] = 0; hdr[2] = 0; }
    __syncthreads();
    auto push = [&](int i, int j, float d1r) {
        const int slot = atomicAdd(&hdr[0], 1);
        keys[slot] = ((unsigned long long)__float_as_uint(d1r) << 32) | ((unsigned long long)i << 16) | (uint32_t)j;
    };
    const float* D1 = desc + (size_t)i1 * kmax * dim;
    const float* D2 = desc + (size_t)i2 * kmax * dim;

    if constexpr (kRes == kResCodes) {
        // Image i2's keypoint j with key nearest i is mutual iff i's best distance equals d(i, j) and i has no tie at
        // its minimum (then j, reaching that minimum, is i's unique nearest). A tied i whose own ratio test can pass
        // is recomputed exactly ("row redo"); one that cannot is in no match. Key fields equal to dsat are padding
        // ("no neighbour") when ib <= 12 and possibly clamped distances when ib = 13: those keypoints are recomputed
        // exactly too ("key redo"), unless their nearest i is a row redo (which finds the same match).
        const uint32_t imask = (1u << ib) - 1u, dsat = (1u << (32 - ib)) - 1u;
        const bool clamped = ib > 12;
        const uint2* rv = (const uint2*)rowres_v + (size_t)p * kmax;
        const uint2* ck = (const uint2*)colres_v + (size_t)p * kmax;
        auto rdec = [](uint32_t bits) { return (uint32_t)__uint_as_float(bits); };  // trunc: d2
        auto row_redo = [&](uint2 v) {
            const uint32_t a = rdec(v.x);
            return a == rdec(v.y) && ratio_ok(sqrt_cr((float)a), sqrt_cr((float)a), ratio);
        };
        auto row_d2 = [&](uint32_t bits) {
            const uint32_t d = rdec(bits);
            return d >= kRowPoisonD2 ? __builtin_inff() : sqrt_cr((float)d);
        };
        if (n1 > 0 && n2 > 0) {
            for (int i = tid; i < n1; i += kFinThreads)
                if (row_redo(rv[i])) redo[atomicAdd(&hdr[1], 1)] = i;
            for (int j = tid; j < n2; j += kFinThreads) {
                const uint2 k = ck[j];
                const uint32_t kd1 = k.x >> ib, kd2 = k.y >> ib;
                if (kd1 == dsat || (clamped && kd2 == dsat)) {
                    if (clamped) redo[2 * kmax - 1 - atomicAdd(&hdr[2], 1)] = j;
                    continue;
                }
                const int i = (int)(k.x & imask);
                const uint2 v = rv[i];
                if (row_redo(v) || rdec(v.x) != kd1 || rdec(v.y) == kd1) continue;
                const float d1r = sqrt_cr((float)kd1);
                const float d2c = kd2 == dsat ? __builtin_inff() : sqrt_cr((float)kd2);
                if (ratio_ok(d1r, row_d2(v.y), ratio) && ratio_ok(d1r, d2c, ratio)) push(i, j, d1r);
            }
        }
        __syncthreads();
        const int nrow = hdr[1], nkey = hdr[2];
        for (int r = 0; r < nrow; ++r) {
            const int i = redo[r];
            float d1r, d2r, d1c, d2c;
            int j, ic;
            block_exact_top2(D1 + (size_t)i * dim, D2, n2, dim, red_d, red_j, d1r, d2r, j);
            if (j < 0) continue;
            block_exact_top2(D2 + (size_t)j * dim, D1, n1, dim, red_d, red_j, d1c, d2c, ic);
            if (tid == 0 && ic == i && ratio_ok(d1r, d2r, ratio) && ratio_ok(d1c, d2c, ratio)) push(i, j, d1r);
            __syncthreads();
        }
        for (int r = 0; r < nkey; ++r) {
            const int j = redo[2 * kmax - 1 - r];
            float d1r, d2r, d1c, d2c;
            int i, jj;
            block_exact_top2(D2 + (size_t)j * dim, D1, n1, dim, red_d, red_j, d1c, d2c, i);
            if (i < 0 || row_redo(rv[i])) continue;  // uniform: every thread reads the same i
            block_exact_top2(D1 + (size_t)i * dim, D2, n2, dim, red_d, red_j, d1r, d2r, jj);
            if (tid == 0 && jj == j && ratio_ok(d1r, d2r, ratio) && ratio_ok(d1c, d2c, ratio)) push(i, j, d1r);
            __syncthreads();
        }
    } else {
        for (int i = tid; i < n1 && n2 > 0; i += kFinThreads) {
            const ExactTop2 r = ((const ExactTop2*)rowres_v)[(size_t)p * kmax + i];
            if (r.j1 < 0) continue;
            const int j = r.j1;
            const ExactTop2 c = ((const ExactTop2*)colres_v)[(size_t)p * kmax + j];
            if (c.j1 == i && ratio_ok(r.d1, r.d2, ratio) && ratio_ok(c.d1, c.d2, ratio)) push(i, j, r.d1);
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
inline int pack_kpad(int kmax) { return (int)gtsfm_align_up((size_t)kmax, kRowAlign); }
inline int pp_kmax64(int kmax) { return (int)gtsfm_align_up((size_t)kmax, kUnitCols); }

// dynamic LDS (column state) and total LDS (+ the static B ring and slot table) of mnn_pp_kernel<NK>
inline size_t pp_dyn_lds_bytes(int kmax, int group_size) {
    return (size_t)group_size * 2 * pp_kmax64(kmax) * sizeof(uint32_t);
}
template <int NK>
size_t pp_lds_bytes(int kmax, int group_size) {
    return 2 * (size_t)PpCfg<NK>::kUnitBytes + kMaxGroup * 8 * sizeof(int) +
           pp_dyn_lds_bytes(kmax, group_size);  // B ring + slot table (static) + column state
}

// Largest group size (pairs per workgroup) whose column state fits the LDS next to the B ring.
int pp_max_group(int kmax, int dim) {
    const int nk = pack_da(dim) / 16;
    for (int g = kMaxGroup; g >= 1; --g) {
        const size_t lds = nk == 2 ? pp_lds_bytes<2>(kmax, g) : nk == 5 ? pp_lds_bytes<5>(kmax, g) : pp_lds_bytes<9>(kmax, g);
        if (lds <= (size_t)kPpLdsBudget) return g;
    }
    return 0;
}

// Pass split of a launch: the n_split in {1, 2, 4} (at most the passes of kmax rows) that minimises the estimated
// time ceil(n_groups * n_split / CUs) * (passes / n_split) of one workgroup per CU; ties keep fewer workgroups.
// gtsfm_amd.device.match_plan mirrors this to choose the group size.
int pp_split(int n_groups, int kmax, int n_cu) {
    const int npass = (kmax + kPpRowsPerPass - 1) / kPpRowsPerPass;
    int best = 1;
    double best_t = 1e300;
    for (int s = 1; s <= 4 && s <= npass; s *= 2) {
        const double t = (double)((n_groups * s + n_cu - 1) / n_cu) * ((npass + s - 1) / s);
        if (t < best_t) { best_t = t; best = s; }
    }
    return best;
}

// CU count of the CURRENT device (cached per device id: a process may drive several GPUs)
int device_cu_count() {
    constexpr int kDevs = 64;
    static std::atomic<int> cached[kDevs];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev >= 0 && dev < kDevs) {
        const int c = cached[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev >= 0 && dev < kDevs) cached[dev].store(n, std::memory_order_relaxed);
    return n;
}

template <int NK, bool kClamp>
int launch_pp_t(const _Float16* a_form, const _Float16* b_form, const int* counts, const int* pairs, int n_pairs,
                const int* groups, int n_groups, int group_size, int kpad, int kmax, int ib, int dim, uint2* rowres,
                uint2* colres, hipStream_t stream) {
    const int gs = groups ? group_size : 1;
    if (pp_lds_bytes<NK>(kmax, gs) > (size_t)kPpLdsBudget) return GTSFM_ERR_ARG;
    const size_t lds = pp_dyn_lds_bytes(kmax, gs);
    int n_split = pp_split(n_groups, kmax, device_cu_count());
    // test hook: GTSFM_MATCH_PASS_SPLIT=1|2|4 forces the split, so tests can pin every path against the oracle
    if (const char* f = getenv("GTSFM_MATCH_PASS_SPLIT")) {
        const int v = atoi(f);
        if (v == 1 || v == 2 || v == 4) n_split = v;
    }
    if (n_split > 1)  // the workgroups fold their column state into colres with atomics
        GTSFM_CHECK_HIP(hipMemsetAsync(colres, 0xFF, (size_t)n_pairs * kmax * sizeof(uint2), stream));
    GTSFM_CHECK_HIP(gtsfm_set_dynamic_lds((const void*)mnn_pp_kernel<NK, kClamp>, (int)lds));
    hipLaunchKernelGGL((mnn_pp_kernel<NK, kClamp>), dim3(n_groups * n_split), dim3(kPpThreads), lds, stream, a_form,
                       b_form, counts, pairs, n_pairs, groups, n_groups, group_size, n_split, kpad, kmax,
                       pp_kmax64(kmax), ib, rowres, colres);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

template <int NK>
int launch_pp(const _Float16* a_form, const _Float16* b_form, const int* counts, const int* pairs, int n_pairs,
              const int* groups, int n_groups, int group_size, int kpad, int kmax, int ib, int dim, uint2* rowres,
              uint2* colres, hipStream_t stream) {
    if (ib <= 12)
        return launch_pp_t<NK, false>(a_form, b_form, counts, pairs, n_pairs, groups, n_groups, group_size, kpad,
                                      kmax, ib, dim, rowres, colres, stream);
    return launch_pp_t<NK, true>(a_form, b_form, counts, pairs, n_pairs, groups, n_groups, group_size, kpad, kmax,
                                 ib, dim, rowres, colres, stream);
}

// side1 / side2: per-keypoint top-2 of image i1 / image i2 of each pair (encoding kRes)
template <int kRes>
int launch_finalize(const void* side1, const void* side2, const float* desc, const int* counts, const int* pairs,
                    int n_pairs, int kmax, int dim, int ib, double ratio, uint32_t* out_idx, int* out_count,
                    hipStream_t stream) {
    const size_t lds = 16 + 12 * kFinThreads + gtsfm_align_up((size_t)kmax * kRedoIntsOf<kRes> * 4, 16) +
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
typedef float fl_float2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void fl_insert(float x, int j, float (&v)[kFlCand], int (&id)[kFlCand]) {
    // v sorted ascending and x < v[kFlCand - 1]: branch-free insertion (each slot takes its left neighbour, x or
    // itself). The key of slot m is med3(v[m-1], x, v[m]) -- v[m-1] when x < v[m-1], x when v[m-1] <= x < v[m], else
    // v[m] -- one v_med3_f32; the ids follow the same strict comparisons, each computed once.
    bool lt[kFlCand];
#pragma unroll
    for (int m = 0; m < kFlCand; ++m) lt[m] = x < v[m];
#pragma unroll
    for (int m = kFlCand - 1; m > 0; --m) {
        v[m] = __builtin_amdgcn_fmed3f(v[m - 1], x, v[m]);
        id[m] = lt[m - 1] ? id[m - 1] : (lt[m] ? j : id[m]);
    }
    v[0] = lt[0] ? x : v[0];
    id[0] = lt[0] ? j : id[0];
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
    // 1-D grid, XCD-contiguous: the hardware deals consecutive workgroups to the 8 XCDs in turn, so workgroup b runs
    // logical block (b & 7) * per_xcd + (b >> 3); each XCD then walks whole (pair, side) groups of query blocks in
    // order and the group's train image is read into that XCD's L2 once, not by every XCD
    const int n_qb = kpad / kFlQ, total = n_qb * n_pairs * 2, per_xcd = (total + 7) / 8;
    const int lb = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (lb >= total) return;
    const int qb = lb % n_qb, p = (lb / n_qb) % n_pairs, side = lb / (n_qb * n_pairs);
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, h = l >> 5;
    const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
    const int nq = counts[iq], nt = counts[it];
    const int q0 = qb * kFlQ;
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
    const int n_chunks = (nt + kFlRows - 1) / kFlRows;
    // one chunk: two 32-row MFMA tiles against the wave's 32 queries, then the top-8 epilogue per tile
    auto process = [&](int c, int buf) {
        const int c0 = c * kFlRows;
        const _Float16* tb = tl + buf * kFlRows * RS;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            fl_float16 acc = {};
            const _Float16* arow = tb + (t * 32 + (l & 31)) * RS + 8 * h;
#pragma unroll
            for (int s = 0; s < NS; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const fl_half8*)(arow + 16 * s), bq[s], acc, 0, 0, 0);
            // the tile's 16 keys of this lane, a mask of those below the shortlist's current last key, then one
            // insert per wave iteration for every lane that still has a set bit, in index order: the same insertion
            // sequence as testing the keys one by one, but the wave runs max(popcount) inserts instead of one per
            // key that ANY lane accepts
            float kk[16];
            uint32_t mask = 0;
            const float thr = v[kFlCand - 1];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 nb = *(const float4*)(nbl + buf * kFlRows + t * 32 + 8 * g + 4 * h);
                kk[4 * g] = fmaf(-2.f, acc[4 * g], nb.x);
                kk[4 * g + 1] = fmaf(-2.f, acc[4 * g + 1], nb.y);
                kk[4 * g + 2] = fmaf(-2.f, acc[4 * g + 2], nb.z);
                kk[4 * g + 3] = fmaf(-2.f, acc[4 * g + 3], nb.w);
#pragma unroll
                for (int e = 0; e < 4; ++e) mask |= (kk[4 * g + e] < thr ? 1u : 0u) << (4 * g + e);
            }
            // branch-free body: a lane without a pending key (or whose key no longer beats the last slot) inserts
            // +inf, which leaves the sorted list and its ids unchanged
            while (__ballot(mask != 0u) != 0ull) {
                const int i = __builtin_ctz(mask | 0x10000u);  // 16: nothing pending
                mask &= mask - 1u;
                float x = __builtin_inff();
#pragma unroll
                for (int q = 0; q < 16; ++q) x = i == q ? kk[q] : x;
                x = x < v[kFlCand - 1] ? x : __builtin_inff();
                fl_insert(x, c0 + t * 32 + 8 * (i >> 2) + 4 * h + (i & 3), v, id);
            }
        }
    };
    // register prefetch two chunks ahead (chunk c + 2 is loaded while chunk c is computed, chunk c + 1 waits in the
    // other register set and is stashed at the end of chunk c): each load has two chunks of work to land
    fl_u32x4 preA[NV], preB[NV];
    float pnA = 0.f, pnB = 0.f;
    if (n_chunks > 0) {
        fl_fetch<NV, DP>(preA, pnA, tbase, nbase, 0, tid);
        fl_stash<NV, DP>(preA, pnA, tl, nbl, 0, tid);
    }
    if (n_chunks > 1) fl_fetch<NV, DP>(preB, pnB, tbase, nbase, kFlRows, tid);
    __syncthreads();
    for (int c = 0; c < n_chunks; c += 2) {
        if (c + 2 < n_chunks) fl_fetch<NV, DP>(preA, pnA, tbase, nbase, (c + 2) * kFlRows, tid);
        process(c, 0);
        if (c + 1 < n_chunks) fl_stash<NV, DP>(preB, pnB, tl, nbl, 1, tid);
        __syncthreads();
        if (c + 1 >= n_chunks) break;
        if (c + 3 < n_chunks) fl_fetch<NV, DP>(preB, pnB, tbase, nbase, (c + 3) * kFlRows, tid);
        process(c + 1, 1);
        if (c + 2 < n_chunks) fl_stash<NV, DP>(preA, pnA, tl, nbl, 0, tid);
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
        for (int c = 0; c < kFlCand; ++c) {
            cand[o * kFlCand + c] = id[c];
            tkey[o * kFlCand + c] = v[c];  // ascending keys; the last one bounds every keypoint off the shortlist
        }
    }
}

// grid ceil(2P / 8) * 8 units x ceil(kmax / 128) row blocks (1-D, XCD-ordered below), 256 threads, keypoints
// i0 .. i0 + 127 of one (pair, side): the exact squared distance of each keypoint to its shortlisted candidates, each
// summed by one thread straight from HBM/L2 (float4 row walks), sequentially and unfused: exact_top2_kernel's
// arithmetic. Two rounds, every lane busy in both: first the two best keys' candidates (two threads per keypoint);
// then the other six, minus those whose key bound already exceeds the larger of the first two exact distances
// (d^2 >= (|a|^2 + key) - eps > that: neither of the exact top two, nor tied with them), compacted into a work list
// the 256 threads share. Then one thread per keypoint scans its 8 candidates in index order (the exact scan's b1 / j1
// / b2 updates) and checks the certificate; uncertified keypoints go to `redo`.
constexpr int kFlRerankRows = 128;
__global__ __launch_bounds__(256) void fl_rerank_kernel(const float* __restrict__ desc, const int* __restrict__ counts,
                                                        int kmax, int dim, const int* __restrict__ pairs, int n_pairs,
                                                        int kpad, const float* __restrict__ norm2,
                                                        const unsigned* __restrict__ img_maxnorm,
                                                        const unsigned* __restrict__ img_unsafe,
                                                        const int* __restrict__ cand, const float* __restrict__ tkey,
                                                        ExactTop2* __restrict__ rowres, ExactTop2* __restrict__ colres,
                                                        int* __restrict__ redo_count, int4* __restrict__ redo,
                                                        int* __restrict__ unc) {
#pragma clang fp contract(off)
    constexpr int R = kFlRerankRows, C = kFlCand;
    static_assert(2 * R == 256, "round 1: two threads per keypoint");
    __shared__ float sacc[R][C];
    __shared__ int sj[R][C];
    __shared__ uint16_t work[R * (C - 2)];
    __shared__ int n_work;
    // XCD-aware order: workgroups go round-robin over the 8 XCDs in dispatch order, so XCD x runs every row block of
    // units x, x + 8, ... (unit = one (pair, side)); a unit's train rows, read at random by all of its blocks, are
    // fetched into one XCD's L2. Side-1 units come first, in pair order (consecutive ones share their train image).
    const int nb = (kmax + R - 1) / R;
    const int xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
    const int u = (kx / nb) * 8 + xcd;
    if (u >= 2 * n_pairs) return;
    const int side = u < n_pairs ? 1 : 0, p = u < n_pairs ? u : u - n_pairs, tid = threadIdx.x;
    const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
    const int nq = counts[iq], nt = counts[it];
    const int i0 = (kx % nb) * R;
    if (i0 >= nq) return;
    // the exact squared distance of keypoint i to train keypoint jj, sequential and unfused
    auto exact_d2 = [&](int i, int jj) {
        const float* q = desc + ((size_t)iq * kmax + i) * dim;
        const float* t = desc + ((size_t)it * kmax + jj) * dim;
        float a = 0.f;
        if ((dim & 3) == 0) {
            const float4* q4 = (const float4*)q;
            const float4* t4 = (const float4*)t;
#pragma unroll 8
            for (int k = 0; k < dim / 4; ++k) {
                const float4 x = q4[k], y = t4[k];
                const float e0 = x.x - y.x, e1 = x.y - y.y, e2 = x.z - y.z, e3 = x.w - y.w;
                a = a + e0 * e0;  // unfused, in index order: contract(off) above
                a = a + e1 * e1;
                a = a + e2 * e2;
                a = a + e3 * e3;
            }
        } else {
            for (int k = 0; k < dim; ++k) {
                const float df = q[k] - t[k];
                a = a + df * df;
            }
        }
        return a;
    };
    // the certificate's bound on the fp16 key error: (|a|^2 + key) - eps <= exact d^2 for every train keypoint
    const bool safe = img_unsafe[iq] == 0u && img_unsafe[it] == 0u;
    auto key_eps = [&](float na) {
        const float an = sqrtf(na), bn = __uint_as_float(img_maxnorm[it]);
        const float u = 1.f / 2048.f, eta = 1.f / 33554432.f, D = (float)dim;
        const float e_dot = (2.f * u + u * u + D * 1.01f / 16777216.f) * an * bn + eta * sqrtf(D) * (an + bn) +
                            D * eta * eta;
        return 1.5f * (2.f * e_dot + (D + 4.f) * 2.f / 16777216.f * (na + bn * bn));
    };
    const size_t obase = ((size_t)side * n_pairs + p) * kmax;  // + i: this (pair, side)'s shortlist row of keypoint i
    // candidate ids (-1: none)
    for (int s = tid; s < R * C; s += 256) {
        const int r = s / C, c = s % C, i = i0 + r;
        int j = -1;
        if (i < nq) {
            j = cand[(obase + i) * C + c];
            if (j >= nt) j = -1;
        }
        sj[r][c] = j;
        sacc[r][c] = __builtin_inff();
    }
    if (tid == 0) n_work = 0;
    __syncthreads();
    {  // round 1: the two best keys' candidates
        const int r = tid >> 1, c = tid & 1, j = sj[r][c];
        if (j >= 0) sacc[r][c] = exact_d2(i0 + r, j);
    }
    __syncthreads();
    // round 2's work list: candidates 2..7 that the bound cannot drop
    for (int s = tid; s < R * (C - 2); s += 256) {
        const int r = s / (C - 2), c = 2 + s % (C - 2), i = i0 + r;
        const int j = sj[r][c];
        if (j < 0) continue;
        const float a2 = fmaxf(sacc[r][0], sacc[r][1]);
        bool skip = false;
        if (safe && a2 < __builtin_inff()) {
            const float na = norm2[(size_t)iq * kpad + i];
            skip = (na + tkey[(obase + i) * C + c]) - key_eps(na) > a2 * (1.f + 1e-4f) + key_eps(na);
        }
        if (skip) sj[r][c] = -1;
        else work[atomicAdd(&n_work, 1)] = (uint16_t)(r * C + c);
    }
    __syncthreads();
    const int nw = n_work;
    for (int w = tid; w < nw; w += 256) {
        const int rc = work[w], r = rc / C, c = rc % C;
        sacc[r][c] = exact_d2(i0 + r, sj[r][c]);
    }
    __syncthreads();
    if (tid >= R) return;
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
    if (!certified && safe) {
        const float na = norm2[(size_t)iq * kpad + ii];
        const float eps = key_eps(na);
        certified = (na + tkey[(obase + ii) * kFlCand + kFlCand - 1]) - eps > a2 * (1.f + 1e-4f) + eps;
    }
    if (!certified) {
        redo[atomicAdd(redo_count, 1)] = make_int4(side, p, ii, 0);
        atomicAdd(&unc[side * n_pairs + p], 1);
    }
    (side ? colres : rowres)[(size_t)p * kmax + ii] = ExactTop2{b1, b2, j1, certified ? 0 : 1};
}

// A (pair, side) whose uncertified share reaches 1/kFlTileFrac of its keypoints is recomputed whole by
// fl_exact_tile_kernel (clustered descriptors, e.g. random-weight SuperPoint: the shortlist rarely certifies); fewer
// uncertified keypoints are rescanned one by one.
constexpr int kFlTileFrac = 32;
__device__ __forceinline__ bool fl_use_tile(int n_unc, int nq) { return n_unc > 0 && n_unc * kFlTileFrac >= nq; }
// both sides of pair p are tiled: one pass computes each exact distance once and reduces it both ways
__device__ __forceinline__ bool fl_both(const int* unc, const int* counts, const int* pairs, int n_pairs, int p) {
    return fl_use_tile(unc[p], counts[pairs[2 * p]]) && fl_use_tile(unc[n_pairs + p], counts[pairs[2 * p + 1]]);
}

// Exact top-2 of every keypoint of a flagged (pair, side), tiled: a block takes 64 query rows against all train rows
// in 64-row tiles, K in 32-deep LDS chunks; thread (tq, tt) runs the 16 chains of query rows tq + 16 i and train rows
// tt + 16 j, each the sequential unfused sum over k of exact_top2_kernel (zero padding past dim adds exact zeros), and
// folds its train rows in increasing order with the strict-'<' update. The 16 partial (b1, j1, b2) of a row merge by
// (b1, j1) lexicographic minimum with b2 = min(other b1, own b2): the scan's result in any merge order.
// kBoth (pairs with both sides tiled, grid z = 1): the block's distances also feed the columns -- per column a
// top-2 over the thread's 4 rows, merged across the 16 row threads by shuffles, then folded into the pair's side-1
// state in colres with a returning 64-bit atomicMin on (d1 bits << 32 | row) (slots j1 | pad of the record) and a
// 32-bit atomicMin of min(max(old d1, d1), d2) on d2 -- the exact top-2 in any arrival order, ties to the lowest row,
// as the strict-'<' scan of that side. Distances are symmetric bit for bit ((a - b)^2 == (b - a)^2).
constexpr int kXT = 64, kXK = 16;
template <bool kBoth>
__global__ __launch_bounds__(256) void fl_exact_tile_kernel(const float* __restrict__ desc,
                                                            const int* __restrict__ counts, int kmax, int dim,
                                                            const int* __restrict__ pairs, int n_pairs,
                                                            const int* __restrict__ unc, ExactTop2* __restrict__ rowres,
                                                            ExactTop2* __restrict__ colres) {
#pragma clang fp contract(off)
    // k-major tiles (row stride kXT + 4: 16-B aligned b128 reads, 2-way store conflicts): a thread's 4 rows / columns
    // of one k are one ds_read_b128 each
    __shared__ __attribute__((aligned(16))) float Qs[kXK][kXT + 4];
    __shared__ __attribute__((aligned(16))) float Ts[kXK][kXT + 4];
    __shared__ float mb1[16][kXT], mb2[16][kXT];
    __shared__ int mj[16][kXT];
    const int p = blockIdx.y, side = kBoth ? 0 : blockIdx.z, tid = threadIdx.x;
    const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
    const int nq = counts[iq], nt = counts[it];
    const int q0 = blockIdx.x * kXT;
    if (q0 >= nq || !fl_use_tile(unc[side * n_pairs + p], nq)) return;
    if (fl_both(unc, counts, pairs, n_pairs, p) != kBoth) return;
    const int tq = tid & 15, tt = tid >> 4;
    const float* Q = desc + ((size_t)iq * kmax + q0) * dim;
    const float* T = desc + (size_t)it * kmax * dim;
    float b1[4], b2[4];
    int j1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { b1[i] = b2[i] = __builtin_inff(); j1[i] = -1; }
    for (int t0 = 0; t0 < nt; t0 += kXT) {
        // packed fp32 (v_pk_add_f32 / v_pk_mul_f32: two IEEE lanes, never fused): acc2[i][h] holds columns j = 2h, 2h+1
        fl_float2 acc2[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc2[i][0] = acc2[i][1] = fl_float2{0.f, 0.f};
        for (int k0 = 0; k0 < dim; k0 += kXK) {
            __syncthreads();
            for (int e = tid; e < kXT * kXK; e += 256) {
                const int r = e / kXK, k = e % kXK;
                const bool kin = k0 + k < dim;
                Qs[k][r] = (kin && q0 + r < nq) ? Q[(size_t)r * dim + k0 + k] : 0.f;
                Ts[k][r] = (kin && t0 + r < nt) ? T[(size_t)(t0 + r) * dim + k0 + k] : 0.f;
            }
            __syncthreads();
#pragma unroll 4
            for (int k = 0; k < kXK; ++k) {
                const f32x4 qv = *(const f32x4*)&Qs[k][4 * tq];  // rows 4 tq + i
                const f32x4 tv = *(const f32x4*)&Ts[k][4 * tt];  // columns 4 tt + j
                const fl_float2 t01 = {tv[0], tv[1]}, t23 = {tv[2], tv[3]};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const fl_float2 qq = {qv[i], qv[i]};
                    const fl_float2 d0 = qq - t01, d1 = qq - t23;
                    acc2[i][0] = acc2[i][0] + d0 * d0;  // unfused, k ascending: contract(off) above
                    acc2[i][1] = acc2[i][1] + d1 * d1;
                }
            }
        }
        float acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[i][0] = acc2[i][0].x; acc[i][1] = acc2[i][0].y;
            acc[i][2] = acc2[i][1].x; acc[i][3] = acc2[i][1].y;
        }
        float dd[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) dd[i][j] = sqrt_cr(acc[i][j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = t0 + 4 * tt + j;
            if (t >= nt) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = dd[i][j];
                if (d < b2[i]) {
                    if (d < b1[i]) { b2[i] = b1[i]; b1[i] = d; j1[i] = t; } else { b2[i] = d; }
                }
            }
        }
        if constexpr (kBoth) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // this thread's 4 rows of column t0 + 4 tt + j (rows past nq excluded), in row order
                float c1 = __builtin_inff(), c2 = __builtin_inff();
                int ci = 0x7fffffff;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = q0 + 4 * tq + i;
                    if (r < nq) {
                        const float d = dd[i][j];
                        if (d < c2) {
                            if (d < c1) { c2 = c1; c1 = d; ci = r; } else { c2 = d; }
                        }
                    }
                }
#pragma unroll
                for (int m = 1; m < 16; m <<= 1) {  // the 16 row threads of this column group: lanes tq ^ m
                    const float o1 = __shfl_xor(c1, m), o2 = __shfl_xor(c2, m);
                    const int oi = __shfl_xor(ci, m);
                    const bool tb = o1 < c1 || (o1 == c1 && oi < ci);
                    const float n2 = tb ? fminf(c1, o2) : fminf(c2, o1);
                    c1 = tb ? o1 : c1;
                    ci = tb ? oi : ci;
                    c2 = n2;
                }
                const int t = t0 + 4 * tt + j;
                if (tq == 0 && t < nt && ci != 0x7fffffff) {
                    ExactTop2* e = colres + (size_t)p * kmax + t;
                    const unsigned long long key =
                        ((unsigned long long)__float_as_uint(c1) << 32) | (unsigned long long)(uint32_t)ci;
                    const unsigned long long old = atomicMin((unsigned long long*)&e->j1, key);
                    const uint32_t oh = (uint32_t)(old >> 32);
                    atomicMin((unsigned int*)&e->d2, umin(umax(oh, __float_as_uint(c1)), __float_as_uint(c2)));
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mb1[tt][4 * tq + i] = b1[i];
        mb2[tt][4 * tq + i] = b2[i];
        mj[tt][4 * tq + i] = j1[i];
    }
    __syncthreads();
    if (tid >= kXT || q0 + tid >= nq) return;
    float c1 = __builtin_inff(), c2 = __builtin_inff();
    int cj = -1;
    for (int u = 0; u < 16; ++u) {
        const float e1 = mb1[u][tid], e2 = mb2[u][tid];
        const int ej = mj[u][tid];
        if (ej < 0) continue;
        if (cj < 0 || e1 < c1 || (e1 == c1 && ej < cj)) {
            c2 = fminf(c1, e2);
            c1 = e1;
            cj = ej;
        } else {
            c2 = fminf(c2, e1);
        }
    }
    (side ? colres : rowres)[(size_t)p * kmax + q0 + tid] = ExactTop2{c1, c2, cj, 1};
}

// Side-1 state of the both-sides pairs before / after fl_exact_tile_kernel<true>: (d2 = +inf, j1 | pad = ~0), then
// d1 from the pad slot and pad = 1 (recomputed), as the per-side kernel leaves its records.
__global__ __launch_bounds__(256) void fl_tile2_init_kernel(const int* __restrict__ counts,
                                                            const int* __restrict__ pairs, int n_pairs, int kmax,
                                                            const int* __restrict__ unc, ExactTop2* __restrict__ colres,
                                                            int fix) {
    const int p = blockIdx.y, t = blockIdx.x * 256 + threadIdx.x;
    if (!fl_both(unc, counts, pairs, n_pairs, p)) return;
    if (t >= counts[pairs[2 * p + 1]]) return;
    ExactTop2* e = colres + (size_t)p * kmax + t;
    if (!fix) {
        *e = ExactTop2{0.f, __builtin_inff(), -1, -1};
    } else {
        const ExactTop2 v = *e;
        *e = ExactTop2{__int_as_float(v.pad), v.d2, v.j1, 1};
    }
}

// Exact rescan of the uncertified keypoints: one 256-thread block per keypoint (block_exact_top2), except those of
// (pair, side)s that fl_exact_tile_kernel recomputes whole.
__global__ __launch_bounds__(kFinThreads) void fl_rescan_kernel(const float* __restrict__ desc,
                                                                const int* __restrict__ counts, int kmax, int dim,
                                                                const int* __restrict__ pairs, int n_pairs,
                                                                const int* __restrict__ redo_count,
                                                                const int4* __restrict__ redo,
                                                                const int* __restrict__ unc,
                                                                ExactTop2* __restrict__ rowres,
                                                                ExactTop2* __restrict__ colres) {
    __shared__ float red_d[2 * kFinThreads];
    __shared__ int red_j[kFinThreads];
    const int n = *redo_count;
    for (int e = blockIdx.x; e < n; e += gridDim.x) {
        const int4 r = redo[e];
        const int side = r.x, p = r.y, i = r.z;
        const int iq = pairs[2 * p + side], it = pairs[2 * p + 1 - side];
        if (fl_use_tile(unc[side * n_pairs + p], counts[iq])) continue;
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
    off[4] = o; o += gtsfm_align_up((size_t)2 * n_pairs * kmax * kFlCand * sizeof(float), 256);  // tkey
    off[5] = o; o += gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);       // rowres
    off[6] = o; o += gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);       // colres
    off[7] = o; o += 256;                                                                     // redo count
    off[8] = o; o += gtsfm_align_up((size_t)2 * n_pairs * kmax * sizeof(int4), 256);        // redo list
    off[9] = o; o += gtsfm_align_up((size_t)2 * n_pairs * sizeof(int), 256);                // uncertified per side
    return o;
}

template <int NS>
int launch_fl_shortlist(const _Float16* form, const float* norm2, const int* counts, const int* pairs, int n_pairs,
                        int kpad, int kmax, int* cand, float* tkey, hipStream_t stream) {
    const size_t lds = 2 * kFlRows * (NS * 16 + 8) * sizeof(_Float16) + 2 * kFlRows * sizeof(float);
    GTSFM_CHECK_HIP(gtsfm_set_dynamic_lds((const void*)fl_shortlist_kernel<NS>, (int)lds));
    const dim3 grid((unsigned)((kpad / kFlQ * (size_t)n_pairs * 2 + 7) / 8 * 8));
    hipLaunchKernelGGL(fl_shortlist_kernel<NS>, grid, dim3(256), lds, stream, form, norm2,
                       counts, pairs, n_pairs, kpad, kmax, cand, tkey);
    return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
}

int run_fl_match(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim, const int* d_pairs,
                 int n_pairs, double ratio, unsigned char* ws, uint32_t* d_out_idx, int* d_out_count,
                 hipStream_t stream) {
    size_t off[10];
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
    int* unc = (int*)(ws + off[9]);
    GTSFM_CHECK_HIP(hipMemsetAsync(maxnorm, 0, 2 * (size_t)n_img * sizeof(unsigned), stream));
    GTSFM_CHECK_HIP(hipMemsetAsync(redo_count, 0, sizeof(int), stream));
    GTSFM_CHECK_HIP(hipMemsetAsync(unc, 0, 2 * (size_t)n_pairs * sizeof(int), stream));
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
    hipLaunchKernelGGL(fl_rerank_kernel, dim3((unsigned)(((2 * (size_t)n_pairs + 7) / 8) * 8 *
                                                ((kmax + kFlRerankRows - 1) / kFlRerankRows))), dim3(256), 0,
                       stream, d_desc, d_counts, kmax, dim, d_pairs, n_pairs, kpad, norm2, maxnorm, unsafe, cand, tkey,
                       rowres, colres, redo_count, redo, unc);
    GTSFM_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(fl_exact_tile_kernel<false>, dim3((kmax + kXT - 1) / kXT, n_pairs, 2), dim3(256), 0, stream,
                       d_desc, d_counts, kmax, dim, d_pairs, n_pairs, unc, rowres, colres);
    hipLaunchKernelGGL(fl_tile2_init_kernel, dim3((kmax + 255) / 256, n_pairs), dim3(256), 0, stream, d_counts,
                       d_pairs, n_pairs, kmax, unc, colres, 0);
    hipLaunchKernelGGL(fl_exact_tile_kernel<true>, dim3((kmax + kXT - 1) / kXT, n_pairs, 1), dim3(256), 0, stream,
                       d_desc, d_counts, kmax, dim, d_pairs, n_pairs, unc, rowres, colres);
    hipLaunchKernelGGL(fl_tile2_init_kernel, dim3((kmax + 255) / 256, n_pairs), dim3(256), 0, stream, d_counts,
                       d_pairs, n_pairs, kmax, unc, colres, 1);
    hipLaunchKernelGGL(fl_rescan_kernel, dim3(2048), dim3(kFinThreads), 0, stream, d_desc, d_counts, kmax, dim,
                       d_pairs, n_pairs, redo_count, redo, unc, rowres, colres);
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
        size_t off[10];
        return fl_layout(n_img, kmax, dim, n_pairs, off);
    }
    return 2 * gtsfm_align_up((size_t)n_pairs * kmax * sizeof(ExactTop2), 256);
}

int gtsfm_match_rerank_stats(const void* d_workspace, size_t workspace_bytes, int n_img, int kmax, int dim,
                             int n_pairs, int* h_uncertified, int* h_uncertified_per_side, void* stream_v) {
    if (!d_workspace || !h_uncertified || n_img <= 0 || kmax <= 0 || dim <= 0 || dim > kFlMaxDim || n_pairs < 0)
        return GTSFM_ERR_ARG;
    size_t off[10];
    if (workspace_bytes < fl_layout(n_img, kmax, dim, n_pairs, off)) return GTSFM_ERR_CAPACITY;
    hipStream_t stream = (hipStream_t)stream_v;
    const unsigned char* ws = (const unsigned char*)d_workspace;
    GTSFM_CHECK_HIP(hipMemcpyAsync(h_uncertified, ws + off[7], sizeof(int), hipMemcpyDeviceToHost, stream));
    if (h_uncertified_per_side && n_pairs)
        GTSFM_CHECK_HIP(hipMemcpyAsync(h_uncertified_per_side, ws + off[9], 2 * (size_t)n_pairs * sizeof(int),
                                       hipMemcpyDeviceToHost, stream));
    GTSFM_CHECK_HIP(hipStreamSynchronize(stream));
    return GTSFM_OK;
}

int gtsfm_match_max_group(int kmax, int dim) {
    if (kmax <= 0 || kmax > kMaxKmaxPacked || dim <= 0 || dim > 139) return 0;
    return pp_max_group(kmax, dim);
}

int gtsfm_match_batched_grouped(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim,
                                const int* d_pairs, int n_pairs, const int* d_groups, int n_groups, int group_size,
                                double ratio, int mode, void* d_workspace, size_t workspace_bytes, uint32_t* d_out_idx,
                                int* d_out_count, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_desc || !d_counts || !d_pairs || !d_out_idx || !d_out_count || n_img <= 0 || kmax <= 0 || dim <= 0 ||
        n_pairs < 0 || kmax > kMaxKmax)
        return GTSFM_ERR_ARG;
    if (d_groups && (n_groups <= 0 || group_size <= 0 || group_size > kMaxGroup)) return GTSFM_ERR_ARG;
    if (workspace_bytes < gtsfm_match_workspace_bytes(n_img, kmax, dim, n_pairs, mode)) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;

    if (mode == GTSFM_MATCH_INT_F16) {
        const int da = pack_da(dim), kpad = pack_kpad(kmax), nk = da / 16, ib = index_bits(kmax);
        if (dim > 139 || kmax > kMaxKmaxPacked) return GTSFM_ERR_ARG;
        if (d_groups && group_size > pp_max_group(kmax, dim)) return GTSFM_ERR_ARG;
        const size_t form_bytes = gtsfm_align_up((size_t)n_img * kpad * da * sizeof(_Float16), 256);
        _Float16* a_form = (_Float16*)ws;
        _Float16* b_form = (_Float16*)(ws + form_bytes);
        const size_t res_bytes = gtsfm_align_up((size_t)n_pairs * kmax * sizeof(uint2), 256);
        uint2* rowres = (uint2*)(ws + 2 * form_bytes);
        uint2* colres = (uint2*)(ws + 2 * form_bytes + res_bytes);
        hipLaunchKernelGGL(pack_code_kernel, dim3(kpad / 4, n_img), dim3(64, 4), 0, stream, d_desc, d_counts, kmax,
                           dim, kpad, da, code_poison(ib), a_form, b_form);
        GTSFM_CHECK_HIP(hipGetLastError());
        const int ng = d_groups ? n_groups : n_pairs, gs = d_groups ? group_size : 1;
        int rc;
        if (g_mnn_events[0]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[0], stream));
        switch (nk) {
            case 2: rc = launch_pp<2>(a_form, b_form, d_counts, d_pairs, n_pairs, d_groups, ng, gs, kpad, kmax, ib, dim, rowres, colres, stream); break;
            case 5: rc = launch_pp<5>(a_form, b_form, d_counts, d_pairs, n_pairs, d_groups, ng, gs, kpad, kmax, ib, dim, rowres, colres, stream); break;
            case 9: rc = launch_pp<9>(a_form, b_form, d_counts, d_pairs, n_pairs, d_groups, ng, gs, kpad, kmax, ib, dim, rowres, colres, stream); break;
            default: return GTSFM_ERR_ARG;
        }
        if (rc != GTSFM_OK) return rc;
        if (g_mnn_events[1]) GTSFM_CHECK_HIP(hipEventRecord(g_mnn_events[1], stream));
        return launch_finalize<kResCodes>(rowres, colres, d_desc, d_counts, d_pairs, n_pairs, kmax, dim, ib, ratio,
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

int gtsfm_match_batched(const float* d_desc, const int* d_counts, int n_img, int kmax, int dim, const int* d_pairs,
                        int n_pairs, double ratio, int mode, void* d_workspace, size_t workspace_bytes,
                        uint32_t* d_out_idx, int* d_out_count, void* stream_v) {
    return gtsfm_match_batched_grouped(d_desc, d_counts, n_img, kmax, dim, d_pairs, n_pairs, nullptr, 0, 0, ratio,
                                       mode, d_workspace, workspace_bytes, d_out_idx, d_out_count, stream_v);
}

}  // extern "C"
