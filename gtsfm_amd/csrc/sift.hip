// SIFT detector-descriptor for batches of same-sized images (gfx950).
//
// Replaces gtsfm/frontend/detector_descriptor/sift.py:27-56: rgb_to_gray_cv (utils/images.py:14-41),
// cv.SIFT_create().detectAndCompute with OpenCV's defaults, cast_to_gtsfm_keypoints (utils/features.py:16-37) and
// Keypoints.get_top_k (keypoints.py:89-110). Arithmetic is the one restated in oracle/sift.c (pinned to the reference's
// OpenCV fixture), including its deterministic exp/sin/cos polynomials and fixed-point histograms, so the HIP path
// and the oracle agree bit for bit; FMA contraction is off for this file (explicit fmaf only).
//
// Pipeline per batch (every launch covers all images of the batch):
//   gray+2x upsample -> per octave: [decimate] + 5 x (row blur -> column blur fused with the DoG difference)
//   -> extrema (26-neighbourhood) -> refinement (thread per candidate, location dedup by atomic bitmap)
//   -> orientation (wave per location, fixed-point LDS histogram) ; then per image top-k by response
//   (radix select + bitonic sort in LDS) -> descriptors only for the kept keypoints (wave per keypoint,
//   fixed-point 360-bin LDS histogram).
// The blur passes are the HBM-bound part: each level is read once per pass through an LDS tile and written once
// (+ the DoG level).
#pragma clang fp contract(off)
#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "common.hpp"

namespace {

constexpr int kLayers = 3;
constexpr int kLevels = kLayers + 3;
constexpr int kDogs = kLayers + 2;
constexpr int kMaxOct = 16;
constexpr int kMaxDevices = 16;
constexpr int kMaxR = 31;
constexpr float kSigma = 1.6f;
constexpr float kInitSigma = 0.5f;
constexpr int kBorder = 5;
constexpr int kMaxInterp = 5;
constexpr int kOriBins = 36;
constexpr float kOriSigFctr = 1.5f;
constexpr float kOriRadius = 3 * kOriSigFctr;
constexpr float kOriPeakRatio = 0.8f;
constexpr float kDescrSclFctr = 3.f;
constexpr float kDescrMagThr = 0.2f;
constexpr float kIntDescrFctr = 512.f;
constexpr float kContrast = 0.04f;
constexpr float kEdge = 10.f;
constexpr float kFixScale = 16777216.0f;  // 2^24

struct Taps {
    float k[kMaxR + 1];
    int r;
};

// ------------------------------------------------------------------ deterministic math (== oracle/sift.c)
__device__ __forceinline__ float exp2_det(float t) {
    if (t < -126.f) return 0.f;
    const float n = floorf(t);
    const float f = t - n;
    float q = fmaf(1.32154867901443053e-06f, f, 1.52527338040598377e-05f);
    q = fmaf(q, f, 1.54035303933816061e-04f);
    q = fmaf(q, f, 1.33335581464284411e-03f);
    q = fmaf(q, f, 9.61812910762847688e-03f);
    q = fmaf(q, f, 5.55041086648215762e-02f);
    q = fmaf(q, f, 2.40226506959100694e-01f);
    q = fmaf(q, f, 6.93147180559945286e-01f);
    q = fmaf(q, f, 1.0f);
    return ldexpf(q, (int)n);
}

__device__ __forceinline__ float exp_det(float x) { return exp2_det(x * 1.4426950408889634f); }

__device__ __forceinline__ void sincos_det(float a, float* s, float* c) {
    const float k = rintf(a * 0.63661977236758134f);
    float r = fmaf(-k, 1.5707963705062866f, a);
    r = fmaf(-k, -4.3711388286737929e-08f, r);
    const float r2 = r * r;
    const float sp =
        fmaf(fmaf(fmaf(-1.9841269841269841e-04f, r2, 8.3333333333333333e-03f), r2, -1.6666666666666667e-01f), r2 * r, r);
    const float cp = fmaf(fmaf(fmaf(fmaf(2.4801587301587302e-05f, r2, -1.3888888888888889e-03f), r2,
                                    4.1666666666666667e-02f), r2, -0.5f), r2, 1.0f);
    const int q = ((int)k) & 3;
    if (q == 0) { *s = sp; *c = cp; }
    else if (q == 1) { *s = cp; *c = -sp; }
    else if (q == 2) { *s = -sp; *c = -cp; }
    else { *s = -cp; *c = sp; }
}

__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * 57.29577951308232f, p3 = -0.3258083974640975f * 57.29577951308232f,
                p5 = 0.1555786518463281f * 57.29577951308232f, p7 = -0.04432655554792128f * 57.29577951308232f;
    const float ax = fabsf(x), ay = fabsf(y);
    // both octants in one evaluation (one division): c = min / (max + eps), a = poly(c) or 90 - poly(c)
    const bool xmaj = ax >= ay;
    const float c = (xmaj ? ay : ax) / ((xmaj ? ax : ay) + (float)DBL_EPSILON);
    const float c2 = c * c;
    const float t = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    float a = xmaj ? t : 90.f - t;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__device__ __forceinline__ float from_fix(unsigned long long v) { return (float)(long long)v * (1.0f / kFixScale); }
// Fixed-point histogram value (long long)(v 2^24) as in oracle/sift.c, for v >= 0 (every contribution is a magnitude
// times non-negative weights), without the signed 64-bit conversion sequence: x = v 2^24 splits exactly into hi = floor(x / 2^32) and lo = x - hi 2^32 (a multiple of ulp(x)
// below 2^32), both truncated by v_cvt_u32_f32 -- the same integer as (long long)x.
__device__ __forceinline__ unsigned long long to_fix_scaled(float x) {  // x = v 2^24 already
    const uint32_t hi = (uint32_t)(x * 2.3283064365386963e-10f);
    const uint32_t lo = (uint32_t)__builtin_fmaf(-(float)hi, 4294967296.0f, x);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long to_fix_nn(float v) { return to_fix_scaled(v * kFixScale); }

__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// ------------------------------------------------------------------ records
struct Cand {
    int img, layer, r, c;
};
struct Refined {
    int img, layer, r, c;
    float xc, xr, xi, contr;
};
struct KeyRec {
    float x, y, size, angle, response, xc, xr, scl;
    int o, layer, r, c;
};

struct LevelTable {  // gauss levels 1..3 of every octave (descriptor stage)
    const float* g[kMaxOct][kLayers];
    int H[kMaxOct], W[kMaxOct];
    size_t img_stride[kMaxOct];
};

// ------------------------------------------------------------------ kernels: pyramid
// Octave-0 base sample: gray conversion (cv::cvtColor fixed point) + 2x INTER_LINEAR upsampling, evaluated on the fly
// by the first blur (gtsfm/frontend/detector_descriptor/sift.py:44-66 -> cv2 SIFT_create().detectAndCompute).
// Separable Gaussian (cv::GaussianBlur, BORDER_REFLECT_101: rows then columns) fused in one pass over a 64 x 64
// output tile: the input tile and its halo are staged once in LDS (interior tiles by LDS-DMA); the row pass (8 outputs
// per thread from one conflict-free ds_read_b64 window, 17 B of LDS reads per output at R = 13) writes its results
// back in place -- the 8 lanes of a row are lanes of one wave whose window reads are all issued before any of its
// writes (LDS executes a wave's operations in order), so no barrier is needed -- and the column pass (16 outputs per thread from one register window) writes the level. Every output is the same fmaf chain as
// the oracle (acc = k0*c; acc = fmaf(kj, l + r, acc)), so the pyramid stays bit-exact.
// kFromU8: the input is the 2x-upsampled gray image, computed from a gray tile of the u8 source staged in LDS.
// Tiles are mapped XCD-contiguously (consecutive workgroups land on different XCDs; each XCD gets a contiguous run
// of tiles so halos are shared through its own L2).
constexpr int kBlurTX = 64;
// Tile height per radius: 64 rows x 4 waves, or for the wide kernels (and the upsampling one) 96 rows x 8 waves, where
// the smaller row-pass halo share pays for the coarser tiling (measured per radius on octave 0).
__host__ __device__ constexpr int blur_ty(int r, bool u8) {
    return u8 ? 96 : (r >= 9 ? 96 : 64);
}
__host__ __device__ constexpr int blur_tyt(int r, bool u8) { return blur_ty(r, u8) == 64 ? 4 : 8; }
constexpr int kBlurRowOut = 8, kBlurRowThr = kBlurTX / kBlurRowOut;  // row pass: outputs per thread, threads per row
typedef float pf2 __attribute__((ext_vector_type(2)));
constexpr int kBlurMaxR = 16;

// LDS row stride of the input tile: >= 64 + 2r and = 2 (mod 8), so the row pass's ds_read_b64 windows (8 lanes per
// row at 32-B steps, four rows per 32-lane group) hit 64 distinct banks
__host__ __device__ constexpr int blur_iwp(int r) { return (kBlurTX + 2 * r + 5) / 8 * 8 + 2; }
__host__ __device__ constexpr int blur_gh(int r) { return (blur_ty(r, true) + 2 * r) / 2 + 4; }
__host__ __device__ constexpr int blur_gw(int r) { return (kBlurTX + 2 * r) / 2 + 4; }
// u8 variant: input tile | per-row upsampling table (float4 per tile row) | gray source tile
__host__ __device__ constexpr int blur_rtab_off(int r) { return ((blur_ty(r, true) + 2 * r) * blur_iwp(r) + 3) / 4 * 4; }
__host__ __device__ constexpr size_t blur_lds_bytes(int r, bool u8) {
    return (size_t)(u8 ? blur_rtab_off(r) + 4 * (blur_ty(r, true) + 2 * r) + blur_gh(r) * blur_gw(r)
                       : (blur_ty(r, false) + 2 * r) * blur_iwp(r)) *
           sizeof(float);
}

// INTER_LINEAR 2x source coordinate of output index x (cv::resize, half-pixel centres, clamped at the border)
__device__ __forceinline__ void up_coord(int x, int W, int& s0, int& s1, float& f) {
    float fx = (float)((x + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) { sx = 0; fx = 0; }
    if (sx >= W - 1) { sx = W - 1; fx = 0; }
    s0 = sx;
    s1 = sx + 1 < W ? sx + 1 : W - 1;
    f = fx;
}

template <int R, bool kFromU8>
__global__ __launch_bounds__(kBlurTX* blur_tyt(R, kFromU8)) void blur2d_kernel(const float* __restrict__ src,
                                                                  const uint8_t* __restrict__ img8, int C, int H0,
                                                                  int W0, float* __restrict__ dst,
                                                                  float* __restrict__ dec, int H, int W, int n_tx,
                                                                  int n_ty, int n_img, Taps t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int kBlurTY = blur_ty(R, kFromU8), kBlurTYT = blur_tyt(R, kFromU8), kBlurColRows = kBlurTY / kBlurTYT;
    constexpr int IW = kBlurTX + 2 * R, IH = kBlurTY + 2 * R, IWP = blur_iwp(R);
    constexpr int NV = (kBlurRowOut + 2 * R) / 2;  // float2 words per row-pass window
    static_assert((kBlurRowThr - 1) * kBlurRowOut + 2 * NV <= IWP, "row-pass window past the LDS row");
    float* in = lds;  // IH x IWP: input tile, then (columns 0..63) the row-blurred tile
    const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * kBlurTX + tx;
    // XCD-contiguous tile order
    const int total = n_tx * n_ty * n_img;
    const int per_xcd = (total + 7) / 8;
    const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= total) return;
    const int b = tile / (n_tx * n_ty);
    const int rem = tile - b * n_tx * n_ty;
    const int x0 = (rem % n_tx) * kBlurTX, y0 = (rem / n_tx) * kBlurTY;
    const size_t base = (size_t)b * H * W;
    float k[R + 1];
#pragma unroll
    for (int j = 0; j <= R; ++j) k[j] = t.k[j];
    int xx[(IW + kBlurTX - 1) / kBlurTX];
#pragma unroll
    for (int q = 0; q < (IW + kBlurTX - 1) / kBlurTX; ++q) xx[q] = reflect101(x0 - R + tx + q * kBlurTX, W);
    if constexpr (kFromU8) {
        float4* rtab = (float4*)(in + blur_rtab_off(R));  // per tile row: gray row offsets of sy0 / sy1, fy, 1 - fy
        float* g = in + blur_rtab_off(R) + 4 * IH;
        constexpr int GW = blur_gw(R);
        const int ylo = max(y0 - R, 0), yhi = min(y0 + kBlurTY + R, H) - 1;
        const int xlo = max(x0 - R, 0), xhi = min(x0 + kBlurTX + R, W) - 1;
        const int gy0 = max((ylo - 1) / 2, 0), gy1 = min(yhi / 2 + 1, H0 - 1);
        const int gx0 = max((xlo - 1) / 2, 0), gx1 = min(xhi / 2 + 1, W0 - 1);
        const uint8_t* s8 = img8 + (size_t)b * H0 * W0 * C;
        {
            // gray = cv::cvtColor's fixed point (R 4899 + G 9617 + B 1868 + 2^13) >> 14; every byte load of the tile is
            // issued before any is converted (one HBM round trip per block instead of one per pixel row)
            constexpr int NGR = (blur_gh(R) + kBlurTYT - 1) / kBlurTYT;
            float gv[NGR];
            const int gx = gx0 + tx;
            if (C == 1) {
                uint32_t b0[NGR];
#pragma unroll
                for (int i = 0; i < NGR; ++i) {
                    const int gy = min(gy0 + ty + i * kBlurTYT, gy1);
                    b0[i] = s8[(size_t)gy * W0 + min(gx, gx1)];
                }
#pragma unroll
                for (int i = 0; i < NGR; ++i) gv[i] = (float)b0[i];
            } else {
                uint32_t b0[NGR], b1[NGR], b2[NGR];
#pragma unroll
                for (int i = 0; i < NGR; ++i) {
                    const int gy = min(gy0 + ty + i * kBlurTYT, gy1);
                    const uint8_t* px = s8 + ((size_t)gy * W0 + min(gx, gx1)) * 3;
                    b0[i] = px[0];
                    b1[i] = px[1];
                    b2[i] = px[2];
                }
#pragma unroll
                for (int i = 0; i < NGR; ++i)
                    gv[i] = (float)((b0[i] * 4899 + b1[i] * 9617 + b2[i] * 1868 + (1 << 13)) >> 14);
            }
#pragma unroll
            for (int i = 0; i < NGR; ++i) {
                const int gy = gy0 + ty + i * kBlurTYT;
                if (gy <= gy1 && gx <= gx1) g[(gy - gy0) * GW + tx] = gv[i];
            }
        }
        if (tid < IH) {  // the row half of the upsampling coordinates, once per tile row
            int sy0, sy1;
            float fy;
            up_coord(reflect101(y0 - R + tid, H), H0, sy0, sy1, fy);
            rtab[tid] = make_float4(__int_as_float((sy0 - gy0) * GW), __int_as_float((sy1 - gy0) * GW), fy, 1.f - fy);
        }
        __syncthreads();
        constexpr int NQ = (IW + kBlurTX - 1) / kBlurTX;
        int cx0[NQ], cx1[NQ];
        float cfx[NQ], cfx1[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            up_coord(xx[q], W0, cx0[q], cx1[q], cfx[q]);
            cx0[q] -= gx0;
            cx1[q] -= gx0;
            cfx1[q] = 1.f - cfx[q];
        }
        for (int iy = ty; iy < IH; iy += kBlurTYT) {
            const float4 rt = rtab[iy];  // same address across the wave: broadcast
            const float* r0p = g + __float_as_int(rt.x);
            const float* r1p = g + __float_as_int(rt.y);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int ix = tx + q * kBlurTX;
                if (ix < IW) {
                    const float r0 = r0p[cx0[q]] * cfx1[q] + r0p[cx1[q]] * cfx[q];
                    const float r1 = r1p[cx0[q]] * cfx1[q] + r1p[cx1[q]] * cfx[q];
                    in[iy * IWP + ix] = r0 * rt.w + r1 * rt.z;
                }
            }
        }
    } else if (x0 - R >= 0 && x0 + kBlurTX + R <= W && y0 - R >= 0 && y0 + kBlurTY + R <= H) {
        // interior tile: rows straight from HBM into LDS (global_load_lds, no VGPR round trip, no ds_write)
        const float* srow0 = src + base + (size_t)(y0 - R) * W + (x0 - R) + tx;
        for (int iy = ty; iy < IH; iy += kBlurTYT) {
            const float* g = srow0 + (size_t)iy * W;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                             (__attribute__((address_space(3))) void*)(in + iy * IWP), 4, 0, 0);
            if (tx < IW - kBlurTX)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + kBlurTX),
                                                 (__attribute__((address_space(3))) void*)(in + iy * IWP + kBlurTX),
                                                 4, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        // border tile (reflected halo): every load of the tile issued before any LDS store
        constexpr int NR = (IH + kBlurTYT - 1) / kBlurTYT, NQ = (IW + kBlurTX - 1) / kBlurTX;
        float v[NR][NQ];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int iy = ty + i * kBlurTYT;
            const float* srow = src + base + (size_t)reflect101(min(y0 - R + iy, y0 + IH - 1 - R), H) * W;
#pragma unroll
            for (int q = 0; q < NQ; ++q) v[i][q] = (iy < IH && tx + q * kBlurTX < IW) ? srow[xx[q]] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int iy = ty + i * kBlurTYT;
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                if (iy < IH && tx + q * kBlurTX < IW) in[iy * IWP + tx + q * kBlurTX] = v[i][q];
        }
    }
    __syncthreads();
    // row pass: kBlurRowThr threads per row (consecutive lanes of one wave), kBlurRowOut consecutive outputs each,
    // written back in place at columns [g8, g8 + 8) (output column x sits at input column x + R)
    for (int iy = tid / kBlurRowThr; iy < IH; iy += kBlurTX * kBlurTYT / kBlurRowThr) {
        const int g8 = (tid % kBlurRowThr) * kBlurRowOut;
        float* rowp = in + iy * IWP;
        // volatile 8-byte reads: the compiler would otherwise pair them into ds_read2_b64, which banks by 16-lane
        // groups mod 32 dwords (two rows x 8 lanes at an 8-dword stride: 2-way conflicts); ds_read_b64 banks by
        // 32-lane groups mod 64, where the row stride IWP = 2 (mod 8) keeps the four rows' windows conflict-free
        typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
        lds_u64* wp = (lds_u64*)(rowp + g8);
        float v[2 * NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const unsigned long long w2 = wp[q];
            v[2 * q] = __uint_as_float((uint32_t)w2); v[2 * q + 1] = __uint_as_float((uint32_t)(w2 >> 32));
        }
        asm volatile("" ::: "memory");  // all window reads issue before the in-place writes (neighbour lanes' windows)
        // two outputs per packed-fp32 op (v_pk_add_f32 / v_pk_fma_f32); per-lane rounding unchanged
        // tap-major over the output pairs (independent neighbours between dependent packed ops: no hazard NOPs)
        pf2 o[kBlurRowOut / 2];
#pragma unroll
        for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = pf2{k[0], k[0]} * pf2{v[R + 2 * h], v[R + 2 * h + 1]};
#pragma unroll
        for (int j = 1; j <= R; ++j) {
            pf2 sm[kBlurRowOut / 2];
#pragma unroll
            for (int h = 0; h < kBlurRowOut / 2; ++h)
                sm[h] = pf2{v[R + 2 * h - j], v[R + 2 * h + 1 - j]} + pf2{v[R + 2 * h + j], v[R + 2 * h + 1 + j]};
#pragma unroll
            for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm[h], o[h]);
        }
#pragma unroll
        for (int h = 0; h < kBlurRowOut / 2; ++h) *(float2*)(rowp + g8 + 2 * h) = make_float2(o[h].x, o[h].y);
    }
    __syncthreads();
    // column pass: kBlurColRows consecutive outputs per thread
    const int x = x0 + tx;
    if (x >= W) return;
    const int ly0 = ty * kBlurColRows;
    float c[kBlurColRows + 2 * R];
#pragma unroll
    for (int i = 0; i < kBlurColRows + 2 * R; ++i) c[i] = in[(ly0 + i) * IWP + tx];
    // tap-major: the kBlurColRows / 2 output pairs' chains advance together (independent neighbours between dependent
    // packed ops, so no hazard NOPs); each output's operation order is unchanged
    constexpr int NP = kBlurColRows / 2;
    pf2 acc[NP];
#pragma unroll
    for (int h = 0; h < NP; ++h) acc[h] = pf2{k[0], k[0]} * pf2{c[R + 2 * h], c[R + 2 * h + 1]};
#pragma unroll
    for (int j = 1; j <= R; ++j) {
        pf2 sm[NP];
#pragma unroll
        for (int h = 0; h < NP; ++h)
            sm[h] = pf2{c[R + 2 * h - j], c[R + 2 * h + 1 - j]} + pf2{c[R + 2 * h + j], c[R + 2 * h + 1 + j]};
#pragma unroll
        for (int h = 0; h < NP; ++h) acc[h] = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm[h], acc[h]);
    }
    // output rows y0 + ly0 + 2h (even: tiles and ly0 are) and the next; running store pointers
    float* dp = dst + base + (size_t)(y0 + ly0) * W + x;
    const int rows_left = H - (y0 + ly0);  // rows of this thread's outputs inside the image
    if (rows_left >= kBlurColRows && dec == nullptr) {
#pragma unroll
        for (int h = 0; h < NP; ++h) {
            dp[0] = acc[h].x;
            dp[W] = acc[h].y;
            dp += 2 * (size_t)W;
        }
        return;
    }
    // the image's last tile row, or the one level per octave that also writes the next octave's base (dec:
    // cv::resize INTER_NEAREST to (H/2, W/2) of this level, pixel (2y', 2x'))
    const bool dec_lane = dec != nullptr && (x & 1) == 0 && (x >> 1) < (W >> 1);
    float* decp = dec_lane ? dec + (size_t)b * (H >> 1) * (W >> 1) + (size_t)((y0 + ly0) >> 1) * (W >> 1) + (x >> 1)
                           : nullptr;
#pragma unroll
    for (int h = 0; h < NP; ++h) {
        if (2 * h < rows_left) dp[0] = acc[h].x;
        if (2 * h + 1 < rows_left) dp[W] = acc[h].y;
        dp += 2 * (size_t)W;
        if (decp != nullptr) {
            const int y = y0 + ly0 + 2 * h;
            if (y < H && (y >> 1) < (H >> 1)) *decp = acc[h].x;
            decp += W >> 1;
        }
    }
}

// Streaming variant of the float-input blur: one wave per (image, 64-column strip, row segment), no tile barriers.
// Input rows arrive 8 at a time (a chunk) by global_load_lds into a per-wave LDS ring of kStreamPD + 1 chunks, issued
// kStreamPD chunks ahead; each chunk is row-blurred in place (the row pass of blur2d_kernel) and every lane then takes
// its own column of the 8 row-blurred values into a register window of M = 1 + ceil(2R / 8) chunks, so the vertical
// halo is kept across chunks instead of being re-read and re-blurred per tile. From the M-th chunk on, each chunk
// completes 8 output rows, and the column pass emits them from the window. Same fmaf chains as blur2d_kernel (row
// pass identical; column pass acc = k0 c_y, acc = fma(kj, c_{y-j} + c_{y+j}, acc)), so the output is bit-identical.
__host__ __device__ constexpr int blur_stream_m(int r) { return 1 + (2 * r + 7) / 8; }
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}
constexpr int kStreamWaves = 4, kStreamPD = 2, kStreamBufs = kStreamPD + 1;
// Octave 0 of C2, per level (us, tiled / streaming): r 5: 1289 / 1455, r 6: 1332 / 1442, r 8: 1635 / 1507,
// r 10: 1902 / 1467, r 13: 1996 / 1697 (profiles/r05x_*): the tiles stay at their HBM bound for narrow kernels, and
// the streaming form wins once the row-pass halo and tile-phase serialisation dominate.
constexpr int kBlurStreamMinR = 8;
__host__ __device__ constexpr size_t blur_stream_lds_bytes(int r) {
    return (size_t)kStreamWaves * kStreamBufs * 8 * blur_iwp(r) * sizeof(float);
}

template <int R>
__global__ __launch_bounds__(64 * kStreamWaves) void blur_stream_kernel(const float* __restrict__ src,
                                                                        float* __restrict__ dst,
                                                                        float* __restrict__ dec, int H, int W,
                                                                        int n_strips, int n_parts, int n_img,
                                                                        Taps t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int M = blur_stream_m(R);
    constexpr int IW = kBlurTX + 2 * R, IWP = blur_iwp(R), CH = 8 * IWP;
    constexpr int NV = (kBlurRowOut + 2 * R) / 2;
    static_assert(8 * (M - 1) >= 2 * R, "the window must cover the halo");
    static_assert((kBlurRowThr - 1) * kBlurRowOut + 2 * NV <= IWP, "row-pass window past the LDS row");
    static_assert(IW <= 2 * kBlurTX, "two load columns per row");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // A strip's 8-row groups of every image, taken in (image, row) order, are cut into n_parts equal runs, one per wave
    // (a run that crosses an image boundary restarts the window there). XCD-contiguous unit order, strip fastest:
    // neighbouring strips (shared halo columns) run on one XCD at about the same rows. The unit is wave-uniform, so
    // everything derived from it stays in scalar registers.
    const int n_blocks = gridDim.x, per_xcd = n_blocks >> 3;
    const int u = __builtin_amdgcn_readfirstlane((((blockIdx.x & 7) * per_xcd) + (blockIdx.x >> 3)) * kStreamWaves +
                                                 wave);
    if (u >= n_strips * n_parts) return;
    const int strip = u % n_strips, part = u / n_strips;
    const int x0 = strip * kBlurTX;
    const int G = (H + 7) / 8, BG = n_img * G;
    const int g_beg = (int)((long long)part * BG / n_parts), g_end = (int)((long long)(part + 1) * BG / n_parts);
    float* ring = lds + __builtin_amdgcn_readfirstlane(wave) * (kStreamBufs * CH);
    float k[R + 1];
#pragma unroll
    for (int j = 0; j <= R; ++j) k[j] = t.k[j];
    const uint32_t oa = 4u * (uint32_t)reflect101(x0 - R + lane, W);
    const uint32_t ob = 4u * (uint32_t)reflect101(x0 - R + kBlurTX + lane, W);
    for (int g = g_beg; g < g_end;) {
        const int b = g / G, gy0 = g - b * G, gy1 = min(G, gy0 + (g_end - g));
        g += gy1 - gy0;
        const int ys = 8 * gy0, ye = min(H, 8 * gy1);
        // chunk c = input rows base + 8c .. + 7 (reflect-101 outside the image); chunk c >= M - 1 completes output rows
        // ys + 8 (c - M + 1) .. + 7
        const int base = ys + R - 8 * (M - 1);
        const int n_chunks = (ye - ys + 7) / 8 + M - 1;
        const float* img = src + (size_t)b * H * W;
        // global_load_lds_dword (saddr form: scalar row base, the lane's byte offset), issued by inline asm: the compiler's
        // own LDS-DMA tracking would wait for every chunk in flight before each chunk's LDS accesses; the waits here are
        // explicit. 16 load instructions per chunk, always issued (chunks past the segment reload valid rows). The LDS
        // address goes in as an M0 operand ("{m0}" constraint): the compiler writes M0 itself and knows the asm reads
        // it, so no register it keeps live can alias M0 (tests/test_build_isa.py checks the built code object); the
        // s_nop covers the M0-write -> LDS-DMA hazard.
        auto issue = [&](int c) {
            const uint32_t d = __builtin_amdgcn_readfirstlane(
                (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(ring + (c % kStreamBufs) * CH));
            const int r0 = base + 8 * c;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const float* row = img + (size_t)reflect101(r0 + r, H) * W;
                const uint32_t la = d + 4u * r * IWP;
                asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(oa), "s"(row), "{m0}"(la) : "memory");
                if (lane < IW - kBlurTX)
                    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(ob), "s"(row), "{m0}"(la + 4u * kBlurTX)
                                 : "memory");
            }
        };
        float win[8 * M];  // chunk c's column values at win[8 (c mod M) ..]
        const int x = x0 + lane;
        const bool dec_lane = dec != nullptr && (x & 1) == 0 && (x >> 1) < (W >> 1);
        float* decb = dec_lane ? dec + (size_t)b * (H >> 1) * (W >> 1) + (x >> 1) : nullptr;
        // chunk c with c mod M = K (static): wait for its rows (the kStreamPD younger chunks' loads stay in flight; stores
        // issued in between only make the wait stricter), row-blur in place, take column `lane` into the window, then (c >=
        // M - 1) the column pass for output rows y = ys + 8 (c - M + 1) + o: input row y + d sits (o + d - R) rows from
        // chunk c's first row, i.e. in chunk K + floor((o + d - R) / 8) (mod M), row (o + d - R) mod 8
        auto chunk = [&](int c, auto kc) {
            constexpr int K = decltype(kc)::value;
            issue(c + kStreamPD);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 * kStreamPD) : "memory");
            float* in = ring + (c % kStreamBufs) * CH;
            {
                const int g8 = (lane % kBlurRowThr) * kBlurRowOut;
                float* rowp = in + (lane / kBlurRowThr) * IWP;
                typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
                lds_u64* wp = (lds_u64*)(rowp + g8);
                float v[2 * NV];
#pragma unroll
                for (int q = 0; q < NV; ++q) {
                    const unsigned long long w2 = wp[q];
                    v[2 * q] = __uint_as_float((uint32_t)w2); v[2 * q + 1] = __uint_as_float((uint32_t)(w2 >> 32));
                }
                asm volatile("" ::: "memory");
                pf2 o[kBlurRowOut / 2];
#pragma unroll
                for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = pf2{k[0], k[0]} * pf2{v[R + 2 * h], v[R + 2 * h + 1]};
#pragma unroll
                for (int j = 1; j <= R; ++j) {
                    pf2 sm[kBlurRowOut / 2];
#pragma unroll
                    for (int h = 0; h < kBlurRowOut / 2; ++h)
                        sm[h] = pf2{v[R + 2 * h - j], v[R + 2 * h + 1 - j]} + pf2{v[R + 2 * h + j], v[R + 2 * h + 1 + j]};
#pragma unroll
                    for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm[h], o[h]);
                }
#pragma unroll
                for (int h = 0; h < kBlurRowOut / 2; ++h) *(float2*)(rowp + g8 + 2 * h) = make_float2(o[h].x, o[h].y);
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int r = 0; r < 8; ++r) win[8 * K + r] = in[r * IWP + lane];
            if (c < M - 1) return;
            auto slot = [](int off) {  // off = o + d - R in [-2R, 7]
                const int q = (off + 8 * M) / 8 - M;  // floor(off / 8)
                return 8 * ((K + q + M) % M) + (off - 8 * q);
            };
            const int y_base = ys + 8 * (c - M + 1);
            float* dp = dst + (size_t)b * H * W + (size_t)y_base * W + x;
#pragma unroll
            for (int o = 0; o < 8; o += 2) {
                pf2 acc = pf2{k[0], k[0]} * pf2{win[slot(o - R)], win[slot(o + 1 - R)]};
#pragma unroll
                for (int j = 1; j <= R; ++j) {
                    const pf2 sm = pf2{win[slot(o - R - j)], win[slot(o + 1 - R - j)]} +
                                   pf2{win[slot(o - R + j)], win[slot(o + 1 - R + j)]};
                    acc = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm, acc);
                }
                const int y = y_base + o;
                if (x < W) {
                    if (y < ye) dp[(size_t)o * W] = acc.x;
                    if (y + 1 < ye) dp[(size_t)(o + 1) * W] = acc.y;
                }
                if (decb != nullptr && y < ye && (y >> 1) < (H >> 1)) decb[(size_t)(y >> 1) * (W >> 1)] = acc.x;
            }
        };
#pragma unroll
        for (int c = 0; c < kStreamPD; ++c) issue(c);
        // M chunks per iteration: the window slots stay static
        for (int c = 0; c < n_chunks; c += M)
            static_for<M>([&](auto kc) {
                if (c + decltype(kc)::value < n_chunks) chunk(c + decltype(kc)::value, kc);
            });
        // the prefetched chunks land before the next run reuses the ring (and before the wave retires)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

using BlurStreamFn = void (*)(const float*, float*, float*, int, int, int, int, int, Taps);
BlurStreamFn blur_stream_get(int r) {
    switch (r) {
#define GTSFM_BLURS_CASE(RR) \
    case RR:                 \
        return blur_stream_kernel<RR>;
        GTSFM_BLURS_CASE(1) GTSFM_BLURS_CASE(2) GTSFM_BLURS_CASE(3) GTSFM_BLURS_CASE(4) GTSFM_BLURS_CASE(5)
        GTSFM_BLURS_CASE(6) GTSFM_BLURS_CASE(7) GTSFM_BLURS_CASE(8) GTSFM_BLURS_CASE(9) GTSFM_BLURS_CASE(10)
        GTSFM_BLURS_CASE(11) GTSFM_BLURS_CASE(12) GTSFM_BLURS_CASE(13) GTSFM_BLURS_CASE(14) GTSFM_BLURS_CASE(15)
        GTSFM_BLURS_CASE(16)
#undef GTSFM_BLURS_CASE
        default:
            return nullptr;
    }
}

// Row pass of one 8-row chunk held in LDS (row stride IWP, input column x + R for output column x), in place: 8
// threads per row, 8 outputs each, the same packed fmaf chains and window reads as blur_stream_kernel's row pass.
template <int R, int IWP>
__device__ __forceinline__ void row_blur_chunk(float* chunk, const float (&k)[R + 1], int lane) {
    constexpr int NV = (kBlurRowOut + 2 * R) / 2;
    static_assert((kBlurRowThr - 1) * kBlurRowOut + 2 * NV <= IWP, "row-pass window past the LDS row");
    const int g8 = (lane % kBlurRowThr) * kBlurRowOut;
    float* rowp = chunk + (lane / kBlurRowThr) * IWP;
    typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
    lds_u64* wp = (lds_u64*)(rowp + g8);
    float v[2 * NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const unsigned long long w2 = wp[q];
        v[2 * q] = __uint_as_float((uint32_t)w2); v[2 * q + 1] = __uint_as_float((uint32_t)(w2 >> 32));
    }
    asm volatile("" ::: "memory");
    pf2 o[kBlurRowOut / 2];
#pragma unroll
    for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = pf2{k[0], k[0]} * pf2{v[R + 2 * h], v[R + 2 * h + 1]};
#pragma unroll
    for (int j = 1; j <= R; ++j) {
        pf2 sm[kBlurRowOut / 2];
#pragma unroll
        for (int h = 0; h < kBlurRowOut / 2; ++h)
            sm[h] = pf2{v[R + 2 * h - j], v[R + 2 * h + 1 - j]} + pf2{v[R + 2 * h + j], v[R + 2 * h + 1 + j]};
#pragma unroll
        for (int h = 0; h < kBlurRowOut / 2; ++h) o[h] = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm[h], o[h]);
    }
#pragma unroll
    for (int h = 0; h < kBlurRowOut / 2; ++h) *(float2*)(rowp + g8 + 2 * h) = make_float2(o[h].x, o[h].y);
    asm volatile("" ::: "memory");
}

// Column pass over a three-chunk register window (8 rows per chunk, chunk slots rotating mod 3, the newest chunk in
// slot J): the 8 outputs of the middle chunk, acc = k0 c_y, acc = fma(kj, c_{y-j} + c_{y+j}, acc) (R <= 8).
template <int R, int J>
__device__ __forceinline__ void col_blur_window(const float (&win)[24], const float (&k)[R + 1], float (&out)[8]) {
    static_assert(R <= 8, "the halo fits the neighbouring chunks");
    auto slot = [](int off) {  // off = output row offset + tap in [-R, 7 + R], relative to the middle chunk's first row
        const int q = (off + 16) / 8 - 2;  // floor(off / 8) in {-1, 0, 1}
        return 8 * ((J - 1 + q + 6) % 3) + (off - 8 * q);
    };
#pragma unroll
    for (int o = 0; o < 8; o += 2) {
        pf2 acc = pf2{k[0], k[0]} * pf2{win[slot(o)], win[slot(o + 1)]};
#pragma unroll
        for (int j = 1; j <= R; ++j) {
            const pf2 sm = pf2{win[slot(o - j)], win[slot(o + 1 - j)]} + pf2{win[slot(o + j)], win[slot(o + 1 + j)]};
            acc = __builtin_elementwise_fma(pf2{k[j], k[j]}, sm, acc);
        }
        out[o] = acc.x;
        out[o + 1] = acc.y;
    }
}

// Octave 0's base level as a streaming pass from the gray bytes (no upsampled image in memory, no tile barriers):
//   G0 = GaussianBlur_{sig_diff}(resize_2x(gray(image)))
// (sift.py:44-66 -> cv::SIFT createInitialImage). gray_pad_kernel first writes the gray image (cv::cvtColor's fixed
// point for RGB) with a padded row pitch; then one wave per (image, row segment, 64-column strip), lane = G0 column.
// Per 8-row chunk of upsampled rows: the chunk's gray source rows (at most 6, 48 aligned bytes each) arrive in a
// per-wave LDS slot by LDS-DMA issued two chunks ahead; the upsampled rows (INTER_LINEAR 2x: gray integers times
// quarter weights, so every product and sum is exact in fp32 in any order) are written to an LDS chunk, row-blurred in
// place, and each lane takes its column into a three-chunk window whose column pass gives the lane's 8 G0 values one
// chunk later. Every fmaf chain is the one blur2d_kernel<5, true> evaluates (reflect-101 rows and columns past the
// image edge compute the mirrored pixel's value bit for bit), so the pyramid is unchanged.
// Octave 0 of C2 (100 x 3840 x 2160 from RGB): 0.99 ms + 0.20 ms gray staging, against 1.82 ms for the upsampling tile
// kernel (profiles/r06j_*; with the source bytes prefetched one chunk ahead into registers instead, the compiler's
// vmcnt(0) at every chunk left it at 1.13 ms). Measured and not kept: the same wave also running G1's row and column
// passes on its G0 chunks (strips of 54 G1 columns, no G0 re-read): 179 VGPRs, 2 waves per SIMD, 3.5 ms for both
// levels (4.2 ms with spills at 128 VGPRs) against about 2.3 ms as two launches -- the serial LDS round trips of two
// blur stages per chunk need more waves in flight than that register budget leaves.
// The kernel is OpenCV's for its default sigma (1.6, 3 layers, input sigma 0.5): sig_diff = 1.249, 11 taps, compiled
// in (literal operands); the host takes this path only when the taps it computed for the call are these bits.
constexpr int kBaseR = 5;
constexpr float kBaseTaps[kBaseR + 1] = {0x1.4713ccp-2f, 0x1.dac53p-3f,   0x1.6b0372p-4f,
                                         0x1.2469fap-6f, 0x1.f04b72p-10f, 0x1.bbb2a4p-14f};
// Gray source rows are staged with a padded pitch (kBasePitchPad bytes past the row, rounded to 64) so that every
// chunk's source window -- 12 aligned dwords from the strip's first source column rounded down to 4 -- is one
// in-bounds, aligned read per dword.
constexpr int kBaseRowDw = 12;                 // dwords per staged source row: >= ((64 + 2 R) / 2 + 3 + 3) / 4
constexpr int kBaseRowB = 4 * kBaseRowDw;      // LDS ring row stride (bytes)
constexpr int kBaseRingRows = 6;               // source rows of one chunk
constexpr int kBasePD = 2;                     // chunks prefetched ahead
constexpr int kBasePitchPad = kBaseRowB;
constexpr int kBaseWaveFloats = (kBasePD + 1) * kBaseRingRows * kBaseRowDw + 8 * blur_iwp(kBaseR);
__host__ __device__ constexpr int base_pitch(int w0) { return (w0 + kBasePitchPad + 63) / 64 * 64; }

// cv::cvtColor RGB -> gray fixed point, (R 4899 + G 9617 + B 1868 + 2^13) >> 14 (C = 3), or a copy (C = 1), into rows of
// base_pitch(W0) bytes (zero padded): one thread per 4 output bytes of a row, one dword store; the source as C aligned
// dwords when the source rows are dword aligned (`aligned`: base address and W0 C both multiples of 4) and the 4
// pixels lie inside the row, else byte by byte.
__device__ __forceinline__ uint32_t cv_gray(uint32_t r, uint32_t g, uint32_t b) {
    return (r * 4899u + g * 9617u + b * 1868u + (1u << 13)) >> 14;
}
template <int C>
__global__ __launch_bounds__(256) void gray_pad_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ gray,
                                                       int n_rows, int W0, int pitch, int aligned) {
    const int dw_per_row = pitch / 4;
    const long long n = (long long)n_rows * dw_per_row;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int row = (int)(i / dw_per_row), x0 = 4 * (int)(i - (long long)row * dw_per_row);
        const uint8_t* s = src + ((size_t)row * W0 + x0) * C;
        uint32_t out = 0;
        if (aligned && x0 + 4 <= W0) {
            const uint32_t* w = (const uint32_t*)s;
            if constexpr (C == 1) {
                out = w[0];
            } else {
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                out = cv_gray(w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255) |
                      cv_gray(w0 >> 24, w1 & 255, (w1 >> 8) & 255) << 8 |
                      cv_gray((w1 >> 16) & 255, w1 >> 24, w2 & 255) << 16 |
                      cv_gray((w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24) << 24;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (x0 + q < W0) out |= (C == 1 ? s[q] : cv_gray(s[C * q], s[C * q + 1 % C], s[C * q + 2 % C])) << (8 * q);
        }
        ((uint32_t*)gray)[i] = out;
    }
}

__global__ __launch_bounds__(64 * kStreamWaves) __attribute__((amdgpu_waves_per_eu(4))) void base_stream_kernel(
    const uint8_t* __restrict__ gray8, int H0, int W0, int pitch, float* __restrict__ g0, float* __restrict__ sink,
    int H, int W, int n_strips, int n_seg, int n_img) {
    constexpr int R1 = kBaseR, IW1 = 64 + 2 * R1, IWP1 = blur_iwp(R1), WF = kBaseWaveFloats;
    // chunk j holds upsampled rows ys - kLead + 8 j ..; its G0 chunk (the middle one of the window) starts 8 rows earlier
    constexpr int kLead = 8;
    constexpr int kItems = kBaseRingRows * kBaseRowDw;
    static_assert(IW1 <= 128 && (IW1 / 2 + 3) + 3 <= kBaseRowB, "one extra column per lane; the source span fits");
    static_assert(kItems <= 2 * 64, "two dword loads per lane cover a chunk's source rows");
    __shared__ __attribute__((aligned(16))) float lds[kStreamWaves * WF];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n_blocks = gridDim.x, per_xcd = n_blocks >> 3;
    const int u = __builtin_amdgcn_readfirstlane((((blockIdx.x & 7) * per_xcd) + (blockIdx.x >> 3)) * kStreamWaves +
                                                 wave);
    if (u >= n_strips * n_seg * n_img) return;
    const int strip = u % n_strips, part = u / n_strips;
    const int b = part / n_seg, seg = part - b * n_seg;
    const int G8 = (H + 7) / 8;
    const int ys = 8 * (int)((long long)seg * G8 / n_seg);
    const int ye = min(H, 8 * (int)((long long)(seg + 1) * G8 / n_seg));
    if (ys >= ye) return;
    const int s0 = strip * 64;
    float* wl = lds + __builtin_amdgcn_readfirstlane(wave) * WF;
    float* ring = wl;  // kBasePD + 1 slots of a chunk's source rows (kBaseRowB bytes each), filled by LDS-DMA
    float* ch1 = wl + (kBasePD + 1) * kBaseRingRows * kBaseRowDw;  // upsampled chunk, then its row blur
    float k1[R1 + 1];
#pragma unroll
    for (int j = 0; j <= R1; ++j) k1[j] = kBaseTaps[j];

    // upsampled columns of this lane, as a (set a, set b) pair: s0 - R1 + lane and (lanes < IW1 - 64) s0 - R1 + 64 + lane
    const bool has_b = lane < IW1 - 64;
    int ca0, ca1, cb0, cb1;
    float fa, fb;
    up_coord(reflect101(s0 - R1 + lane, W), W0, ca0, ca1, fa);
    up_coord(reflect101(s0 - R1 + 64 + (has_b ? lane : 0), W), W0, cb0, cb1, fb);
    int gx0 = has_b ? min(ca0, cb0) : ca0;
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) gx0 = min(gx0, __shfl_xor(gx0, m));
    const int a0 = __builtin_amdgcn_readfirstlane(gx0) & ~3;  // first staged source column (dword aligned)
    ca0 -= a0; ca1 -= a0; cb0 -= a0; cb1 -= a0;
    const pf2 fx = {fa, fb}, fx1 = {1.f - fa, 1.f - fb};
    // staged item i (lane + 64 q) = dword i % kBaseRowDw of source row lo + i / kBaseRowDw (clamped to the image: rows
    // past a border chunk's range are loaded but not read)
    const uint8_t* src = gray8 + (size_t)b * H0 * pitch + a0;
    const int it_row0 = lane / kBaseRowDw, it_col0 = 4 * (lane % kBaseRowDw);
    const int it_row1 = (64 + lane) / kBaseRowDw, it_col1 = 4 * ((64 + lane) % kBaseRowDw);

    // chunk j holds upsampled (virtual) rows u = ys - kLead + 8 j .. + 7; G0 chunk j - 2 completes there. An interior
    // chunk (u >= 2, u + 10 <= H; u is even) reads source rows u / 2 - 1 .. u / 2 + 4 with no reflection
    // or clamping: row u + 2t is h_t / 4 + 3 h_{t+1} / 4 and row u + 2t + 1 is 3 h_{t+1} / 4 + h_{t+2} / 4 (h_t: source
    // row lo + t interpolated across); other chunks take the per-row coordinates.
    const int n_chunks = (ye - ys + 7) / 8 + 2;
    auto interior = [&](int j) {
        const int u0 = ys - kLead + 8 * j;
        return u0 >= 2 && u0 + 10 <= H;
    };
    // per-row upsampling coordinates of a border chunk on lanes 0..7, and its first source row
    auto row_params = [&](int j, int& sy0, int& sy1, float& fy) {
        int a_0 = 0, a_1 = 0;
        float f = 0.f;
        up_coord(reflect101(ys - kLead + 8 * j + (lane & 7), H), H0, a_0, a_1, f);
        sy0 = a_0; sy1 = a_1; fy = f;
        int l = a_0;
#pragma unroll
        for (int m = 4; m > 0; m >>= 1) l = min(l, __shfl_xor(l, m));
        return __builtin_amdgcn_readfirstlane(l);
    };
    auto first_row = [&](int j) {
        if (interior(j)) return (ys - kLead + 8 * j) / 2 - 1;
        int s_0, s_1;
        float f;
        return row_params(j, s_0, s_1, f);
    };
    // Chunk j's source rows go to ring slot j mod 3 by global_load_lds_dword (two per chunk, always issued: past the
    // last chunk the last one is reloaded into the free slot), kBasePD chunks ahead, with the waits explicit as in
    // blur_stream_kernel. Every chunk from the third on also issues exactly 8 global stores (rows or lanes outside the
    // image go to `sink`), so the count of vector-memory operations issued after chunk j's loads is known:
    // 4 for j <= 2, 12 for j = 3 and 20 after.
    int plo[3];
    auto issue = [&](int j, auto kb) {
        constexpr int K = decltype(kb)::value;
        const int lo = first_row(j);
        plo[K] = lo;
        const uint32_t d = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(ring + K * kBaseRingRows * kBaseRowDw));
        const uint32_t o0 = (uint32_t)(min(lo + it_row0, H0 - 1) * pitch + it_col0);
        const uint32_t o1 = (uint32_t)(min(lo + it_row1, H0 - 1) * pitch + it_col1);
        asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(o0), "s"(src), "{m0}"(d) : "memory");
        if (64 + lane < kItems)
            asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(o1), "s"(src), "{m0}"(d + 256u) : "memory");
    };
    auto put_u = [&](int r, pf2 v) {
        ch1[r * IWP1 + lane] = v.x;
        if (has_b) ch1[r * IWP1 + 64 + lane] = v.y;
    };
    float win1[24];
    issue(0, std::integral_constant<int, 0>{});
    issue(min(1, n_chunks - 1), std::integral_constant<int, 1>{});
    const int x = s0 + lane;
    const bool out_lane = x < W;
    float* g0i = g0 + (size_t)b * H * W;
    auto chunk = [&](int j, auto jc) {
        constexpr int J = decltype(jc)::value;  // j mod 3
        const int lo = plo[J];
        issue(min(j + kBasePD, n_chunks - 1), std::integral_constant<int, (J + kBasePD) % 3>{});
        if (j >= 4)
            asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
        else if (j == 3)
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        const uint8_t* rg = (const uint8_t*)(ring + J * kBaseRingRows * kBaseRowDw);
        // upsampled rows of chunk j
        if (interior(j)) {
            pf2 h[6];
#pragma unroll
            for (int t = 0; t < 6; ++t) {
                const uint8_t* rr = rg + t * kBaseRowB;
                const pf2 p0 = {(float)rr[ca0], (float)rr[cb0]}, p1 = {(float)rr[ca1], (float)rr[cb1]};
                h[t] = __builtin_elementwise_fma(p0, fx1, p1 * fx);
            }
            const pf2 q1 = {0.25f, 0.25f}, q3 = {0.75f, 0.75f};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                put_u(2 * t, __builtin_elementwise_fma(h[t], q1, h[t + 1] * q3));
                put_u(2 * t + 1, __builtin_elementwise_fma(h[t + 1], q3, h[t + 2] * q1));
            }
        } else {
            int c_sy0, c_sy1;
            float c_fy;
            row_params(j, c_sy0, c_sy1, c_fy);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int sy0 = __shfl(c_sy0, r), sy1 = __shfl(c_sy1, r);
                const float fy = __shfl(c_fy, r);
                const uint8_t* r0 = rg + (sy0 - lo) * kBaseRowB;
                const uint8_t* r1 = rg + (sy1 - lo) * kBaseRowB;
                const pf2 a = __builtin_elementwise_fma(pf2{(float)r0[ca0], (float)r0[cb0]}, fx1,
                                                        pf2{(float)r0[ca1], (float)r0[cb1]} * fx);
                const pf2 c = __builtin_elementwise_fma(pf2{(float)r1[ca0], (float)r1[cb0]}, fx1,
                                                        pf2{(float)r1[ca1], (float)r1[cb1]} * fx);
                put_u(r, __builtin_elementwise_fma(a, pf2{1.f - fy, 1.f - fy}, c * pf2{fy, fy}));
            }
        }
        asm volatile("" ::: "memory");
        row_blur_chunk<R1, IWP1>(ch1, k1, lane);
#pragma unroll
        for (int r = 0; r < 8; ++r) win1[8 * J + r] = ch1[r * IWP1 + lane];
        if (j < 2) return;
        float gv[8];
        col_blur_window<R1, J>(win1, k1, gv);
        const int y0 = ys - kLead - 8 + 8 * j;  // G0 chunk j - 2
#pragma unroll
        for (int o = 0; o < 8; ++o) {
            const int y = y0 + o;
            // (y >= ys: the lead is one chunk)
            float* dp = (out_lane && y < ye) ? g0i + (size_t)y * W + x : sink + lane;
            *dp = gv[o];
        }
    };
    for (int j = 0; j < n_chunks; j += 3)
        static_for<3>([&](auto jc) {
            if (j + decltype(jc)::value < n_chunks) chunk(j + decltype(jc)::value, jc);
        });
    // the prefetched rows land before the wave retires
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool kFromU8>
struct BlurTable {
    using Fn = void (*)(const float*, const uint8_t*, int, int, int, float*, float*, int, int, int, int, int, Taps);
    static Fn get(int r) {
        switch (r) {
#define GTSFM_BLUR_CASE(RR) \
    case RR:                \
        return blur2d_kernel<RR, kFromU8>;
            GTSFM_BLUR_CASE(1) GTSFM_BLUR_CASE(2) GTSFM_BLUR_CASE(3) GTSFM_BLUR_CASE(4) GTSFM_BLUR_CASE(5)
            GTSFM_BLUR_CASE(6) GTSFM_BLUR_CASE(7) GTSFM_BLUR_CASE(8) GTSFM_BLUR_CASE(9) GTSFM_BLUR_CASE(10)
            GTSFM_BLUR_CASE(11) GTSFM_BLUR_CASE(12) GTSFM_BLUR_CASE(13) GTSFM_BLUR_CASE(14) GTSFM_BLUR_CASE(15)
            GTSFM_BLUR_CASE(16)
#undef GTSFM_BLUR_CASE
            default:
                return nullptr;
        }
    }
};


// ------------------------------------------------------------------ kernels: detection
struct GaussSet {
    const float* g[kLevels];
};

#define DAT(l, r, c) (G.g[(l) + 1][base + (size_t)(r) * W + (c)] - G.g[(l)][base + (size_t)(r) * W + (c)])

// Sub-pixel refinement (cv::SIFT adjustLocalExtrema) of one candidate: true and `res` for a kept keypoint. Duplicates
// (same refined location) are identical keypoints: the first claimant of the location's `seen` bit keeps it.
__device__ __forceinline__ bool refine_one(const Cand cd, const GaussSet& G, int H, int W, uint32_t* __restrict__ seen,
                                           Refined& res) {
    const float img_scale = 1.f / 255.f;
    const float deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale, cross_deriv_scale = img_scale * 0.25f;
    const size_t base = (size_t)cd.img * H * W;
    int layer = cd.layer, r = cd.r, c = cd.c;
    float xi = 0, xr = 0, xc = 0;
    int i = 0;
    bool ok = true;
    // the last iteration's derivatives: the loop only leaves with ok on a converged step, which does not move
    // (layer, r, c), so the final contrast and edge tests reuse them instead of gathering the same values again
    float l_dD0 = 0, l_dD1 = 0, l_dD2 = 0, l_ctr = 0, l_dxx = 0, l_dyy = 0, l_dxy = 0;
    for (; i < kMaxInterp; i++) {
        const int img = layer, prev = layer - 1, next = layer + 1;
        const float dD0 = (DAT(img, r, c + 1) - DAT(img, r, c - 1)) * deriv_scale;
        const float dD1 = (DAT(img, r + 1, c) - DAT(img, r - 1, c)) * deriv_scale;
        const float dD2 = (DAT(next, r, c) - DAT(prev, r, c)) * deriv_scale;
        const float ctr = DAT(img, r, c);
        const float v2 = ctr * 2;
        const float dxx = (DAT(img, r, c + 1) + DAT(img, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (DAT(img, r + 1, c) + DAT(img, r - 1, c) - v2) * second_deriv_scale;
        const float dss = (DAT(next, r, c) + DAT(prev, r, c) - v2) * second_deriv_scale;
        const float dxy = (DAT(img, r + 1, c + 1) - DAT(img, r + 1, c - 1) - DAT(img, r - 1, c + 1) +
                           DAT(img, r - 1, c - 1)) * cross_deriv_scale;
        const float dxs = (DAT(next, r, c + 1) - DAT(next, r, c - 1) - DAT(prev, r, c + 1) +
                           DAT(prev, r, c - 1)) * cross_deriv_scale;
        const float dys = (DAT(next, r + 1, c) - DAT(next, r - 1, c) - DAT(prev, r + 1, c) +
                           DAT(prev, r - 1, c)) * cross_deriv_scale;
        l_dD0 = dD0; l_dD1 = dD1; l_dD2 = dD2; l_ctr = ctr; l_dxx = dxx; l_dyy = dyy; l_dxy = dxy;
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys,
                    a22 = dss;
        float det = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
        float X0 = 0, X1 = 0, X2 = 0;
        if (det != 0) {
            det = 1 / det;
            X0 = det * (dD0 * (a11 * a22 - a12 * a21) - a01 * (dD1 * a22 - a12 * dD2) + a02 * (dD1 * a21 - a11 * dD2));
            X1 = det * (a00 * (dD1 * a22 - a12 * dD2) - dD0 * (a10 * a22 - a12 * a20) + a02 * (a10 * dD2 - dD1 * a20));
            X2 = det * (a00 * (a11 * dD2 - dD1 * a21) - a01 * (a10 * dD2 - dD1 * a20) + dD0 * (a10 * a21 - a11 * a20));
        }
        xi = -X2;
        xr = -X1;
        xc = -X0;
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT32_MAX / 3) || fabsf(xr) > (float)(INT32_MAX / 3) ||
            fabsf(xc) > (float)(INT32_MAX / 3)) {
            ok = false;
            break;
        }
        c += (int)rintf(xc);
        r += (int)rintf(xr);
        layer += (int)rintf(xi);
        if (layer < 1 || layer > kLayers || c < kBorder || c >= W - kBorder || r < kBorder || r >= H - kBorder) {
            ok = false;
            break;
        }
    }
    if (!ok || i >= kMaxInterp) return false;
    const float tt = l_dD0 * xc + l_dD1 * xr + l_dD2 * xi;
    const float contr = l_ctr * img_scale + tt * 0.5f;
    if (fabsf(contr) * kLayers < kContrast) return false;
    const float dxx = l_dxx, dyy = l_dyy, dxy = l_dxy;
    const float tr = dxx + dyy;
    const float det = dxx * dyy - dxy * dxy;
    if (det <= 0 || tr * tr * kEdge >= (kEdge + 1) * (kEdge + 1) * det) return false;
    // duplicates (same refined location) are identical keypoints: keep the first claimant
    const size_t bit = (((size_t)cd.img * kLayers + (layer - 1)) * H + r) * W + c;
    const uint32_t m = 1u << (bit & 31);
    if (atomicOr(&seen[bit >> 5], m) & m) return false;
    res = Refined{cd.img, layer, r, c, xc, xr, xi, contr};
    return true;
}

// Wave-aggregated append of the kept refinements (ballot + prefix popcount, one atomic per wave); every lane of the
// wave calls it.
__device__ __forceinline__ void append_refined(bool keep, const Refined& res, Refined* __restrict__ out,
                                               int* __restrict__ n_out, int out_cap) {
    const int lane = threadIdx.x & 63;
    const unsigned long long bal = __ballot(keep);
    if (bal) {
        int wbase = 0;
        if (lane == 0) wbase = atomicAdd(n_out, (int)__popcll(bal));
        wbase = __shfl(wbase, 0);
        const int slot = wbase + (int)__popcll(bal & ((1ull << lane) - 1ull));
        if (keep && slot < out_cap) out[slot] = res;
    }
}

// DoG levels are never stored: DoG_l = G_{l+1} - G_l is recomputed from the Gaussian levels (the same fp32
// subtraction cv::subtract performs), which removes 5 level writes per octave.
// Extrema scan: each wave sweeps a strip of kExStrip rows down 64 consecutive columns (lanes 1..62 produce outputs,
// lanes 0 and 63 are the left/right halo), one image row per step. Per row a lane loads Gaussian levels 1..4 at its
// pixel (coalesced 256-B rows, saddr + 32-bit offset), forms DoG 1..3, gets its horizontal neighbours by wave-wide DPP
// shifts, and keeps per DoG level the 3-wide row max/min of the last three rows in registers (rolling slots, the loop
// unrolled by three so no register moves). The 27-neighbourhood test "val >= every neighbour" is val == max over the
// 3x3x3 block (the centre included), from those max3/min3 partials. The outer DoG levels 0 and 4 only matter for a
// layer-1 / layer-3 pixel that already passed the threshold and beats its two in-register levels (a few per
// thousand): they are queued in LDS and their 3x3 blocks gathered after the sweep, all lanes at once. Each pixel's
// levels 1..4 are read once (plus 2 halo rows per strip and 2 halo lanes per wave): 16 B per pixel instead of all six
// levels' 24. Measured in round 5 and not kept: windows of 64 outputs aligned to 128-B lines, the halo columns
// loaded separately (lanes 0 / 63 take them through the DPP's old operand): bit-exact, but 366 vs 367 us per launch
// with the same FETCH_SIZE (the straddled lines are L2 hits) and 103 instead of 79 VGPRs (profiles/r05d_*).
#ifndef GTSFM_EX_STRIP
#define GTSFM_EX_STRIP 72
#endif
#ifndef GTSFM_EX_AHEAD
#define GTSFM_EX_AHEAD 6
#endif
constexpr int kExWaves = 4, kExOut = 62, kExStrip = GTSFM_EX_STRIP;
// rows of loads in flight per wave (a multiple of 3 dividing kExStrip): 6 / 9 / 12 measured 4.98 / 5.08 / 5.10 ms for
// octave 0 beside the next octave's blurs (profiles/r05at_*): the sweep is not waiting on its prefetch depth
constexpr int kExAhead = GTSFM_EX_AHEAD;
static_assert(kExAhead % 3 == 0 && kExStrip % kExAhead == 0, "row slots rotate by 3 within a strip");
// Candidate list sharded over kCandShards counters/segments (one global atomic per block on one of 256 counters).
constexpr int kCandShards = 256;
constexpr int kExList = 1024;  // per-block LDS list; overflow goes straight to the global list
constexpr int kExPend = 512;   // per-block queue of layer-1 / layer-3 pixels awaiting the outer-level test
struct ExPend {
    int y, c, layer;
    float val;
};

__device__ __forceinline__ float dpp_from_left(float v) {  // lane l gets lane l-1's value (lane 0: its own)
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane l gets lane l+1's value (lane 63: its own)
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x130, 0xf, 0xf, false));
}

__global__ __launch_bounds__(64 * kExWaves) void extrema_kernel(GaussSet G, int H, int W, Cand* __restrict__ cands,
                                                                int* __restrict__ n_cand, int cap,
                                                                uint32_t* __restrict__ seen, Refined* __restrict__ out,
                                                                int* __restrict__ n_out, int out_cap) {
    __shared__ Cand list[kExList];
    __shared__ ExPend pend[kExPend];
    __shared__ int n_list, n_pend, gbase;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, b = blockIdx.z;
    const int c = (blockIdx.x * kExWaves + wave) * kExOut + lane - 1;  // this lane's column
    const int y0 = blockIdx.y * kExStrip;
    const int shard = (int)((blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z)) %
                            kCandShards);  // cap is per shard
    if (threadIdx.x == 0) {
        n_list = 0;
        n_pend = 0;
    }
    __syncthreads();
    const float* gl[kLevels];
#pragma unroll
    for (int l = 0; l < kLevels; ++l) gl[l] = G.g[l] + (size_t)b * H * W;
    const int cx = min(max(c, 0), W - 1);
    const bool col_ok = lane >= 1 && lane <= kExOut && c >= kBorder && c < W - kBorder;
    const float threshold = floorf(0.5f * kContrast / kLayers * 255.f);

    // in registers: DoG levels 1..kLayers (index l - 1), from Gaussian levels 1..kLayers + 1
    constexpr int kIn = kLayers, kInLv = kLayers + 1;
    float hmax[kIn][3], hmin[kIn][3], ctr[kLayers][3];
    // Row y (clamped) of Gaussian levels 1..4 -> g; then into slot s: DoG 1..3, their 3-wide row extrema, and the
    // centre values of layers 1..3.
    auto fetch = [&](int y, float (&g)[kInLv]) {
        const uint32_t off = (uint32_t)(min(max(y, 0), H - 1) * W + cx);
#pragma unroll
        for (int l = 0; l < kInLv; ++l) g[l] = gl[l + 1][off];
    };
    auto finish = [&](const float (&g)[kInLv], auto slot) {
        constexpr int s = decltype(slot)::value;
#pragma unroll
        for (int l = 0; l < kIn; ++l) {
            const float d = g[l + 1] - g[l];
            const float lf = dpp_from_left(d), rt = dpp_from_right(d);
            hmax[l][s] = fmaxf(fmaxf(lf, d), rt);
            hmin[l][s] = fminf(fminf(lf, d), rt);
            ctr[l][s] = d;
        }
    };
    // 3x3 max / min of DoG level lo (= G_{lo+1} - G_lo, the same fp32 subtraction) around (y, c), from HBM/L2
    auto outer_block = [&](int lo, int y, float& emax, float& emin) {
        emax = -__builtin_inff();
        emin = __builtin_inff();
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const uint32_t off = (uint32_t)((y + dy) * W + c + dx);
                const float d = gl[lo + 1][off] - gl[lo][off];
                emax = fmaxf(emax, d);
                emin = fminf(emin, d);
            }
    };
    // Test row y: the three slots hold DoG rows y-1, y, y+1, row y in `slot`.
    auto emit = [&](int layer, int y) {
        const int slot_i = atomicAdd(&n_list, 1);
        if (slot_i < kExList) {
            list[slot_i] = Cand{b, layer, y, c};
        } else {  // plateau-heavy block: spill straight to the global list
            const int gi = atomicAdd(&n_cand[shard], 1);
            if (gi < cap) cands[(size_t)shard * cap + gi] = Cand{b, layer, y, c};
        }
    };
    // Branch-free per layer: "val > thr and val >= the 3x3x3 max" is val >= max(block max, thr_up) with thr_up the
    // next float above thr (val > thr >= 0 also gives val > 0), and the same on the min side; the wave leaves the
    // row at one exec test unless some lane has a flag (a few per thousand pixels).
    const float thr_up = __uint_as_float(__float_as_uint(threshold) + 1u);  // threshold >= 0
    auto test_row = [&](int y, auto slot) {
        constexpr int s = decltype(slot)::value;
        if (y < kBorder || y >= H - kBorder) return;
        float bmax[kIn], bmin[kIn];
#pragma unroll
        for (int l = 0; l < kIn; ++l) {
            bmax[l] = fmaxf(fmaxf(hmax[l][0], hmax[l][1]), hmax[l][2]);
            bmin[l] = fminf(fminf(hmin[l][0], hmin[l][1]), hmin[l][2]);
        }
        bool fmax_[kLayers], fmin_[kLayers];
        bool any = false;
#pragma unroll
        for (int layer = 1; layer <= kLayers; ++layer) {
            // DoG levels layer - 1 .. layer + 1; in registers: indices layer - 2 .. layer within [0, kIn)
            float mx = fmaxf(bmax[layer - 1], thr_up), mn = fminf(bmin[layer - 1], -thr_up);
            if (layer >= 2) { mx = fmaxf(mx, bmax[layer - 2]); mn = fminf(mn, bmin[layer - 2]); }
            if (layer < kIn) { mx = fmaxf(mx, bmax[layer]); mn = fminf(mn, bmin[layer]); }
            const float val = ctr[layer - 1][s];
            fmax_[layer - 1] = val >= mx;
            fmin_[layer - 1] = val <= mn;
            any = any || fmax_[layer - 1] || fmin_[layer - 1];
        }
        if (!col_ok || !any) return;
#pragma unroll
        for (int layer = 1; layer <= kLayers; ++layer) {
            const float val = ctr[layer - 1][s];
            bool ismax = fmax_[layer - 1], ismin = fmin_[layer - 1];
            if (!ismax && !ismin) continue;
            if (layer == 1 || layer == kLayers) {  // the outer DoG level (0 or kLayers + 1): queued
                const int qi = atomicAdd(&n_pend, 1);
                if (qi < kExPend) {
                    pend[qi] = ExPend{y, c, layer, val};
                    continue;
                }
                float emax, emin;  // queue full: test in place
                outer_block(layer == 1 ? 0 : kLayers + 1, y, emax, emin);
                ismax = ismax && val >= emax;
                ismin = ismin && val <= emin;
                if (!ismax && !ismin) continue;
            }
            emit(layer, y);
        }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    // rows y0-1 (slot 0) and y0 (slot 1) first; then row y0+1+3k+j goes to slot (2+j)%3 and completes the window of
    // row y0+3k+j, whose centre sits in slot (1+j)%3.
    // kExAhead rows' loads stay in flight: a row's buffer is refilled with the row kExAhead below as soon as it has
    // been consumed (rows past the strip's last needed row y_end re-read row y_end, an L2 hit).
    const int y_end = min(y0 + kExStrip, H);
    {
        float ga[kInLv], gb[kInLv];
        fetch(y0 - 1, ga);
        fetch(y0, gb);
        finish(ga, S0{});
        finish(gb, S1{});
    }
    float gq[kExAhead][kInLv];
    static_for<kExAhead>([&](auto jc) {
        fetch(y0 + 1 + decltype(jc)::value, gq[decltype(jc)::value]);
        __builtin_amdgcn_sched_barrier(0);  // in row order, so the loop's waits count the younger rows exactly
    });
    for (int y = y0; y < y_end; y += kExAhead)
        static_for<kExAhead>([&](auto jc) {
            constexpr int jj = decltype(jc)::value;
            finish(gq[jj], std::integral_constant<int, (2 + jj) % 3>{});
            fetch(min(y + kExAhead + 1 + jj, y_end), gq[jj]);
            test_row(y + jj, std::integral_constant<int, (1 + jj) % 3>{});
        });
    __syncthreads();
    // the queued layer-1 / layer-3 pixels: outer DoG level's 3x3 block, every lane gathering at once
    for (int i = threadIdx.x; i < min(n_pend, kExPend); i += 64 * kExWaves) {
        const ExPend e = pend[i];
        const int lo = e.layer == 1 ? 0 : kLayers + 1;
        float emax = -__builtin_inff(), emin = __builtin_inff();
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const uint32_t off = (uint32_t)((e.y + dy) * W + e.c + dx);
                const float d = gl[lo + 1][off] - gl[lo][off];
                emax = fmaxf(emax, d);
                emin = fminf(emin, d);
            }
        if ((e.val > 0 && e.val >= emax) || (e.val < 0 && e.val <= emin)) {
            const int slot_i = atomicAdd(&n_list, 1);
            if (slot_i < kExList) {
                list[slot_i] = Cand{b, e.layer, e.y, e.c};
            } else {
                const int gi = atomicAdd(&n_cand[shard], 1);
                if (gi < cap) cands[(size_t)shard * cap + gi] = Cand{b, e.layer, e.y, e.c};
            }
        }
    }
    __syncthreads();
    const int n = min(n_list, kExList);
    // refine the block's own candidates now, while the strip's Gaussian rows are still in L2 (a separate pass
    // re-fetched each candidate's 3x3x3 window from HBM)
    // (entries dealt round-robin to the waves: a short list keeps every wave busy on the dependent gathers)
#ifndef GTSFM_ABL_NO_REFINE  // timing ablation (tools/build_variants_src.sh): candidates found, not refined. C2
    // octave 0 (r06, profiles/r06s_*): 5.03 ms with the refinement, 4.15 without -- the sweep is the cost
    for (int base0 = 0; base0 < n; base0 += 64 * kExWaves) {
        const int i = base0 + lane * kExWaves + wave;
        Refined res;
        const bool keep = i < n && refine_one(list[i], G, H, W, seen, res);
        append_refined(keep, res, out, n_out, out_cap);
    }
#endif
}

// Candidates left in the kCandShards global segments (extrema blocks whose LDS list overflowed) are refined here.
__global__ __launch_bounds__(256) void refine_kernel(const Cand* __restrict__ cands,
                                                     const int* __restrict__ shard_counts, int cap, GaussSet G, int H,
                                                     int W, int n_img, uint32_t* __restrict__ seen,
                                                     Refined* __restrict__ out, int* __restrict__ n_out, int out_cap) {
    // gridDim.x is a multiple of kCandShards: each shard is worked by gridDim.x / kCandShards blocks
    const int sh = blockIdx.x % kCandShards, sub = blockIdx.x / kCandShards, nsub = gridDim.x / kCandShards;
    const int n_cand = min(shard_counts[sh], cap);
    for (int base0 = sub * blockDim.x; base0 < n_cand; base0 += nsub * blockDim.x) {
        const int id = base0 + threadIdx.x;
        Refined res;
        const bool keep = id < n_cand && refine_one(cands[(size_t)sh * cap + id], G, H, W, seen, res);
        append_refined(keep, res, out, n_out, out_cap);
    }
}

// Keypoint records are appended to kKpShards per-image shards (shard = workgroup mod kKpShards, each with its own
// counter on its own 128-B line and kKpCapPerImg / kKpShards slots): with one counter per image, every peak's
// atomicAdd of a small batch hit a few addresses (13 at one rank of 8 on C2) and serialised in L2 -- 395 -> 152 us for
// octave 0's orientation with the counter removed. kp_gather_kernel packs the shards into one run per image (record
// order is irrelevant: top-k sorts by a total order on the records' contents).
constexpr int kKpShards = 16, kKpCntStride = 32;  // counter of (img, shard) at (img * kKpShards + shard) * stride
// One wave per refined location: orientation histogram (fixed point, LDS u64 atomics), peaks -> keypoints.
__global__ __launch_bounds__(64) void orientation_kernel(const Refined* __restrict__ refs,
                                                         const int* __restrict__ n_ref_p, int ref_cap, GaussSet G,
                                                         int H, int W, int o, KeyRec* __restrict__ kps,
                                                         int* __restrict__ kp_shard_counts, int kp_cap) {
    __shared__ unsigned long long hist[kOriBins];
    const int lane = threadIdx.x;
    const int n_ref = min(*n_ref_p, ref_cap);
    for (int id = blockIdx.x; id < n_ref; id += gridDim.x) {
        if (lane < kOriBins) hist[lane] = 0ull;
        __syncthreads();
        // the refinement appends in extrema-block order (spatial clusters); a fixed bijective scramble spreads
        // concurrent waves over the image (2654435761 is prime, n_ref < 2^31)
        const Refined rf = refs[(int)(((unsigned long long)id * 2654435761ull) % (unsigned)n_ref)];
        const float size_oct = kSigma * exp2_det(((float)rf.layer + rf.xi) / kLayers);
        const float scl = size_oct;
        const int radius = (int)rintf(kOriRadius * scl);
        const float sigma = kOriSigFctr * scl;
        const float expf_scale = -1.f / (2.f * sigma * sigma);
        const float* img = G.g[rf.layer] + (size_t)rf.img * H * W;
        const int side = 2 * radius + 1;
        // Each lane takes a contiguous chunk of the patch, so the 64 concurrent LDS atomics of one instruction land on
        // bins of 64 different neighbourhoods instead of the same few bins (fixed-point sums: order-independent).
        const int total = side * side, chunk = (total + 63) / 64;
        const int kbeg = lane * chunk, kend = min(kbeg + chunk, total);
        int ci = kbeg / side, cj = kbeg % side;  // (row, column) of sample k, advanced incrementally
        for (int k = kbeg; k < kend; ++k) {
            const int i = ci - radius, j = cj - radius;
            if (++cj == side) {
                cj = 0;
                ++ci;
            }
            const int y = rf.r + i, x = rf.c + j;
            if (y <= 0 || y >= H - 1 || x <= 0 || x >= W - 1) continue;
            const float dx = img[(size_t)y * W + x + 1] - img[(size_t)y * W + x - 1];
            const float dy = img[(size_t)(y - 1) * W + x] - img[(size_t)(y + 1) * W + x];
            const float w = exp_det((float)(i * i + j * j) * expf_scale);
            const float ori = fast_atan2(dy, dx);
            const float mag = sqrtf(fmaf(dx, dx, dy * dy));
            int bin = (int)rintf((kOriBins / 360.f) * ori);
            if (bin >= kOriBins) bin -= kOriBins;
            if (bin < 0) bin += kOriBins;
            atomicAdd(&hist[bin], to_fix_nn(w * mag));
        }
        __syncthreads();
        // smoothing, maximum and peaks one bin per lane (the serial loops' arithmetic per bin; t[q] = hist[(q - 2) mod n]
        // is the circularly padded histogram)
        {
            constexpr int n = kOriBins;
            auto T = [&](int q) { return from_fix(hist[(q - 2 + n) % n]); };
            float hj = -__builtin_inff();
            if (lane < n)
                hj = (T(lane) + T(lane + 4)) * (1.f / 16.f) + (T(lane + 1) + T(lane + 3)) * (4.f / 16.f) +
                     T(lane + 2) * (6.f / 16.f);
            float maxval = hj;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) maxval = fmaxf(maxval, __shfl_xor(maxval, m));
            const float mag_thr = maxval * kOriPeakRatio;
            const int j = lane;
            const int l = j > 0 ? j - 1 : n - 1;
            const int r2 = j < n - 1 ? j + 1 : 0;
            const float hl = __shfl(hj, l), hr = __shfl(hj, r2);
            if (j < n && hj > hl && hj > hr && hj >= mag_thr) {
                float bin = j + 0.5f * (hl - hr) / (hl - 2 * hj + hr);
                bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
                float angle = 360.f - (360.f / n) * bin;
                if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
                const int shard = blockIdx.x & (kKpShards - 1), shard_cap = kp_cap / kKpShards;
                const int slot = atomicAdd(&kp_shard_counts[(rf.img * kKpShards + shard) * kKpCntStride], 1);
                if (slot < shard_cap) {
                    const float sc = (float)(1 << o) * 0.5f;
                    KeyRec kr;
                    kr.x = ((float)rf.c + rf.xc) * sc;
                    kr.y = ((float)rf.r + rf.xr) * sc;
                    kr.size = size_oct * (float)(1 << o) * 2.f * 0.5f;
                    kr.angle = angle;
                    kr.response = fabsf(rf.contr);
                    kr.xc = rf.xc;
                    kr.xr = rf.xr;
                    kr.scl = scl;
                    kr.o = o;
                    kr.layer = rf.layer;
                    kr.r = rf.r;
                    kr.c = rf.c;
                    kps[(size_t)rf.img * kp_cap + shard * shard_cap + slot] = kr;
                }
            }
        }
        __syncthreads();
    }
}

// One workgroup per image: the shards' records packed into one run at the image's region of `out` (shard order, then
// slot order), kp_counts[img] = the records kept (a shard keeps at most kp_cap / kKpShards).
__global__ __launch_bounds__(256) void kp_gather_kernel(const KeyRec* __restrict__ sharded,
                                                        const int* __restrict__ kp_shard_counts, int kp_cap,
                                                        KeyRec* __restrict__ out, int* __restrict__ kp_counts) {
    const int img = blockIdx.x, shard_cap = kp_cap / kKpShards;
    __shared__ int off[kKpShards + 1];
    if (threadIdx.x == 0) {
        int o = 0;
        for (int s = 0; s < kKpShards; ++s) {
            off[s] = o;
            o += min(kp_shard_counts[(img * kKpShards + s) * kKpCntStride], shard_cap);
        }
        off[kKpShards] = o;
        kp_counts[img] = o;
    }
    __syncthreads();
    const KeyRec* src = sharded + (size_t)img * kp_cap;
    KeyRec* dst = out + (size_t)img * kp_cap;
    for (int s = 0; s < kKpShards; ++s) {
        const int n = off[s + 1] - off[s];
        for (int i = threadIdx.x; i < n; i += blockDim.x) dst[off[s] + i] = src[s * shard_cap + i];
    }
}

// ------------------------------------------------------------------ image mask (cv::KeyPointsFilter::runByPixelsMask)
// One 1024-thread block per image: keeps the records whose pixel mask[(int)(y + 0.5f)][(int)(x + 0.5f)] is non-zero,
// compacting them in place in their original order (read a chunk, barrier, write), and updates the image's count.
// x, y are already in input-image pixels, as OpenCV applies the mask after scaling keypoints back from the
// upsampled octave (sift.dispatch.cpp detectAndCompute).
constexpr int kMaskThreads = 1024;

__global__ __launch_bounds__(kMaskThreads) void mask_filter_kernel(KeyRec* __restrict__ kps, int* __restrict__ kp_counts,
                                                                   int kp_cap, const uint8_t* __restrict__ masks, int H0,
                                                                   int W0) {
    __shared__ int wave_tot[kMaskThreads / 64];
    __shared__ int base_sh;
    const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = min(kp_counts[img], kp_cap);
    KeyRec* K = kps + (size_t)img * kp_cap;
    const uint8_t* mk = masks + (size_t)img * H0 * W0;
    if (tid == 0) base_sh = 0;
    __syncthreads();
    for (int c0 = 0; c0 < N; c0 += kMaskThreads) {
        const int i = c0 + tid;
        KeyRec r;
        bool keep = false;
        if (i < N) {
            r = K[i];
            const int yy = (int)(r.y + 0.5f), xx = (int)(r.x + 0.5f);
            keep = yy >= 0 && yy < H0 && xx >= 0 && xx < W0 && mk[(size_t)yy * W0 + xx] != 0;
        }
        const unsigned long long bal = __ballot(keep);
        const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
        if (lane == 0) wave_tot[wave] = __popcll(bal);
        __syncthreads();
        int before = base_sh;
        for (int w = 0; w < wave; ++w) before += wave_tot[w];
        __syncthreads();  // every record of the chunk is in registers before any slot is overwritten
        if (keep) K[before + rank] = r;
        if (tid == kMaskThreads - 1) {
            int tot = base_sh;
            for (int w = 0; w < kMaskThreads / 64; ++w) tot += wave_tot[w];
            base_sh = tot;
        }
        __syncthreads();
    }
    if (tid == 0) kp_counts[img] = base_sh;
}

// ------------------------------------------------------------------ top-k per image
constexpr int kTopkThreads = 1024;
constexpr int kTopkTieCap = 512;  // tie slots after the np2 sort slots

struct SortRec {
    unsigned long long key;  // (~response bits) << 32 | location code
    uint32_t angle;          // angle bits (non-negative float)
    int idx;
};

__device__ __forceinline__ bool rec_less(const SortRec& a, const SortRec& b) {
    if (a.key != b.key) return a.key < b.key;
    if (a.angle != b.angle) return a.angle < b.angle;
    return a.idx < b.idx;
}

__device__ __forceinline__ SortRec make_rec(const KeyRec& k, int idx) {
    const uint32_t hi = ~__float_as_uint(k.response);
    const uint32_t lo = ((uint32_t)k.o << 28) | ((uint32_t)k.layer << 26) | ((uint32_t)k.r << 13) | (uint32_t)k.c;
    return SortRec{((unsigned long long)hi << 32) | lo, __float_as_uint(k.angle), idx};
}

__device__ void bitonic_sort(SortRec* a, int n_pow2) {
    for (int size = 2; size <= n_pow2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int k = threadIdx.x; k < n_pow2; k += blockDim.x) {
                const int o = k ^ stride;
                if (o > k) {
                    const SortRec x = a[k], y = a[o];
                    const bool up = ((k & size) == 0);
                    if (rec_less(y, x) == up) {
                        a[k] = y;
                        a[o] = x;
                    }
                }
            }
            __syncthreads();
        }
}

// Selects the max_kpts keypoints of largest response (ties: octave, layer, row, col, angle) and orders them.
__global__ __launch_bounds__(kTopkThreads) void topk_kernel(const KeyRec* __restrict__ kps,
                                                            const int* __restrict__ kp_counts, int kp_cap,
                                                            int max_kpts, int* __restrict__ sel, int* __restrict__ n_sel) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int* hdr = (int*)smem;                         // [0] n_less, [1] n_eq, [2] scratch
    int* histo = (int*)(smem + 16);                // [256]
    SortRec* recs = (SortRec*)(smem + 16 + 1024);  // [pow2(max_kpts) + kTopkTieCap]
    const int img = blockIdx.x, tid = threadIdx.x;
    const int N = min(kp_counts[img], kp_cap);
    const KeyRec* K = kps + (size_t)img * kp_cap;
    const int k = min(N, max_kpts);
    int np2 = 1;
    while (np2 < k) np2 <<= 1;
    uint32_t T = 0xFFFFFFFFu;  // threshold on the hi word: take all hi < T, then the smallest ties hi == T
    if (N > max_kpts) {
        uint32_t prefix = 0;
        int need = k;
        for (int pass = 0; pass < 4; ++pass) {
            const int shift = 24 - 8 * pass;
            const uint32_t pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
            for (int i = tid; i < 256; i += kTopkThreads) histo[i] = 0;
            __syncthreads();
            for (int i = tid; i < N; i += kTopkThreads) {
                const uint32_t hi = ~__float_as_uint(K[i].response);
                if ((hi & pmask) == (prefix & pmask)) atomicAdd(&histo[(hi >> shift) & 255], 1);
            }
            __syncthreads();
            if (tid == 0) {
                int acc = 0, d = 0;
                for (; d < 256; ++d) {
                    if (acc + histo[d] >= need) break;
                    acc += histo[d];
                }
                hdr[2] = d;
                hdr[3] = need - acc;
            }
            __syncthreads();
            prefix |= (uint32_t)hdr[2] << shift;
            need = hdr[3];
            __syncthreads();
        }
        T = prefix;
    }
    // gather: all with hi < T (count k - need_eq), then ties hi == T sorted, truncated
    if (tid == 0) { hdr[0] = 0; hdr[1] = 0; }
    __syncthreads();
    for (int i = tid; i < N; i += kTopkThreads) {
        const uint32_t hi = ~__float_as_uint(K[i].response);
        if (N <= max_kpts || hi < T) recs[atomicAdd(&hdr[0], 1)] = make_rec(K[i], i);
    }
    __syncthreads();
    const int n_less = hdr[0];
    if (N > max_kpts) {
        // ties at the threshold: the (k - n_less) smallest in (location, angle, index) order. They are collected after
        // the strict set into the np2 + kTopkTieCap slots (ties are usually a handful: the orientations of one
        // location share its response) and selection-sorted; should they overflow the slots, they are instead picked
        // one at a time by block-wide minimum, each strictly after the previous pick in the total order.
        const int take = k - n_less;
        for (int i = tid; i < N; i += kTopkThreads) {
            const uint32_t hi = ~__float_as_uint(K[i].response);
            if (hi == T) {
                const int s = atomicAdd(&hdr[1], 1);
                if (n_less + s < np2 + kTopkTieCap) recs[n_less + s] = make_rec(K[i], i);
            }
        }
        __syncthreads();
        const int n_eq = hdr[1];
        if (n_less + n_eq <= np2 + kTopkTieCap) {
            if (tid == 0) {
                for (int a = 0; a < take; ++a) {
                    int m = a;
                    for (int b = a + 1; b < n_eq; ++b)
                        if (rec_less(recs[n_less + b], recs[n_less + m])) m = b;
                    const SortRec t = recs[n_less + a];
                    recs[n_less + a] = recs[n_less + m];
                    recs[n_less + m] = t;
                }
            }
        } else {
            SortRec* red = recs + np2;  // [kTopkThreads / 64] per-wave minima (the tie slots are not needed here)
            SortRec prev{0, 0, -1};
            for (int a = 0; a < take; ++a) {
                SortRec best{~0ull, ~0u, 0x7FFFFFFF};
                for (int i = tid; i < N; i += kTopkThreads) {
                    if (~__float_as_uint(K[i].response) != T) continue;
                    const SortRec r = make_rec(K[i], i);
                    if ((a == 0 || rec_less(prev, r)) && rec_less(r, best)) best = r;
                }
                for (int m = 32; m > 0; m >>= 1) {
                    SortRec o;
                    o.key = __shfl_xor(best.key, m);
                    o.angle = __shfl_xor(best.angle, m);
                    o.idx = __shfl_xor(best.idx, m);
                    if (rec_less(o, best)) best = o;
                }
                if ((tid & 63) == 0) red[tid >> 6] = best;
                __syncthreads();
                best = red[0];
                for (int w = 1; w < kTopkThreads / 64; ++w)
                    if (rec_less(red[w], best)) best = red[w];
                __syncthreads();
                if (tid == 0) recs[n_less + a] = best;
                prev = best;
            }
        }
        __syncthreads();
    }
    for (int i = k + tid; i < np2; i += kTopkThreads) recs[i] = SortRec{~0ull, ~0u, 0x7FFFFFFF};
    __syncthreads();
    bitonic_sort(recs, np2);
    for (int i = tid; i < k; i += kTopkThreads) sel[(size_t)img * max_kpts + i] = recs[i].idx;
    if (tid == 0) n_sel[img] = k;
}

// ------------------------------------------------------------------ descriptors: one wave per kept keypoint
#ifndef GTSFM_DESC_CHUNK
#define GTSFM_DESC_CHUNK 512
#endif
#ifndef GTSFM_DESC_COPIES
#define GTSFM_DESC_COPIES 2
#endif
constexpr int kDescChunk = GTSFM_DESC_CHUNK;
static_assert(kDescChunk >= 128 && kDescChunk % 64 == 0, "the descriptor's 128 values reuse the sample list");

__global__ __launch_bounds__(64) void descriptor_kernel(const KeyRec* __restrict__ kps, int kp_cap,
                                                        const int* __restrict__ sel, const int* __restrict__ n_sel,
                                                        int n_img, int max_kpts, LevelTable L, float narrow_below,
                                                        float* __restrict__ out_xy, float* __restrict__ out_attr,
                                                        float* __restrict__ out_desc) {
    constexpr int d = 4, n = 8, HB = (d + 2) * (d + 2) * (n + 2);
    // kCopies private histograms (lane & 1 picks one): adjacent samples usually land in the same bins, and same-address
    // LDS atomics of one instruction serialise. Integer (fixed-point) sums, so merging the copies is exact.
    constexpr int kCopies = GTSFM_DESC_COPIES, HBP = HB + 1;  // +1: copies start on different banks
    __shared__ unsigned long long hist[kCopies * HBP];
    __shared__ int slist[kDescChunk];  // valid samples of the current chunk, (i << 16) | (j & 0xffff)
    float* const dst = (float*)slist;  // the finished descriptor (the sample list is dead by then)
    __shared__ float dnorm;
    const int lane = threadIdx.x;
    for (int slot = blockIdx.x; slot < n_img * max_kpts; slot += gridDim.x) {
        const int img = slot / max_kpts, q = slot % max_kpts;
        if (q >= n_sel[img]) {  // uniform per block: a padding row, zeroed here (no memset of the outputs)
            const size_t row = (size_t)img * max_kpts + q;
            for (int k = lane; k < 128; k += 64) out_desc[row * 128 + k] = 0.f;
            if (lane < 2) out_xy[row * 2 + lane] = 0.f;
            if (lane < 3) out_attr[row * 3 + lane] = 0.f;
            continue;
        }
        const KeyRec kp = kps[(size_t)img * kp_cap + sel[(size_t)img * max_kpts + q]];
        for (int i = lane; i < kCopies * HBP; i += 64) hist[i] = 0ull;
        __syncthreads();
        const int H = L.H[kp.o], W = L.W[kp.o];
        const float* img_p = L.g[kp.o][kp.layer - 1] + (size_t)img * L.img_stride[kp.o];
        const float ptx = (float)kp.c + kp.xc, pty = (float)kp.r + kp.xr;
        float ori = 360.f - kp.angle;
        if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
        const float scl = kp.scl;
        const int px = (int)rintf(ptx), py = (int)rintf(pty);
        float sin_t, cos_t;
        sincos_det(ori * (float)(3.14159265358979323846 / 180), &sin_t, &cos_t);
        const float bins_per_rad = n / 360.f;
        const float exp_scale = -1.f / (d * d * 0.5f);
        const float hist_width = kDescrSclFctr * scl;
        int radius = (int)rintf(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
        const int diag = (int)sqrt(((double)W) * W + ((double)H) * H);
        if (radius > diag) radius = diag;
        cos_t /= hist_width;
        sin_t /= hist_width;
        const int side = 2 * radius + 1;
        unsigned long long* hc = hist + (lane & (kCopies - 1)) * HBP;
        const int di = 64 / side, dj = 64 % side;
        int ii = lane / side, jj = lane % side;  // (row, column) of sample k, advanced incrementally
        const int ss = side * side;
        // Half of the side x side square lies outside the rotated descriptor window: each chunk of kDescChunk samples
        // is first tested (consecutive lanes: consecutive pixels), the valid ones are compacted into slist by a wave
        // ballot, and only those run the gradient / weight / histogram work with every lane busy.
        for (int base = 0; base < ss; base += kDescChunk) {
            int nv = 0;
            for (int cc = 0; cc < kDescChunk; cc += 64) {
                const int i = ii - radius, j = jj - radius;
                ii += di;
                jj += dj;
                if (jj >= side) {
                    jj -= side;
                    ++ii;
                }
                const float c_rot = j * cos_t - i * sin_t;
                const float r_rot = j * sin_t + i * cos_t;
                const float rbin = r_rot + d / 2 - 0.5f;
                const float cbin = c_rot + d / 2 - 0.5f;
                const int r = py + i, c = px + j;
                const bool ok = base + cc + lane < ss && rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 &&
                                r < H - 1 && c > 0 && c < W - 1;
                const unsigned long long m = __ballot(ok);
                if (ok) slist[nv + __popcll(m & ((1ull << lane) - 1))] = (i << 16) | (j & 0xffff);
                nv += __popcll(m);
            }
            __syncthreads();
            // lane l takes the contiguous run [l nit, (l + 1) nit) of the chunk's samples: one instruction's 64 atomics
            // spread over the whole chunk's rows (and bins) instead of one or two raster rows
            // software-pipelined: the next sample's four gradient taps are in flight while this one is binned (lanes
            // past the chunk's end load the last valid sample's taps, in bounds, and skip the binning)
            const int nit = (nv + 63) >> 6;
            auto taps = [&](int t, float (&g)[4], int& sv) {
                sv = slist[min(t, nv - 1)];
                const int r = py + (sv >> 16), c = px + (short)(sv & 0xffff);
                const float* p = img_p + (size_t)r * W + c;
                g[0] = p[1];
                g[1] = p[-1];
                g[2] = p[-W];
                g[3] = p[W];
            };
            float gn[4];
            int svn = 0;
            if (nit > 0) taps(lane * nit, gn, svn);
            for (int it = 0; it < nit; ++it) {
            const int t = lane * nit + it;
            const float g0 = gn[0], g1 = gn[1], g2 = gn[2], g3 = gn[3];
            const int sv = svn;
            if (it + 1 < nit) taps(t + 1, gn, svn);
            if (t >= nv) continue;
            const int i = sv >> 16, j = (short)(sv & 0xffff);
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            float rbin = r_rot + d / 2 - 0.5f;
            float cbin = c_rot + d / 2 - 0.5f;
            const float dx = g0 - g1;
            const float dy = g2 - g3;
            const float wexp = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
            const float o = fast_atan2(dy, dx);
            const float mag0 = sqrtf(fmaf(dx, dx, dy * dy));
            const float w = exp_det(wexp);
            float obin = (o - ori) * bins_per_rad;
            const float mag = mag0 * w;
            // the trilinear weights in fixed-point units (x 2^24, exact): every product and difference below scales
            // with it in the normal range, and a value that left it unscaled is below 2^-102 here, i.e. 0 either way
            const float mags = mag * kFixScale;
            const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
            int o0 = (int)floorf(obin);
            rbin -= r0;
            cbin -= c0;
            obin -= o0;
            if (o0 < 0) o0 += n;
            if (o0 >= n) o0 -= n;
            const float v_r1 = mags * rbin, v_r0 = mags - v_r1;
            const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
            const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
            const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
            const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
            const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
            const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
            const int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
            // every contribution is at most mag (products of mag with fractions in [0, 1]), so while the wave's mags
            // stay below 255 every fixed-point value is below 2^32 and is the single truncating conversion
            // (uint32_t)(v 2^24) -- the same integer as to_fix_nn, at a third of its instructions
            auto put = [&](int at, float v, bool small) {
                atomicAdd(&hc[at], small ? (unsigned long long)(uint32_t)v : to_fix_scaled(v));
            };
            auto put8 = [&](bool small) {
                put(idx, v_rco000, small);
                put(idx + 1, v_rco001, small);
                put(idx + (n + 2), v_rco010, small);
                put(idx + (n + 3), v_rco011, small);
                put(idx + (d + 2) * (n + 2), v_rco100, small);
                put(idx + (d + 2) * (n + 2) + 1, v_rco101, small);
                put(idx + (d + 3) * (n + 2), v_rco110, small);
                put(idx + (d + 3) * (n + 2) + 1, v_rco111, small);
            };
            if (__all(mag < narrow_below))  // narrow_below <= 255 (0: the wide path for every sample, a test hook)
                put8(true);
            else
                put8(false);
            }
            __syncthreads();  // slist is rewritten by the next chunk
        }
        // finalisation: the element-wise steps run one element per lane, the two norms are sequential sums in the
        // oracle's order (lane 0), so every value is bit-identical
        for (int e = lane; e < d * d * n; e += 64) {
            const int cell = e / n, k = e % n;
            const int idx = ((cell / d + 1) * (d + 2) + (cell % d + 1)) * (n + 2);
            unsigned long long a = 0, w = 0;
#pragma unroll
            for (int c = 0; c < kCopies; ++c) {
                a += hist[c * HBP + idx + k];
                w += hist[c * HBP + idx + n + (k & 1)];
            }
            float v = from_fix(a);
            if (k < 2) v += from_fix(w);  // circular wrap of the orientation bins
            dst[e] = v;
        }
        __syncthreads();
        if (lane == 0) {
            float nrm2 = 0;
            for (int k = 0; k < 128; k++) nrm2 += dst[k] * dst[k];
            dnorm = sqrtf(nrm2) * kDescrMagThr;
        }
        __syncthreads();
        {
            const float thr = dnorm;
            for (int e = lane; e < 128; e += 64) dst[e] = fminf(dst[e], thr);
        }
        __syncthreads();
        if (lane == 0) {
            float nrm2 = 0;
            for (int i = 0; i < 128; i++) nrm2 += dst[i] * dst[i];
            dnorm = kIntDescrFctr / fmaxf(sqrtf(nrm2), FLT_EPSILON);
        }
        __syncthreads();
        {
            const float scale = dnorm;
            for (int e = lane; e < 128; e += 64) {
                const int v = (int)rintf(dst[e] * scale);
                dst[e] = (float)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
        __syncthreads();
        float* od = out_desc + ((size_t)img * max_kpts + q) * 128;
        for (int k = lane; k < 128; k += 64) od[k] = dst[k];
        if (lane == 0) {
            out_xy[((size_t)img * max_kpts + q) * 2] = kp.x;
            out_xy[((size_t)img * max_kpts + q) * 2 + 1] = kp.y;
            out_attr[((size_t)img * max_kpts + q) * 3] = kp.size;
            out_attr[((size_t)img * max_kpts + q) * 3 + 1] = kp.angle;
            out_attr[((size_t)img * max_kpts + q) * 3 + 2] = kp.response;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ host-side layout
int gauss_taps(double sigma, Taps* t) {
    int n = (int)lrint(sigma * 4 * 2 + 1) | 1;
    if (n > 2 * kMaxR + 1) return -1;
    float full[2 * kMaxR + 1];
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        full[i] = (float)exp(scale2X * x * x);
        sum += full[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) full[i] = (float)(full[i] * sum);
    t->r = n / 2;
    for (int j = 0; j <= t->r; ++j) t->k[j] = full[t->r + j];
    for (int j = t->r + 1; j <= kMaxR; ++j) t->k[j] = 0.f;
    return 0;
}

constexpr int kCandCapPerImg = 1 << 19;
constexpr int kKpCapPerImg = 1 << 16;

struct Layout {
    int B, H, W, n_oct, max_kpts;
    int Ho[kMaxOct], Wo[kMaxOct];
    size_t g[kMaxOct][kLevels];  // byte offsets
    size_t seen, seen_bytes, seen_off[kMaxOct], cand, ref, kps_sh, kp_shard_counts, kps, kp_counts, counters, sel,
        n_sel, gray, sink, total;
};

int num_octaves(int H, int W) {
    const int m = 2 * (H < W ? H : W);
    int n = (int)lrint(log((double)m) / log(2.) - 2) + 1;
    return n > kMaxOct ? kMaxOct : n;
}

Layout make_layout(int B, int H, int W, int max_kpts) {
    Layout L{};
    L.B = B;
    L.H = H;
    L.W = W;
    L.max_kpts = max_kpts;
    L.n_oct = num_octaves(H, W);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += gtsfm_align_up(bytes, 256);
        return o;
    };
    int h = 2 * H, w = 2 * W;
    for (int o = 0; o < L.n_oct; ++o) {
        L.Ho[o] = h;
        L.Wo[o] = w;
        const size_t lvl = (size_t)B * h * w * sizeof(float);
        // levels are read together (extrema: all six; blur: two); a per-level skew of 1.25 KiB keeps equal pixels of
        // different levels off the same HBM channel / bank
        for (int i = 0; i < kLevels; ++i) L.g[o][i] = take(lvl + (size_t)(5 * i + 3) * 256);
        h /= 2;
        w /= 2;
    }
    // every octave's seen-bitmap and candidate counters have their own region, cleared by one memset per extraction
    // (per-octave memsets were two fill launches of ~5 us per octave)
    L.seen_bytes = 0;
    for (int o = 0; o < L.n_oct; ++o) {
        L.seen_off[o] = L.seen_bytes;
        L.seen_bytes += gtsfm_align_up(((size_t)B * kLayers * L.Ho[o] * L.Wo[o] + 31) / 32 * 4, 256);
    }
    L.seen = take(L.seen_bytes);
    L.cand = take((size_t)B * kCandCapPerImg * sizeof(Cand));
    L.ref = take((size_t)B * kCandCapPerImg * sizeof(Refined));
    L.kps_sh = take((size_t)B * kKpCapPerImg * sizeof(KeyRec));
    L.kps = take((size_t)B * kKpCapPerImg * sizeof(KeyRec));
    L.kp_counts = take((size_t)B * sizeof(int));
    // the two counter blocks are adjacent: one memset clears both
    L.kp_shard_counts = take((size_t)B * kKpShards * kKpCntStride * sizeof(int));
    L.counters = take((size_t)kMaxOct * (kCandShards + 16) * sizeof(int));
    L.sel = take((size_t)B * max_kpts * sizeof(int));
    L.n_sel = take((size_t)B * sizeof(int));
    L.gray = take((size_t)B * H * base_pitch(W));  // the padded gray rows of the streaming base
    L.sink = take(64 * sizeof(float));             // its stores outside the image
    L.total = off;
    return L;
}

}  // namespace

extern "C" {

size_t gtsfm_sift_workspace_bytes(int n_img, int H, int W, int max_kpts) {
    if (n_img <= 0 || H < 16 || W < 16 || max_kpts <= 0) return 0;
    return make_layout(n_img, H, W, max_kpts).total;
}

int gtsfm_sift_batched(const uint8_t* d_images, const uint8_t* d_masks, int n_img, int H, int W, int channels,
                       int max_kpts, void* d_workspace,
                       size_t workspace_bytes, float* d_xy, float* d_attr, float* d_desc, int* d_counts,
                       int* d_n_detected, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_img == 0) return GTSFM_OK;
    if (!d_images || !d_workspace || !d_xy || !d_attr || !d_desc || !d_counts || n_img < 0 || H < 16 || W < 16 ||
        (channels != 1 && channels != 3) || max_kpts <= 0 || max_kpts > 8192 || 2 * H >= 8192 || 2 * W >= 8192)
        return GTSFM_ERR_ARG;
    const Layout L = make_layout(n_img, H, W, max_kpts);
    if (workspace_bytes < L.total) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    auto F = [&](size_t off) { return (float*)(ws + off); };
    int* counters_all = (int*)(ws + L.counters);
    int* kp_counts = (int*)(ws + L.kp_counts);
    const int B = n_img;

    Taps taps[kLevels];
    {
        double sig[kLevels];
        sig[0] = kSigma;
        const double k = pow(2., 1. / kLayers);
        for (int i = 1; i < kLevels; ++i) {
            const double sig_prev = pow(k, (double)(i - 1)) * kSigma;
            const double sig_total = sig_prev * k;
            sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
        }
        const double sig_diff = sqrt(fmax(kSigma * kSigma - kInitSigma * kInitSigma * 4, 0.01));
        if (gauss_taps((double)(float)sig_diff, &taps[0])) return GTSFM_ERR_ARG;
        for (int i = 1; i < kLevels; ++i)
            if (gauss_taps(sig[i], &taps[i])) return GTSFM_ERR_ARG;
    }
    GTSFM_CHECK_HIP(hipMemsetAsync(ws + L.kp_shard_counts, 0,
                                   L.counters + (size_t)kMaxOct * (kCandShards + 16) * sizeof(int) - L.kp_shard_counts,
                                   stream));
    GTSFM_CHECK_HIP(hipMemsetAsync(ws + L.seen, 0, L.seen_bytes, stream));
    GTSFM_CHECK_HIP(hipMemsetAsync(d_counts, 0, (size_t)B * sizeof(int), stream));
    // d_xy / d_attr / d_desc: every row is written by descriptor_kernel (padding rows as zeros)

    for (int i = 0; i < kLevels; ++i)
        if (taps[i].r < 1 || taps[i].r > kBlurMaxR) return GTSFM_ERR_ARG;

    int n_cu = 0;
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            return GTSFM_ERR_HIP;
    }
    auto blur = [&](const float* src, float* dst, float* dec, int h, int w, const Taps& t) -> int {
        const bool u8 = src == nullptr;
        const int ty = blur_ty(t.r, u8), tyt = blur_tyt(t.r, u8);
        const int n_tx = (w + kBlurTX - 1) / kBlurTX, n_ty = (h + ty - 1) / ty;
        const int total = n_tx * n_ty * B;
        const dim3 grid((unsigned)((total + 7) / 8 * 8));
        const void* fn = u8 ? (const void*)BlurTable<true>::get(t.r) : (const void*)BlurTable<false>::get(t.r);
        const size_t lds = blur_lds_bytes(t.r, u8);
        if (lds > 65536) {
            const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return GTSFM_ERR_HIP;
        }
        if (u8)
            hipLaunchKernelGGL(BlurTable<true>::get(t.r), grid, dim3(kBlurTX, tyt), lds, stream, nullptr,
                               d_images, channels, H, W, dst, dec, h, w, n_tx, n_ty, B, t);
        else if (t.r >= kBlurStreamMinR) {  // wide kernels: the streaming variant (narrow ones are HBM-bound as tiles)
            const BlurStreamFn sf = blur_stream_get(t.r);
            const int n_strips = (w + kBlurTX - 1) / kBlurTX;
            const size_t lds_s = blur_stream_lds_bytes(t.r);
            // runs of about h / n_seg rows per (image, strip), all launched at once: at least 3 per image column and
            // 64 waves per CU in all (measured on octave 0: 1 / 3 / 8 runs per column 1.73 / 1.70 / 1.77 ms at r = 13;
            // small octaves need the extra runs), each at least 32 rows long
            const int n_seg = max(1, min(max(3, (64 * n_cu + B * n_strips - 1) / (B * n_strips)), (h + 31) / 32));
            const int n_parts = B * n_seg;
            const int n_blk = ((n_strips * n_parts + kStreamWaves - 1) / kStreamWaves + 7) / 8 * 8;
            hipLaunchKernelGGL(sf, dim3(n_blk), dim3(64 * kStreamWaves), lds_s, stream, src, dst, dec, h, w, n_strips,
                               n_parts, B, t);
        } else
            hipLaunchKernelGGL(BlurTable<false>::get(t.r), grid, dim3(kBlurTX, tyt), lds, stream, src, nullptr, 0,
                               0, 0, dst, dec, h, w, n_tx, n_ty, B, t);
        return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
    };
    // Detection (extrema + refinement, orientation) of octave o reads only octave o's levels, so it runs on a side
    // stream while the main stream goes on with octave o + 1's blurs: the latency-bound refinement and orientation
    // overlap the bandwidth-bound blurs. Octaves stay in order on the side stream (they share the candidate and
    // refinement buffers); the main stream joins it before the keypoints are gathered.
    // The side stream and its events are per device and created once (under a lock). The call as a whole is not
    // safe to run from two host threads on one device at once (they would share the side stream's events); callers
    // serialise per device, as every caller in this package does.
    hipStream_t side = nullptr;
    hipEvent_t* ev = nullptr;
    {
        static std::mutex mu;
        static hipStream_t sides[kMaxDevices] = {};
        static hipEvent_t evs[kMaxDevices][kMaxOct + 1] = {};
        int dev = 0;
        GTSFM_CHECK_HIP(hipGetDevice(&dev));
        if (dev < 0 || dev >= kMaxDevices) return GTSFM_ERR_ARG;
        std::lock_guard<std::mutex> lock(mu);
        if (!sides[dev]) {
            hipStream_t st = nullptr;
            GTSFM_CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            for (int i = 0; i <= kMaxOct; ++i)
                GTSFM_CHECK_HIP(hipEventCreateWithFlags(&evs[dev][i], hipEventDisableTiming));
            sides[dev] = st;
        }
        side = sides[dev];
        // GTSFM_SIFT_SERIAL=1 (profiling hook): detection on the caller's stream, so every kernel runs alone
        const char* serial = getenv("GTSFM_SIFT_SERIAL");
        if (serial && serial[0] == '1') side = stream;
        ev = evs[dev];
    }
    // an error inside the octave loop still joins the side stream's work to the caller's stream
    auto join_side = [&]() {
        if (hipEventRecord(ev[kMaxOct], side) == hipSuccess) (void)hipStreamWaitEvent(stream, ev[kMaxOct], 0);
    };
    // octave 0's base as a streaming launch from the gray bytes when the call's taps are the compiled-in ones
    // (OpenCV's defaults). GTSFM_SIFT_BASE_STREAM (test hooks): 0 selects the upsampling tile kernel, 2 makes an
    // ineligible call fail with GTSFM_ERR_ARG instead of taking it (a test pins the two paths against each other).
    const char* base_env = getenv("GTSFM_SIFT_BASE_STREAM");
    const char base_mode = base_env && base_env[0] ? base_env[0] : '1';
    const bool base_stream = base_mode != '0' && taps[0].r == kBaseR &&
                             memcmp(taps[0].k, kBaseTaps, sizeof(kBaseTaps)) == 0;
    if (base_mode == '2' && !base_stream) return GTSFM_ERR_ARG;
    auto base_stream_launch = [&](int h, int w) -> int {
        const int n_strips = (w + 63) / 64;
        const int n_seg = max(1, min(max(3, (64 * n_cu + B * n_strips - 1) / (B * n_strips)), (h + 31) / 32));
        const int n_blk = ((n_strips * n_seg * B + kStreamWaves - 1) / kStreamWaves + 7) / 8 * 8;
        const int pitch = base_pitch(W);
        const long long n_dw = (long long)B * H * (pitch / 4);
        const dim3 ggrid((unsigned)std::min<long long>((n_dw + 255) / 256, 16 * 1024));
        const int aligned = ((uintptr_t)d_images & 3) == 0 && ((size_t)W * channels) % 4 == 0;
        if (channels == 3)
            hipLaunchKernelGGL(gray_pad_kernel<3>, ggrid, dim3(256), 0, stream, d_images, ws + L.gray, B * H, W, pitch,
                               aligned);
        else
            hipLaunchKernelGGL(gray_pad_kernel<1>, ggrid, dim3(256), 0, stream, d_images, ws + L.gray, B * H, W, pitch,
                               aligned);
        hipLaunchKernelGGL(base_stream_kernel, dim3(n_blk), dim3(64 * kStreamWaves), 0, stream, ws + L.gray, H, W,
                           pitch, F(L.g[0][0]), F(L.sink), h, w, n_strips, n_seg, B);
        return hipGetLastError() == hipSuccess ? GTSFM_OK : GTSFM_ERR_HIP;
    };
    for (int o = 0; o < L.n_oct; ++o) {
        const int h = L.Ho[o], w = L.Wo[o];
        // octave o > 0 starts from the layer-3 level of octave o - 1, decimated by that level's blur launch
        if (o == 0 && (base_stream ? base_stream_launch(h, w) : blur(nullptr, F(L.g[0][0]), nullptr, h, w, taps[0]))) {
            join_side();
            return GTSFM_ERR_HIP;
        }
        for (int i = 1; i < kLevels; ++i) {
            float* dec = (i == kLayers && o + 1 < L.n_oct) ? F(L.g[o + 1][0]) : nullptr;
            if (dec && (L.Ho[o + 1] != h / 2 || L.Wo[o + 1] != w / 2)) {
                join_side();
                return GTSFM_ERR_ARG;
            }
            if (blur(F(L.g[o][i - 1]), F(L.g[o][i]), dec, h, w, taps[i])) {
                join_side();
                return GTSFM_ERR_HIP;
            }
        }
        GTSFM_CHECK_HIP(hipGetLastError());
        if (h <= 2 * kBorder || w <= 2 * kBorder) continue;
        GTSFM_CHECK_HIP(hipEventRecord(ev[o], stream));
        GTSFM_CHECK_HIP(hipStreamWaitEvent(side, ev[o], 0));
        int* counters = counters_all + o * (kCandShards + 16);
        uint32_t* seen = (uint32_t*)(ws + L.seen + L.seen_off[o]);
        GaussSet G;
        for (int i = 0; i < kLevels; ++i) G.g[i] = F(L.g[o][i]);
        const int shard_cap = (int)((size_t)B * kCandCapPerImg / kCandShards);
        hipLaunchKernelGGL(extrema_kernel, dim3((w + kExWaves * kExOut - 1) / (kExWaves * kExOut),
                                                (h + kExStrip - 1) / kExStrip, B),
                           dim3(64 * kExWaves), 0, side, G, h, w, (Cand*)(ws + L.cand), counters, shard_cap,
                           seen, (Refined*)(ws + L.ref), counters + kCandShards,
                           B * kCandCapPerImg);
        // fused: only list overflows reach the shards, so one block per shard
        hipLaunchKernelGGL(refine_kernel, dim3(kCandShards), dim3(256), 0, side, (const Cand*)(ws + L.cand), counters,
                           shard_cap, G, h, w, B, seen, (Refined*)(ws + L.ref),
                           counters + kCandShards, B * kCandCapPerImg);
        hipLaunchKernelGGL(orientation_kernel, dim3(8192), dim3(64), 0, side, (const Refined*)(ws + L.ref),
                           counters + kCandShards, B * kCandCapPerImg, G, h, w, o, (KeyRec*)(ws + L.kps_sh),
                           (int*)(ws + L.kp_shard_counts), kKpCapPerImg);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    GTSFM_CHECK_HIP(hipEventRecord(ev[kMaxOct], side));
    GTSFM_CHECK_HIP(hipStreamWaitEvent(stream, ev[kMaxOct], 0));
    static_assert(kKpCapPerImg % kKpShards == 0, "shards split the per-image capacity evenly");
    hipLaunchKernelGGL(kp_gather_kernel, dim3(B), dim3(256), 0, stream, (const KeyRec*)(ws + L.kps_sh),
                       (const int*)(ws + L.kp_shard_counts), kKpCapPerImg, (KeyRec*)(ws + L.kps), kp_counts);
    GTSFM_CHECK_HIP(hipGetLastError());
    if (d_masks) {
        hipLaunchKernelGGL(mask_filter_kernel, dim3(B), dim3(kMaskThreads), 0, stream, (KeyRec*)(ws + L.kps),
                           kp_counts, kKpCapPerImg, d_masks, H, W);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    int np2 = 1;
    while (np2 < max_kpts) np2 <<= 1;
    const size_t topk_lds = 16 + 1024 + (size_t)(np2 + kTopkTieCap) * sizeof(SortRec);
    if (topk_lds > 160 * 1024) return GTSFM_ERR_ARG;
    if (topk_lds > 65536)
        GTSFM_CHECK_HIP(hipFuncSetAttribute((const void*)topk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)topk_lds));
    hipLaunchKernelGGL(topk_kernel, dim3(B), dim3(kTopkThreads), topk_lds, stream, (const KeyRec*)(ws + L.kps),
                       kp_counts, kKpCapPerImg, max_kpts, (int*)(ws + L.sel), d_counts);
    GTSFM_CHECK_HIP(hipGetLastError());
    LevelTable T{};
    for (int o = 0; o < L.n_oct; ++o) {
        for (int i = 0; i < kLayers; ++i) T.g[o][i] = F(L.g[o][i + 1]);
        T.H[o] = L.Ho[o];
        T.W[o] = L.Wo[o];
        T.img_stride[o] = (size_t)L.Ho[o] * L.Wo[o];
    }
    // Weighted gradient magnitudes of a u8 image stay far below 255 (the Gaussian levels bound every difference of
    // two pixels two apart by about 2 * 255 / (1.25 sqrt(2 pi)) ~ 163), so the wide fixed-point conversion never runs on
    // real inputs; GTSFM_SIFT_DESC_WIDE=1 forces it for every sample so that tests can pin it against the oracle.
    const char* wide = getenv("GTSFM_SIFT_DESC_WIDE");
    const float narrow_below = (wide && wide[0] == '1') ? 0.f : 255.f;
    // one workgroup per output row: the dispatcher balances the keypoints (a grid-stride loop over 16384 workgroups
    // ended on a partial last round: C2 2131 -> 1975 us, profiles/r06v_*)
    hipLaunchKernelGGL(descriptor_kernel, dim3(B * max_kpts), dim3(64), 0, stream,
                       (const KeyRec*)(ws + L.kps), kKpCapPerImg, (const int*)(ws + L.sel), d_counts, B, max_kpts, T,
                       narrow_below, d_xy, d_attr, d_desc);
    GTSFM_CHECK_HIP(hipGetLastError());
    if (d_n_detected) GTSFM_CHECK_HIP(hipMemcpyAsync(d_n_detected, kp_counts, (size_t)B * sizeof(int),
                                                     hipMemcpyDeviceToDevice, stream));
    return GTSFM_OK;
}

}  // extern "C"
