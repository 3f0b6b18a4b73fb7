// SuperPoint detector-descriptor on gfx950: the network of
// thirdparty/SuperGluePretrainedNetwork/models/superpoint.py:145-202 as driven by
// gtsfm/frontend/detector_descriptor/superpoint.py:48-74, batched over same-sized images.
//
//   gray/255 -> conv1a..conv4b (3x3, ReLU, 2x2 max-pool after 1b/2b/3b) -> [convPa | convDa] (one 3x3, 128 -> 512)
//   -> convPb (1x1 -> 65) -> softmax -> 8x8 depth-to-space -> simple_nms(r) -> threshold + border -> top-k
//   -> convDb (1x1 -> 256) -> per-keypoint bilinear sample of the L2-normalised map (grid_sample, align_corners
//   False) -> L2 normalise.
//
// Convolutions are implicit GEMMs on the bf16 matrix cores at fp32 accuracy (conv3.hpp: every operand split into
// three bf16 planes, six plane products per k-step), so the network matches the reference's fp32 torch up to
// summation order. Activations are NHWC fp32 in HBM; a workgroup stages an input patch and the 16-channel weight slab
// in LDS (2x2 max-pool fused into the epilogue, in-lane). Everything after the convolutions is elementwise / stencil
// work on the score map and is HBM-bound.
#include <float.h>

#include "common.hpp"

#pragma clang fp contract(off)

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ packed weight blob (include/gtsfm_hip.h)
struct SpLayer {
    int k, cin, cout_pad;
};
constexpr int kSpLayers = 11;
constexpr SpLayer kSp[kSpLayers] = {
    {3, 1, 64},    {3, 64, 64},   {3, 64, 64},   {3, 64, 64},   {3, 64, 128}, {3, 128, 128},
    {3, 128, 128}, {3, 128, 128}, {3, 128, 512}, {1, 256, 128}, {1, 256, 256},
};
enum { L1A, L1B, L2A, L2B, L3A, L3B, L4A, L4B, LHEAD, LPB, LDB };

__host__ __device__ constexpr size_t sp_layer_floats(int l) {
    return (size_t)kSp[l].k * kSp[l].k * kSp[l].cin * kSp[l].cout_pad + kSp[l].cout_pad;
}
__host__ __device__ constexpr size_t sp_layer_offset(int l) {
    size_t o = 0;
    for (int i = 0; i < l; ++i) o += sp_layer_floats(i);
    return o;
}

// ------------------------------------------------------------------ conv1a: 1 -> 64 channels, direct
// The input is the u8 image (gray, or RGB through cv::COLOR_RGB2GRAY's fixed point); x = (float)g / 255.0f as
// superpoint.py:58 computes it (float32 array / 255.0).
__device__ __forceinline__ float sp_gray(const uint8_t* __restrict__ img, int C, int W, int y, int x) {
    const uint8_t* p = img + ((size_t)y * W + x) * C;
    const int g = C == 1 ? p[0] : ((p[0] * 4899 + p[1] * 9617 + p[2] * 1868 + (1 << 13)) >> 14);
    return (float)g / 255.0f;
}

__global__ __launch_bounds__(256) void conv1a_kernel(const uint8_t* __restrict__ imgs, int n, int H, int W, int C,
                                                     const float* __restrict__ wb, float* __restrict__ out) {
    __shared__ float w[9 * 64 + 64];
    for (int i = threadIdx.x; i < 9 * 64 + 64; i += blockDim.x) w[i] = wb[i];
    __syncthreads();
    const size_t pix = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= (size_t)n * H * W) return;
    const int x = (int)(pix % W);
    const int y = (int)((pix / W) % H);
    const int img = (int)(pix / ((size_t)W * H));
    const uint8_t* im = imgs + (size_t)img * H * W * C;
    float v[9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int yy = y + ky - 1, xx = x + kx - 1;
            v[ky * 3 + kx] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? sp_gray(im, C, W, yy, xx) : 0.0f;
        }
    f32x4_t* o = (f32x4_t*)(out + pix * 64);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        f32x4_t r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int co = 4 * q + e;
            float acc = 0.0f;
#pragma unroll
            for (int t = 0; t < 9; ++t) acc = __builtin_fmaf(v[t], w[t * 64 + co], acc);
            acc = acc + w[9 * 64 + co];
            r[e] = acc > 0.0f ? acc : 0.0f;
        }
        o[q] = r;
    }
}

#include "conv3.hpp"

// fp32 weights [tap][Cin][cout_pad] of layers L1B..LDB -> bf16 planes [tap][Cin / 16][plane][cout_pad][16] at
// sp_w3_offset(layer); blockIdx.y = layer - 1
__host__ __device__ constexpr size_t sp_w3_offset(int l) {
    size_t o = 0;
    for (int i = 1; i < l; ++i) o += (size_t)3 * kSp[i].k * kSp[i].k * kSp[i].cin * kSp[i].cout_pad;
    return o;
}

__global__ void sp_split_weights_kernel(const float* __restrict__ blob, __bf16* __restrict__ w3) {
    const int l = blockIdx.y + 1;
    const int KK = kSp[l].k * kSp[l].k, Cin = kSp[l].cin, Cp = kSp[l].cout_pad;
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (size_t)KK * Cin * Cp) return;
    const int co = (int)(e % Cp), ci = (int)((e / Cp) % Cin), kk = (int)(e / ((size_t)Cp * Cin));
    __bf16 pl[3];
    sp_split3(blob[sp_layer_offset(l) + e], pl[0], pl[1], pl[2]);
    __bf16* out = w3 + sp_w3_offset(l);
#pragma unroll
    for (int p = 0; p < 3; ++p)
        out[((((size_t)kk * (Cin / kCinChunk) + ci / kCinChunk) * 3 + p) * Cp + co) * 16 + ci % kCinChunk] = pl[p];
}

// ------------------------------------------------------------------ dense scores: softmax over 65, depth-to-space
// superpoint.py:168-172: scores = softmax(convPb)[:, :64] reshaped so cell (cy, cx) channel c -> pixel
// (8 cy + c / 8, 8 cx + c % 8).
__global__ __launch_bounds__(64) void scores_kernel(const float* __restrict__ logits /*(n,H8,W8,128)*/, int n, int H8,
                                                    int W8, float* __restrict__ S /*(n, 8 H8, 8 W8)*/) {
    const size_t cell = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (cell >= (size_t)n * H8 * W8) return;
    const int cx = (int)(cell % W8);
    const int cy = (int)((cell / W8) % H8);
    const int img = (int)(cell / ((size_t)W8 * H8));
    const float* l = logits + cell * 128;
    float m = l[0];
    for (int c = 1; c < 65; ++c) m = fmaxf(m, l[c]);
    float e[65];
    float sum = 0.0f;
    for (int c = 0; c < 65; ++c) {
        e[c] = expf(l[c] - m);
        sum = sum + e[c];
    }
    const int Ws = 8 * W8;
    float* s = S + ((size_t)img * 8 * H8 + 8 * cy) * Ws + 8 * cx;
    for (int c = 0; c < 64; ++c) s[(c >> 3) * Ws + (c & 7)] = e[c] / sum;
}

// ------------------------------------------------------------------ simple_nms (superpoint.py:47-61)
// max_pool2d(kernel 2r+1, stride 1, padding r) is separable: row max then column max over the clipped window.
__global__ void rowmax_kernel(const float* __restrict__ in, float* __restrict__ out, int n, int H, int W, int r) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (size_t)n * H * W) return;
    const int x = (int)(p % W);
    const float* row = in + (p - x);
    float m = row[x];
    const int lo = max(0, x - r), hi = min(W - 1, x + r);
    for (int xx = lo; xx <= hi; ++xx) m = fmaxf(m, row[xx]);
    out[p] = m;
}

__global__ void colmax_kernel(const float* __restrict__ in, float* __restrict__ out, int n, int H, int W, int r) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (size_t)n * H * W) return;
    const int x = (int)(p % W);
    const int y = (int)((p / W) % H);
    const float* col = in + (p - (size_t)y * W);
    float m = col[(size_t)y * W];
    const int lo = max(0, y - r), hi = min(H - 1, y + r);
    for (int yy = lo; yy <= hi; ++yy) m = fmaxf(m, col[(size_t)yy * W]);
    out[p] = m;
}

// stage 0: mask = (S == maxpool(S)); stage 1: T = supp ? 0 : S with supp = maxpool(mask) > 0;
// stage 2: mask |= (T == maxpool(T)) & !supp; stage 3: N = mask ? S : 0
__global__ void nms_step_kernel(int stage, size_t total, const float* __restrict__ S, const float* __restrict__ P,
                                float* __restrict__ mask, const float* __restrict__ Q, float* __restrict__ T) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= total) return;
    if (stage == 0) {
        mask[p] = S[p] == P[p] ? 1.0f : 0.0f;
    } else if (stage == 1) {
        T[p] = Q[p] > 0.0f ? 0.0f : S[p];
    } else if (stage == 2) {
        const bool supp = Q[p] > 0.0f;
        const bool nm = T[p] == P[p];
        if (nm && !supp) mask[p] = 1.0f;
    } else {
        T[p] = mask[p] > 0.0f ? S[p] : 0.0f;
    }
}

// ------------------------------------------------------------------ keypoint extraction in raster order
// superpoint.py:175-184: nonzero(s > threshold) (row-major), then remove_borders (y in [b, H - b), x in [b, W - b)).
constexpr int kRowThreads = 256;

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
    // 256 threads: wave-level inclusive scan, then across the 4 waves
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += sh[w];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return off + x - v;
}

// Image masks (gtsfm/frontend/detector_descriptor/superpoint.py:68-70, Keypoints.filter_by_mask): a detection at
// integer pixel (x, y) survives iff mask[y][x] == 1 (the reference compares with == 1, so other nonzero values drop
// it); masks[n][mH][mW] u8 over the full image (the detection grid, 8 * floor(H / 8) x 8 * floor(W / 8), lies inside).
__device__ __forceinline__ bool mask_ok(const uint8_t* __restrict__ masks, int img, int mH, int mW, int y, int x) {
    return masks == nullptr || masks[((size_t)img * mH + y) * mW + x] == 1;
}

__global__ __launch_bounds__(kRowThreads) void row_count_kernel(const float* __restrict__ N, int H, int W, float thr,
                                                                 int border, const uint8_t* __restrict__ masks, int mH,
                                                                 int mW, int* __restrict__ rowcnt) {
    __shared__ int sh[4];
    const int img = blockIdx.y, y = blockIdx.x;
    const float* row = N + ((size_t)img * H + y) * W;
    int c = 0;
    const bool yok = y >= border && y < H - border;
    for (int x = threadIdx.x; x < W; x += kRowThreads)
        c += (yok && x >= border && x < W - border && row[x] > thr && mask_ok(masks, img, mH, mW, y, x)) ? 1 : 0;
    int total;
    block_excl_scan(c, sh, total);
    if (threadIdx.x == 0) rowcnt[(size_t)img * H + y] = total;
}

__global__ __launch_bounds__(kRowThreads) void row_scan_kernel(const int* __restrict__ rowcnt, int H,
                                                                int* __restrict__ rowoff, int* __restrict__ n_det) {
    __shared__ int sh[4];
    const int img = blockIdx.x;
    int carry = 0;
    for (int base = 0; base < H; base += kRowThreads) {
        const int y = base + threadIdx.x;
        const int v = y < H ? rowcnt[(size_t)img * H + y] : 0;
        int total;
        const int ex = block_excl_scan(v, sh, total);
        if (y < H) rowoff[(size_t)img * H + y] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) n_det[img] = carry;
}

// candidates: per image, (y * W + x) raster index and score
__global__ __launch_bounds__(kRowThreads) void row_emit_kernel(const float* __restrict__ N, int H, int W, float thr,
                                                                int border, const uint8_t* __restrict__ masks, int mH,
                                                                int mW, const int* __restrict__ rowoff, int cap,
                                                                int* __restrict__ cand_idx,
                                                                float* __restrict__ cand_score) {
    __shared__ int sh[4];
    const int img = blockIdx.y, y = blockIdx.x;
    if (!(y >= border && y < H - border)) return;
    const float* row = N + ((size_t)img * H + y) * W;
    int off = rowoff[(size_t)img * H + y];
    for (int base = 0; base < W; base += kRowThreads) {
        const int x = base + threadIdx.x;
        const float s = x < W ? row[x] : 0.0f;
        const int f = (x < W && x >= border && x < W - border && s > thr && mask_ok(masks, img, mH, mW, y, x)) ? 1 : 0;
        int total;
        const int ex = block_excl_scan(f, sh, total);
        if (f && off + ex < cap) {
            cand_idx[(size_t)img * cap + off + ex] = y * W + x;
            cand_score[(size_t)img * cap + off + ex] = s;
        }
        off += total;
    }
}

// ------------------------------------------------------------------ top-k by score, kept in raster order
// gtsfm's Keypoints.get_top_k (common/keypoints.py:89-110) keeps the k highest responses (np.argpartition: order
// implementation-defined); here: exact radix select on the score bits, ties at the threshold broken by raster
// order, selected keypoints emitted in raster order (with k >= N this is the reference's own order).
constexpr int kTopThreads = 256;

__global__ __launch_bounds__(kTopThreads) void topk_select_kernel(const int* __restrict__ cand_idx,
                                                                   const float* __restrict__ cand_score, int cap,
                                                                   const int* __restrict__ n_det, int k, int W,
                                                                   float* __restrict__ out_xy,
                                                                   float* __restrict__ out_score,
                                                                   int* __restrict__ out_count) {
    __shared__ int histo[256];
    __shared__ int sh[4];
    __shared__ int pick[2];
    const int img = blockIdx.x, tid = threadIdx.x;
    const int N = min(n_det[img], cap);
    const int* ci = cand_idx + (size_t)img * cap;
    const float* cs = cand_score + (size_t)img * cap;
    const int kk = min(N, k);
    // keys: larger score first -> order by ~bits (scores are > threshold >= 0, so the bits are monotone)
    uint32_t T = 0xFFFFFFFFu;
    int need_eq = 0;
    if (N > k) {
        uint32_t prefix = 0;
        int need = k;
        for (int pass = 0; pass < 4; ++pass) {
            const int shift = 24 - 8 * pass;
            const uint32_t pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
            for (int i = tid; i < 256; i += kTopThreads) histo[i] = 0;
            __syncthreads();
            for (int i = tid; i < N; i += kTopThreads) {
                const uint32_t key = ~__float_as_uint(cs[i]);
                if ((key & pmask) == (prefix & pmask)) atomicAdd(&histo[(key >> shift) & 255], 1);
            }
            __syncthreads();
            if (tid == 0) {
                int acc = 0, d = 0;
                for (; d < 256; ++d) {
                    if (acc + histo[d] >= need) break;
                    acc += histo[d];
                }
                pick[0] = d;
                pick[1] = need - acc;
            }
            __syncthreads();
            prefix |= (uint32_t)pick[0] << shift;
            need = pick[1];
            __syncthreads();
        }
        T = prefix;
        need_eq = need;  // take keys < T, and the first need_eq keys == T in raster order
    }
    int written = 0, eq_seen = 0;
    for (int base = 0; base < N; base += kTopThreads) {
        const int i = base + tid;
        int sel = 0, eq = 0;
        if (i < N) {
            const uint32_t key = ~__float_as_uint(cs[i]);
            if (N <= k || key < T) sel = 1;
            else if (key == T) eq = 1;
        }
        int eq_total;
        const int eq_ex = block_excl_scan(eq, sh, eq_total);
        if (eq && eq_seen + eq_ex < need_eq) sel = 1;
        int total;
        const int ex = block_excl_scan(sel, sh, total);
        if (sel) {
            const int o = written + ex;
            const int r = ci[i];
            out_xy[((size_t)img * k + o) * 2] = (float)(r % W);
            out_xy[((size_t)img * k + o) * 2 + 1] = (float)(r / W);
            out_score[(size_t)img * k + o] = cs[i];
        }
        written += total;
        eq_seen += eq_total;
    }
    if (tid == 0) out_count[img] = kk;
}

// ------------------------------------------------------------------ descriptors at keypoints
// superpoint.py:196-198 + sample_descriptors (:73-91): dense map L2-normalised per cell, bilinear grid_sample at
// ((kp - s/2 + 0.5) / (w s - s/2 - 0.5), ...) * 2 - 1 with align_corners False and zero padding, L2-normalised.
// One wave per keypoint, 4 channels per lane.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

__global__ __launch_bounds__(64) void desc_sample_kernel(const float* __restrict__ D /*(n,H8,W8,256)*/, int H8, int W8,
                                                         const float* __restrict__ xy, const int* __restrict__ count,
                                                         int k, float* __restrict__ out /*(n,k,256)*/) {
    const int img = blockIdx.y, j = blockIdx.x, lane = threadIdx.x;
    f32x4_t* o = (f32x4_t*)(out + ((size_t)img * k + j) * 256) + lane;
    if (j >= count[img]) {
        *o = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
        return;
    }
    const float kx = xy[((size_t)img * k + j) * 2], ky = xy[((size_t)img * k + j) * 2 + 1];
    // grid coordinates (fp32, the module's operation order)
    float gx = kx - 3.5f, gy = ky - 3.5f;
    gx = gx / (float)(W8 * 8.0 - 4.5);
    gy = gy / (float)(H8 * 8.0 - 4.5);
    gx = gx * 2.0f - 1.0f;
    gy = gy * 2.0f - 1.0f;
    // grid_sampler_compute_source_index, align_corners False: ((g + 1) * size - 1) / 2
    const float ix = ((gx + 1.0f) * (float)W8 - 1.0f) / 2.0f;
    const float iy = ((gy + 1.0f) * (float)H8 - 1.0f) / 2.0f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
    const float wne = (ix - (float)x0) * ((float)y1 - iy);
    const float wsw = ((float)x1 - ix) * (iy - (float)y0);
    const float wse = (ix - (float)x0) * (iy - (float)y0);
    const float* Db = D + (size_t)img * H8 * W8 * 256;
    auto corner = [&](int yy, int xx) -> f32x4_t {
        if (yy < 0 || yy >= H8 || xx < 0 || xx >= W8) return f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
        const f32x4_t v = *((const f32x4_t*)(Db + ((size_t)yy * W8 + xx) * 256) + lane);
        const float ss = wave_sum(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
        const float nrm = fmaxf(sqrtf(ss), 1e-12f);
        return f32x4_t{v[0] / nrm, v[1] / nrm, v[2] / nrm, v[3] / nrm};
    };
    const f32x4_t a = corner(y0, x0), b = corner(y0, x1), c = corner(y1, x0), d = corner(y1, x1);
    f32x4_t r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = a[e] * wnw + b[e] * wne + c[e] * wsw + d[e] * wse;
    const float ss = wave_sum(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]);
    const float nrm = fmaxf(sqrtf(ss), 1e-12f);
    *o = f32x4_t{r[0] / nrm, r[1] / nrm, r[2] / nrm, r[3] / nrm};
}

// ------------------------------------------------------------------ workspace layout
struct SpDims {
    int H, W, H2, W2, H4, W4, H8, W8, Hs, Ws;
};

__host__ SpDims sp_dims(int H, int W) {
    SpDims d;
    d.H = H; d.W = W;
    d.H2 = H / 2; d.W2 = W / 2;
    d.H4 = d.H2 / 2; d.W4 = d.W2 / 2;
    d.H8 = d.H4 / 2; d.W8 = d.W4 / 2;
    d.Hs = 8 * d.H8; d.Ws = 8 * d.W8;
    return d;
}

struct SpLayout {
    size_t buf0, buf1, logits, maps, cand_idx, cand_score, rowcnt, rowoff, ndet, w3, total;
    size_t map_floats;
    int cap;
};

__host__ SpLayout sp_layout(int n, const SpDims& d) {
    SpLayout L{};
    const size_t hw = (size_t)d.H * d.W, h8w8 = (size_t)d.H8 * d.W8;
    size_t b0 = hw * 64, b1 = (size_t)d.H2 * d.W2 * 64;
    b0 = b0 > h8w8 * 512 ? b0 : h8w8 * 512;
    b1 = b1 > h8w8 * 256 ? b1 : h8w8 * 256;
    L.map_floats = (size_t)n * d.Hs * d.Ws;
    L.cap = d.Hs * d.Ws > 0 ? d.Hs * d.Ws : 1;
    size_t o = 0;
    L.buf0 = o; o += gtsfm_align_up((size_t)n * b0 * 4, 256);
    L.buf1 = o; o += gtsfm_align_up((size_t)n * b1 * 4, 256);
    L.logits = o; o += gtsfm_align_up((size_t)n * h8w8 * 128 * 4, 256);
    L.maps = o; o += gtsfm_align_up(L.map_floats * 4 * 6, 256);  // S, P, mask, Q, T, row-pass scratch
    L.cand_idx = o; o += gtsfm_align_up((size_t)n * L.cap * 4, 256);
    L.cand_score = o; o += gtsfm_align_up((size_t)n * L.cap * 4, 256);
    L.rowcnt = o; o += gtsfm_align_up((size_t)n * (d.Hs + 1) * 4, 256);
    L.rowoff = o; o += gtsfm_align_up((size_t)n * (d.Hs + 1) * 4, 256);
    L.ndet = o; o += gtsfm_align_up((size_t)n * 4, 256);
    L.w3 = o; o += gtsfm_align_up(sp_w3_offset(kSpLayers) * sizeof(__bf16), 256);
    L.total = o;
    return L;
}

template <int KS, bool POOL>
hipError_t launch_conv(int n, const float* in, int Hi, int Wi, int in_cstride, int in_c0, int Cin, const float* blob,
                       const __bf16* w3, int layer, float* out, int out_cstride, int out_c0, int Cout,
                       hipStream_t stream) {
    ConvArgs a;
    a.in = in; a.Hi = Hi; a.Wi = Wi; a.in_cstride = in_cstride; a.in_c0 = in_c0; a.Cin = Cin;
    a.w = blob + sp_layer_offset(layer);
    a.cout_pad = kSp[layer].cout_pad;
    a.bias = a.w + (size_t)kSp[layer].k * kSp[layer].k * kSp[layer].cin * a.cout_pad;
    a.out = out; a.out_cstride = out_cstride; a.out_c0 = out_c0; a.Cout = Cout; a.relu = 1;
    a.tiles_x = (Wi + 31) / 32;
    a.tiles_y = (Hi + conv3_rows(KS) - 1) / conv3_rows(KS);
    // pooled rows only (MaxPool2d floors; an odd last conv row is dropped): conv3_rp pooled rows per tile
    if (POOL) a.tiles_y = (Hi / 2 + conv3_rp(KS) - 1) / conv3_rp(KS);
    if (a.tiles_x == 0 || a.tiles_y == 0) return hipSuccess;
    const dim3 grid((unsigned)(a.tiles_x * a.tiles_y * n), (unsigned)((Cout + 63) / 64));
    hipLaunchKernelGGL((conv3_kernel<KS, POOL>), grid, dim3(conv3_threads(KS)), 0, stream, a, w3 + sp_w3_offset(layer));
    return hipGetLastError();
}

}  // namespace

extern "C" {

size_t gtsfm_superpoint_weights_floats(void) { return sp_layer_offset(kSpLayers); }

size_t gtsfm_superpoint_workspace_bytes(int n, int H, int W, int max_kpts) {
    (void)max_kpts;
    if (n <= 0 || H <= 0 || W <= 0) return 0;
    return sp_layout(n, sp_dims(H, W)).total;
}

int gtsfm_superpoint_batched(const uint8_t* d_images, const uint8_t* d_masks, int n, int H, int W, int C,
                             const float* d_weights, int max_kpts, float keypoint_threshold, int nms_radius,
                             int remove_borders, void* d_workspace, size_t workspace_bytes, float* d_xy,
                             float* d_scores, float* d_desc, int* d_count, int* d_n_detected, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n == 0) return GTSFM_OK;
    if (!d_images || !d_weights || !d_workspace || !d_xy || !d_scores || !d_desc || !d_count || n < 0 || H <= 0 ||
        W <= 0 || (C != 1 && C != 3) || max_kpts <= 0 || nms_radius < 0 || remove_borders < 0)
        return GTSFM_ERR_ARG;
    const SpDims d = sp_dims(H, W);
    const SpLayout L = sp_layout(n, d);
    if (workspace_bytes < L.total) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    float* buf0 = (float*)(ws + L.buf0);
    float* buf1 = (float*)(ws + L.buf1);
    float* logits = (float*)(ws + L.logits);
    int* ndet = (int*)(ws + L.ndet);
    if (d.H8 == 0 || d.W8 == 0) {  // too small for one 8x8 cell: no keypoints
        GTSFM_CHECK_HIP(hipMemsetAsync(d_count, 0, (size_t)n * sizeof(int), stream));
        if (d_n_detected) GTSFM_CHECK_HIP(hipMemsetAsync(d_n_detected, 0, (size_t)n * sizeof(int), stream));
        return GTSFM_OK;
    }
    const float* blob = d_weights;
    __bf16* w3 = (__bf16*)(ws + L.w3);
    {
        size_t most = 0;
        for (int l = 1; l < kSpLayers; ++l)
            most = std::max(most, (size_t)kSp[l].k * kSp[l].k * kSp[l].cin * kSp[l].cout_pad);
        hipLaunchKernelGGL(sp_split_weights_kernel, dim3((unsigned)((most + 255) / 256), kSpLayers - 1), dim3(256), 0,
                           stream, blob, w3);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    // shared encoder (superpoint.py:147-158)
    {
        const size_t pix = (size_t)n * H * W;
        hipLaunchKernelGGL(conv1a_kernel, dim3((unsigned)((pix + 255) / 256)), dim3(256), 0, stream, d_images, n, H,
                           W, C, blob + sp_layer_offset(L1A), buf0);
        GTSFM_CHECK_HIP(hipGetLastError());
    }
    GTSFM_CHECK_HIP((launch_conv<3, true>(n, buf0, d.H, d.W, 64, 0, 64, blob, w3, L1B, buf1, 64, 0, 64, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, false>(n, buf1, d.H2, d.W2, 64, 0, 64, blob, w3, L2A, buf0, 64, 0, 64, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, true>(n, buf0, d.H2, d.W2, 64, 0, 64, blob, w3, L2B, buf1, 64, 0, 64, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, false>(n, buf1, d.H4, d.W4, 64, 0, 64, blob, w3, L3A, buf0, 128, 0, 128, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, true>(n, buf0, d.H4, d.W4, 128, 0, 128, blob, w3, L3B, buf1, 128, 0, 128, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, false>(n, buf1, d.H8, d.W8, 128, 0, 128, blob, w3, L4A, buf0, 128, 0, 128, stream)));
    GTSFM_CHECK_HIP((launch_conv<3, false>(n, buf0, d.H8, d.W8, 128, 0, 128, blob, w3, L4B, buf1, 128, 0, 128, stream)));
    // heads: [convPa | convDa] in one 3x3 (128 -> 512), then the two 1x1s (superpoint.py:161-162, 190-191)
    GTSFM_CHECK_HIP((launch_conv<3, false>(n, buf1, d.H8, d.W8, 128, 0, 128, blob, w3, LHEAD, buf0, 512, 0, 512, stream)));
    // convPb: no ReLU; convDb: no ReLU
    auto conv1x1 = [&](int layer, int in_c0, float* out, int out_cstride, int Cout) -> hipError_t {
        ConvArgs a;
        a.in = buf0; a.Hi = d.H8; a.Wi = d.W8; a.in_cstride = 512; a.in_c0 = in_c0; a.Cin = 256;
        a.w = blob + sp_layer_offset(layer);
        a.cout_pad = kSp[layer].cout_pad;
        a.bias = a.w + (size_t)256 * a.cout_pad;
        a.out = out; a.out_cstride = out_cstride; a.out_c0 = 0; a.Cout = Cout; a.relu = 0;
        a.tiles_x = (d.W8 + 31) / 32;
        a.tiles_y = (d.H8 + conv3_rows(1) - 1) / conv3_rows(1);
        const dim3 grid((unsigned)(a.tiles_x * a.tiles_y * n), (unsigned)((Cout + 63) / 64));
        hipLaunchKernelGGL((conv3_kernel<1, false>), grid, dim3(conv3_threads(1)), 0, stream, a, w3 + sp_w3_offset(layer));
        return hipGetLastError();
    };
    GTSFM_CHECK_HIP(conv1x1(LPB, 0, logits, 128, 65));
    GTSFM_CHECK_HIP(conv1x1(LDB, 256, buf1, 256, 256));
    // dense scores + NMS
    float* S = (float*)(ws + L.maps);
    float* P = S + L.map_floats;
    float* M = P + L.map_floats;
    float* Q = M + L.map_floats;
    float* T = Q + L.map_floats;
    float* TMP = T + L.map_floats;
    const size_t cells = (size_t)n * d.H8 * d.W8;
    hipLaunchKernelGGL(scores_kernel, dim3((unsigned)((cells + 63) / 64)), dim3(64), 0, stream, logits, n, d.H8, d.W8,
                       S);
    const size_t tot = L.map_floats;
    const dim3 eg((unsigned)((tot + 255) / 256)), eb(256);
    auto maxpool = [&](const float* src, float* dst) {
        hipLaunchKernelGGL(rowmax_kernel, eg, eb, 0, stream, src, TMP, n, d.Hs, d.Ws, nms_radius);
        hipLaunchKernelGGL(colmax_kernel, eg, eb, 0, stream, (const float*)TMP, dst, n, d.Hs, d.Ws, nms_radius);
    };
    maxpool(S, P);  // max_mask = scores == max_pool(scores)
    hipLaunchKernelGGL(nms_step_kernel, eg, eb, 0, stream, 0, tot, S, (const float*)P, M, (const float*)nullptr,
                       (float*)nullptr);
    for (int it = 0; it < 2; ++it) {
        maxpool(M, Q);  // supp_mask = max_pool(max_mask) > 0
        hipLaunchKernelGGL(nms_step_kernel, eg, eb, 0, stream, 1, tot, S, (const float*)nullptr, M, (const float*)Q,
                           T);  // supp_scores
        maxpool(T, P);
        hipLaunchKernelGGL(nms_step_kernel, eg, eb, 0, stream, 2, tot, S, (const float*)P, M, (const float*)Q, T);
    }
    hipLaunchKernelGGL(nms_step_kernel, eg, eb, 0, stream, 3, tot, S, (const float*)nullptr, M, (const float*)nullptr,
                       T);  // where(max_mask, scores, 0)
    GTSFM_CHECK_HIP(hipGetLastError());
    // raster-order candidates, top-k, descriptors
    int* rowcnt = (int*)(ws + L.rowcnt);
    int* rowoff = (int*)(ws + L.rowoff);
    int* cidx = (int*)(ws + L.cand_idx);
    float* cscore = (float*)(ws + L.cand_score);
    hipLaunchKernelGGL(row_count_kernel, dim3(d.Hs, n), dim3(kRowThreads), 0, stream, T, d.Hs, d.Ws,
                       keypoint_threshold, remove_borders, d_masks, H, W, rowcnt);
    hipLaunchKernelGGL(row_scan_kernel, dim3(n), dim3(kRowThreads), 0, stream, rowcnt, d.Hs, rowoff, ndet);
    hipLaunchKernelGGL(row_emit_kernel, dim3(d.Hs, n), dim3(kRowThreads), 0, stream, T, d.Hs, d.Ws,
                       keypoint_threshold, remove_borders, d_masks, H, W, rowoff, L.cap, cidx, cscore);
    hipLaunchKernelGGL(topk_select_kernel, dim3(n), dim3(kTopThreads), 0, stream, cidx, cscore, L.cap, ndet, max_kpts,
                       d.Ws, d_xy, d_scores, d_count);
    hipLaunchKernelGGL(desc_sample_kernel, dim3(max_kpts, n), dim3(64), 0, stream, buf1, d.H8, d.W8, d_xy, d_count,
                       max_kpts, d_desc);
    GTSFM_CHECK_HIP(hipGetLastError());
    if (d_n_detected)
        GTSFM_CHECK_HIP(hipMemcpyAsync(d_n_detected, ndet, (size_t)n * sizeof(int), hipMemcpyDeviceToDevice, stream));
    return GTSFM_OK;
}

}  // extern "C"
