// Implicit-GEMM 3x3 / 1x1 convolution on the bf16 matrix cores at fp32 accuracy (three-plane split products), shared
// by SuperPoint's encoder and heads (superpoint.hip) and NetVLAD's VGG16 backbone (netvlad.hip). Included inside each
// translation unit's anonymous namespace.
#pragma once

constexpr int kCinChunk = 16;

struct ConvArgs {
    const float* in;   // (n, Hi, Wi, in_cstride), channels [in_c0, in_c0 + Cin)
    int Hi, Wi, in_cstride, in_c0, Cin;
    const float* w;    // [k*k][Cin][cout_pad]
    const float* bias; // [cout_pad]
    int cout_pad;
    float* out;        // (n, Ho, Wo, out_cstride), channels [out_c0, out_c0 + Cout)
    int out_cstride, out_c0, Cout, relu;
    int tiles_x, tiles_y;
};

// ------------------------------------------------------------------ implicit-GEMM convolution, fp32-accurate bf16
// A wave's MFMA tile: 2 rows x 16 columns of pixels (pixel i -> row i / 16, column i % 16) x 32 output channels, on
// v_mfma_f32_32x32x16_bf16 with the three-plane split products of superglue.hip's sg_gemm3_kernel (x = x_h + x_m + x_l in bf16; six plane products per MFMA step; the dropped ones
// are below 2^-23 |a b|): one 16-channel tap is one MFMA k-step of 16 instead of eight 32x32x2 f32 steps. The input
// patch is split as it is staged ([plane][pixel][16] bf16); the weights are split once per call into
// [tap][Cin / 16][plane][cout][16] (sp_split_weights_kernel) and staged as [tap][plane][64 couts][16]. A lane's
// 16-byte fragment (8 channels) sits in half kh ^ ((row >> 3) & 1) of its 32-byte row, so the 16 rows one ds_read_b128
// phase touches fall on distinct banks.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void sp_split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

__device__ __forceinline__ int swz16(int row, int half) { return 8 * (half ^ ((row >> 3) & 1)); }

// A workgroup = conv3_rp row pairs x (4 / conv3_nt) waves over conv3_rows conv rows x 32 columns x 64 output
// channels: the staged
// 16-channel weight slab (55 KB at 3 x 3) is shared by all of them, so its L2 traffic per MFMA falls with the rows.
// C3 per step (profiles/r05bj_*, r05bk_*): 1 / 2 / 3 / 4 row pairs -> conv3 3x3+pool 5148 / 4074 / 4117 / 3927 us,
// 3x3 1625 / 1288 / 1364 / 1285 us per launch (4: 16 waves, one workgroup per CU, 104 VGPRs).
// conv3_nt: 32-channel output tiles per wave (2: each A fragment read from LDS feeds both). 3 x 3: 8 row pairs x 2
// tiles -> 3709 / 1250 us (16 waves, 118 VGPRs; profiles/r05bm_*); the 1 x 1 heads on the 1/8 grid keep 4 row
// pairs x 1 tile (285 against 335 us with 16-row tiles).
__host__ __device__ constexpr int conv3_rp(int ks) { return ks == 3 ? 8 : 4; }
__host__ __device__ constexpr int conv3_nt(int ks) { return ks == 3 ? 2 : 1; }
__host__ __device__ constexpr int conv3_rows(int ks) { return 2 * conv3_rp(ks); }
__host__ __device__ constexpr int conv3_threads(int ks) { return 64 * (4 / conv3_nt(ks)) * conv3_rp(ks); }

template <int KS, bool POOL>
__global__ __launch_bounds__(conv3_threads(KS), 1) void conv3_kernel(ConvArgs a, const __bf16* __restrict__ w3) {
    constexpr int kConv3NT = conv3_nt(KS), kConv3Rows = conv3_rows(KS), kConv3Threads = conv3_threads(KS);
    constexpr int R = KS / 2;
    constexpr int PH = kConv3Rows + 2 * R, PW = 32 + 2 * R;
    constexpr int kPU = PH * PW * 2;             // patch staging units (pixel, 8-channel half)
    constexpr int kWU = KS * KS * 3 * 64 * 2;    // weight staging units (tap, plane, cout, half)
    constexpr int kNP = (kPU + kConv3Threads - 1) / kConv3Threads;
    constexpr int kNW = (kWU + kConv3Threads - 1) / kConv3Threads;
    __shared__ __attribute__((aligned(16))) __bf16 patch[3][PH * PW][16];
    __shared__ __attribute__((aligned(16))) __bf16 wt[KS * KS][3][64][16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ct = blockIdx.y;
    int t = blockIdx.x;
    const int tx = t % a.tiles_x;
    t /= a.tiles_x;
    const int ty = t % a.tiles_y;
    const int img = t / a.tiles_y;
    const int y0 = kConv3Rows * ty, x0 = 32 * tx;
    // wr: the wave's row pair; wn: its output-channel tile (kConv3NT == 1)
    const int wx = wave & 1, wn = kConv3NT == 1 ? (wave >> 1) & 1 : 0, wr = kConv3NT == 1 ? wave >> 2 : wave >> 1;
    const int i = lane & 31, kh = lane >> 5;
    const int prow = (i >> 4) + 2 * wr, pcol = 16 * wx + (i & 15);
    const float* inb = a.in + (size_t)img * a.Hi * a.Wi * a.in_cstride + a.in_c0;
    f32x16 acc[kConv3NT];
#pragma unroll
    for (int nt = 0; nt < kConv3NT; ++nt) acc[nt] = f32x16{};
    f32x4 pv[kNP][2];
    u32x4 wv[kNW];
    auto load = [&](int c0) {
#pragma unroll
        for (int u = 0; u < kNP; ++u) {
            const int e = tid + u * kConv3Threads;
            const int pix = e >> 1, hf = e & 1;
            const int py = pix / PW, px = pix - py * PW;
            const int gy = y0 - R + py, gx = x0 - R + px;
            pv[u][0] = pv[u][1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            if (e < kPU && gy >= 0 && gy < a.Hi && gx >= 0 && gx < a.Wi) {
                const float* src = inb + ((size_t)gy * a.Wi + gx) * a.in_cstride + c0 + 8 * hf;
                pv[u][0] = *(const f32x4*)src;
                pv[u][1] = *(const f32x4*)(src + 4);
            }
        }
        const int chunk = c0 / kCinChunk, nchunk = a.Cin / kCinChunk;
#pragma unroll
        for (int u = 0; u < kNW; ++u) {
            const int e = tid + u * kConv3Threads;
            if (e < kWU) {
                const int hf = e & 1, co = (e >> 1) & 63, p = (e >> 7) % 3, kk = (e >> 7) / 3;
                wv[u] = *(const u32x4*)(w3 + ((((size_t)kk * nchunk + chunk) * 3 + p) * a.cout_pad + 64 * ct + co) * 16 +
                                        8 * hf);
            }
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int u = 0; u < kNP; ++u) {
            const int e = tid + u * kConv3Threads;
            if (e < kPU) {
                const int pix = e >> 1, hf = e & 1;
                bf16x8 h, m, l;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    __bf16 hh, mm, ll;
                    sp_split3(pv[u][j >> 2][j & 3], hh, mm, ll);
                    h[j] = hh;
                    m[j] = mm;
                    l[j] = ll;
                }
                const int o = swz16(pix, hf);
                *(bf16x8*)&patch[0][pix][o] = h;
                *(bf16x8*)&patch[1][pix][o] = m;
                *(bf16x8*)&patch[2][pix][o] = l;
            }
        }
#pragma unroll
        for (int u = 0; u < kNW; ++u) {
            const int e = tid + u * kConv3Threads;
            if (e < kWU) {
                const int hf = e & 1, co = (e >> 1) & 63, p = (e >> 7) % 3, kk = (e >> 7) / 3;
                *(u32x4*)&wt[kk][p][co][swz16(co, hf)] = wv[u];
            }
        }
    };
    load(0);
    stash();
    __syncthreads();
    for (int c0 = 0; c0 < a.Cin; c0 += kCinChunk) {
        const bool more = c0 + kCinChunk < a.Cin;
        if (more) load(c0 + kCinChunk);
#pragma unroll
        for (int ky = 0; ky < KS; ++ky)
#pragma unroll
            for (int kx = 0; kx < KS; ++kx) {
                const int pix = (prow + ky) * PW + pcol + kx, kk = ky * KS + kx;
                const int po = swz16(pix, kh);
                const bf16x8 a0 = *(const bf16x8*)&patch[0][pix][po];
                const bf16x8 a1 = *(const bf16x8*)&patch[1][pix][po];
                const bf16x8 a2 = *(const bf16x8*)&patch[2][pix][po];
#pragma unroll
                for (int nt = 0; nt < kConv3NT; ++nt) {
                    const int ncol = (lane & 31) + 32 * (wn + nt), wo = swz16(ncol, kh);
                    const bf16x8 b0 = *(const bf16x8*)&wt[kk][0][ncol][wo];
                    const bf16x8 b1 = *(const bf16x8*)&wt[kk][1][ncol][wo];
                    const bf16x8 b2 = *(const bf16x8*)&wt[kk][2][ncol][wo];
                    f32x16 c = acc[nt];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c, 0, 0, 0);
                    acc[nt] = c;
                }
            }
        if (!more) break;
        __syncthreads();
        stash();
        __syncthreads();
    }
    // epilogue (conv_mfma_kernel's): acc[g] = conv output at tile pixel 4 kh + (g & 3) + 8 (g >> 2), channel ncol
#pragma unroll
    for (int nt = 0; nt < kConv3NT; ++nt) {
    const f32x16& acc_nt = acc[nt];
    const int ncol = (lane & 31) + 32 * (wn + nt);
    const int co = 64 * ct + ncol;
    if (co >= a.Cout) continue;
    const float b = a.bias[co];
    float* outb = a.out + a.out_c0 + co;
    if constexpr (POOL) {
        const int Ho = a.Hi / 2, Wo = a.Wi / 2;
        const int py = y0 / 2 + wr;
        if (py >= Ho) continue;
#pragma unroll
        for (int qa = 0; qa < 2; ++qa)
#pragma unroll
            for (int rp = 0; rp < 2; ++rp) {
                const int g0 = 4 * qa + 2 * rp, g1 = 4 * (qa + 2) + 2 * rp;
                float v = fmaxf(fmaxf(acc_nt[g0], acc_nt[g0 + 1]), fmaxf(acc_nt[g1], acc_nt[g1 + 1]));
                v = v + b;
                if (a.relu) v = v > 0.0f ? v : 0.0f;
                const int px = x0 / 2 + 8 * wx + 4 * qa + 2 * kh + rp;
                if (px < Wo) outb[(((size_t)img * Ho + py) * Wo + px) * a.out_cstride] = v;
            }
    } else {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int ip = 4 * kh + (g & 3) + 8 * (g >> 2);
            const int y = y0 + 2 * wr + (ip >> 4), x = x0 + 16 * wx + (ip & 15);
            if (y >= a.Hi || x >= a.Wi) continue;
            float v = acc_nt[g] + b;
            if (a.relu) v = v > 0.0f ? v : 0.0f;
            outb[(((size_t)img * a.Hi + y) * a.Wi + x) * a.out_cstride] = v;
        }
    }
    }
}
