/*
 * ORACLE — test infrastructure only. CPU restatement of the reference's SIFT detector-descriptor, used as the checker
 * for the HIP extractor and as the CPU baseline. The product path never calls it.
 *
 * Reference path (/root/reference):
 *   gtsfm/frontend/detector_descriptor/sift.py:27-56  rgb_to_gray_cv (utils/images.py:14-41, cv.cvtColor RGB2GRAY),
 *       cv.SIFT_create().detectAndCompute(gray, mask) with every default, cast_to_gtsfm_keypoints
 *       (utils/features.py:16-37: pt, size, response), Keypoints.get_top_k(max_keypoints) (keypoints.py:89-110)
 * Third-party algorithm restated: OpenCV SIFT (opencv-python>=4.5.4.58, environment_linux.yml:50; features2d
 * sift.dispatch.cpp / sift.simd.hpp, float build: SIFT_FIXPT_SCALE 1): nfeatures 0, nOctaveLayers 3,
 * contrastThreshold 0.04, edgeThreshold 10, sigma 1.6, firstOctave -1 (image doubled with INTER_LINEAR and blurred
 * to sigma), nOctaves = round(log2(min side of doubled image) - 2) + 1, Gaussian kernels of size round(8 sigma+1)|1
 * (getGaussianKernel, float taps), separable filtering with BORDER_REFLECT_101, octave bases by INTER_NEAREST
 * decimation of level 3, DoG extrema (threshold floor(0.5*0.04/3*255) = 1, 26-neighbourhood, >= / <=), 5-step
 * quadratic refinement (3x3 solve by Cramer's rule, Matx_FastSolveOp), contrast and edge tests, 36-bin orientation
 * histogram (radius round(4.5 s), sigma 1.5 s, [1 4 6 4 1]/16 smoothing, peaks >= 0.8 max, parabolic interpolation,
 * OpenCV's fastAtan2 polynomial), 4x4x8 descriptor (radius round(3 s sqrt2 5/2), trilinear binning, 0.2 clamp,
 * 512 scaling, saturate_cast<uchar>), removal of duplicated keypoints.
 *
 * Deliberate, documented deviations (shared bit-for-bit with the HIP kernels, so that the two agree exactly):
 *   - exp / exp2 / sin / cos are evaluated by the deterministic polynomial routines below (OpenCV uses its own
 *     exp32f and libm cosf/sinf/powf; differences are ~1 ulp);
 *   - histogram bins accumulate fixed-point int64 contributions (value * 2^24, truncated) instead of float sums, so
 *     the result does not depend on summation order (OpenCV sums in float in pixel order);
 *   - the 2-D Gaussian filtering is computed as acc = k0*s0; acc = fma(k_j, s[-j] + s[+j], acc) rows then columns;
 *   - get_top_k keeps the k largest responses with a deterministic tie-break (octave, layer, row, col, angle) and
 *     returns them in descending response order (the reference's np.argpartition order is implementation-defined).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define N_LAYERS 3
#define SIFT_SIGMA 1.6f
#define SIFT_INIT_SIGMA 0.5f
#define SIFT_IMG_BORDER 5
#define SIFT_MAX_INTERP_STEPS 5
#define SIFT_ORI_HIST_BINS 36
#define SIFT_ORI_SIG_FCTR 1.5f
#define SIFT_ORI_RADIUS (3 * SIFT_ORI_SIG_FCTR)
#define SIFT_ORI_PEAK_RATIO 0.8f
#define SIFT_DESCR_SCL_FCTR 3.f
#define SIFT_DESCR_MAG_THR 0.2f
#define SIFT_INT_DESCR_FCTR 512.f
#define SIFT_CONTRAST 0.04f
#define SIFT_EDGE 10.f
#define MAX_OCTAVES 16
#define MAX_KTAPS 64
#define FIX_SCALE 16777216.0f /* 2^24 */

/* ------------------------------------------------------------------ deterministic math */
float sift_exp2_det(float t) {
    if (t < -126.f) return 0.f;
    const float n = floorf(t);
    const float f = t - n; /* [0, 1) */
    /* 2^f = sum_k (f ln2)^k / k!, degree 8, Horner with fmaf */
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

float sift_exp_det(float x) { return sift_exp2_det(x * 1.4426950408889634f); }

/* sin/cos of an angle in radians (|a| <= 8): Cody-Waite reduction to [-pi/4, pi/4] + Taylor polynomials */
void sift_sincos_det(float a, float* s, float* c) {
    const float k = rintf(a * 0.63661977236758134f); /* 2/pi */
    float r = fmaf(-k, 1.5707963705062866f, a);
    r = fmaf(-k, -4.3711388286737929e-08f, r);
    const float r2 = r * r;
    float sp = fmaf(fmaf(fmaf(-1.9841269841269841e-04f, r2, 8.3333333333333333e-03f), r2, -1.6666666666666667e-01f),
                    r2 * r, r);
    float cp = fmaf(fmaf(fmaf(fmaf(2.4801587301587302e-05f, r2, -1.3888888888888889e-03f), r2,
                              4.1666666666666667e-02f), r2, -0.5f), r2, 1.0f);
    const int q = ((int)k) & 3;
    if (q == 0) { *s = sp; *c = cp; }
    else if (q == 1) { *s = cp; *c = -sp; }
    else if (q == 2) { *s = -sp; *c = -cp; }
    else { *s = -cp; *c = sp; }
}

/* OpenCV hal fastAtan2 (degrees, [0, 360)) */
float sift_fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * 57.29577951308232f, p3 = -0.3258083974640975f * 57.29577951308232f,
                p5 = 0.1555786518463281f * 57.29577951308232f, p7 = -0.04432655554792128f * 57.29577951308232f;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

static inline int64_t to_fix(float v) { return (int64_t)(v * FIX_SCALE); }
static inline float from_fix(int64_t v) { return (float)v * (1.0f / FIX_SCALE); }

/* ------------------------------------------------------------------ Gaussian kernels (getGaussianKernel, float) */
int sift_gauss_kernel(double sigma, float* k) { /* returns ksize; k holds the symmetric half k[0..r] */
    int n = (int)lrint(sigma * 4 * 2 + 1) | 1;
    if (n > 2 * MAX_KTAPS - 1) n = 2 * MAX_KTAPS - 1;
    float full[2 * MAX_KTAPS];
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        full[i] = (float)exp(scale2X * x * x);
        sum += full[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) full[i] = (float)(full[i] * sum);
    const int r = n / 2;
    for (int j = 0; j <= r; ++j) k[j] = full[r + j];
    return n;
}

/* per-level sigmas of buildGaussianPyramid */
void sift_level_sigmas(double* sig) {
    sig[0] = SIFT_SIGMA;
    const double k = pow(2., 1. / N_LAYERS);
    for (int i = 1; i < N_LAYERS + 3; ++i) {
        const double sig_prev = pow(k, (double)(i - 1)) * SIFT_SIGMA;
        const double sig_total = sig_prev * k;
        sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
}

static inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* separable blur, rows then columns (BORDER_REFLECT_101) */
static void blur(const float* src, float* dst, int H, int W, const float* k, int r, float* tmp) {
    for (int y = 0; y < H; ++y) {
        const float* s = src + (size_t)y * W;
        float* t = tmp + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float acc = k[0] * s[x];
            for (int j = 1; j <= r; ++j) acc = fmaf(k[j], s[reflect101(x - j, W)] + s[reflect101(x + j, W)], acc);
            t[x] = acc;
        }
    }
    for (int y = 0; y < H; ++y) {
        float* d = dst + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float acc = k[0] * tmp[(size_t)y * W + x];
            for (int j = 1; j <= r; ++j)
                acc = fmaf(k[j], tmp[(size_t)reflect101(y - j, H) * W + x] + tmp[(size_t)reflect101(y + j, H) * W + x],
                           acc);
            d[x] = acc;
        }
    }
}

/* ------------------------------------------------------------------ image conversions */
void oracle_rgb_to_gray(const uint8_t* rgb, int H, int W, uint8_t* gray) {
    for (int i = 0; i < H * W; ++i) {
        const int R = rgb[3 * i], G = rgb[3 * i + 1], B = rgb[3 * i + 2];
        gray[i] = (uint8_t)((R * 4899 + G * 9617 + B * 1868 + (1 << 13)) >> 14);
    }
}

/* 2x INTER_LINEAR upsampling of a u8 image into float (exact: weights 0.25/0.75 on integers) */
static void upsample2(const uint8_t* g, int H, int W, float* out) {
    const int W2 = 2 * W, H2 = 2 * H;
    for (int y = 0; y < H2; ++y) {
        float fy = (float)((y + 0.5) * 0.5 - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        if (sy < 0) { sy = 0; fy = 0; }
        if (sy >= H - 1) { sy = H - 1; fy = 0; }
        const int sy1 = sy + 1 < H ? sy + 1 : H - 1;
        for (int x = 0; x < W2; ++x) {
            float fx = (float)((x + 0.5) * 0.5 - 0.5);
            int sx = (int)floorf(fx);
            fx -= sx;
            if (sx < 0) { sx = 0; fx = 0; }
            if (sx >= W - 1) { sx = W - 1; fx = 0; }
            const int sx1 = sx + 1 < W ? sx + 1 : W - 1;
            const float r0 = g[sy * W + sx] * (1.f - fx) + g[sy * W + sx1] * fx;
            const float r1 = g[sy1 * W + sx] * (1.f - fx) + g[sy1 * W + sx1] * fx;
            out[(size_t)y * W2 + x] = r0 * (1.f - fy) + r1 * fy;
        }
    }
}

/* ------------------------------------------------------------------ keypoints */
typedef struct {
    float x, y, size, angle, response;
    int o, layer, r, c;      /* pyramid octave (doubled image = 0), layer, refined row/col */
    float xc, xr, xi;        /* sub-pixel offsets */
    float scl_octv;          /* size*0.5/2^o in octave units */
} kp_t;

typedef struct {
    int n_oct;
    int H[MAX_OCTAVES], W[MAX_OCTAVES];
    float* g[MAX_OCTAVES][N_LAYERS + 3];
    float* d[MAX_OCTAVES][N_LAYERS + 2];
} pyr_t;

#define AT(img, W, r, c) ((img)[(size_t)(r) * (W) + (c)])

static int adjust_local_extrema(const pyr_t* P, int o, int* layer_io, int* r_io, int* c_io, float* xc_o, float* xr_o,
                                float* xi_o, float* contr_o) {
    const float img_scale = 1.f / 255.f;
    const float deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale, cross_deriv_scale = img_scale * 0.25f;
    int layer = *layer_io, r = *r_io, c = *c_io;
    const int W = P->W[o], H = P->H[o];
    float xi = 0, xr = 0, xc = 0;
    int i = 0;
    for (; i < SIFT_MAX_INTERP_STEPS; i++) {
        const float* img = P->d[o][layer];
        const float* prev = P->d[o][layer - 1];
        const float* next = P->d[o][layer + 1];
        const float dD0 = (AT(img, W, r, c + 1) - AT(img, W, r, c - 1)) * deriv_scale;
        const float dD1 = (AT(img, W, r + 1, c) - AT(img, W, r - 1, c)) * deriv_scale;
        const float dD2 = (AT(next, W, r, c) - AT(prev, W, r, c)) * deriv_scale;
        const float v2 = AT(img, W, r, c) * 2;
        const float dxx = (AT(img, W, r, c + 1) + AT(img, W, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (AT(img, W, r + 1, c) + AT(img, W, r - 1, c) - v2) * second_deriv_scale;
        const float dss = (AT(next, W, r, c) + AT(prev, W, r, c) - v2) * second_deriv_scale;
        const float dxy = (AT(img, W, r + 1, c + 1) - AT(img, W, r + 1, c - 1) - AT(img, W, r - 1, c + 1) +
                           AT(img, W, r - 1, c - 1)) * cross_deriv_scale;
        const float dxs = (AT(next, W, r, c + 1) - AT(next, W, r, c - 1) - AT(prev, W, r, c + 1) +
                           AT(prev, W, r, c - 1)) * cross_deriv_scale;
        const float dys = (AT(next, W, r + 1, c) - AT(next, W, r - 1, c) - AT(prev, W, r + 1, c) +
                           AT(prev, W, r - 1, c)) * cross_deriv_scale;
        /* H = [dxx dxy dxs; dxy dyy dys; dxs dys dss], X = H^-1 dD by Cramer's rule (Matx_FastSolveOp<3,1>) */
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys, a22 = dss;
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
            fabsf(xc) > (float)(INT32_MAX / 3))
            return 0;
        c += (int)rintf(xc);
        r += (int)rintf(xr);
        layer += (int)rintf(xi);
        if (layer < 1 || layer > N_LAYERS || c < SIFT_IMG_BORDER || c >= W - SIFT_IMG_BORDER ||
            r < SIFT_IMG_BORDER || r >= H - SIFT_IMG_BORDER)
            return 0;
    }
    if (i >= SIFT_MAX_INTERP_STEPS) return 0;
    {
        const float* img = P->d[o][layer];
        const float* prev = P->d[o][layer - 1];
        const float* next = P->d[o][layer + 1];
        const float dD0 = (AT(img, W, r, c + 1) - AT(img, W, r, c - 1)) * deriv_scale;
        const float dD1 = (AT(img, W, r + 1, c) - AT(img, W, r - 1, c)) * deriv_scale;
        const float dD2 = (AT(next, W, r, c) - AT(prev, W, r, c)) * deriv_scale;
        const float t = dD0 * xc + dD1 * xr + dD2 * xi;
        const float contr = AT(img, W, r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * N_LAYERS < SIFT_CONTRAST) return 0;
        const float v2 = AT(img, W, r, c) * 2.f;
        const float dxx = (AT(img, W, r, c + 1) + AT(img, W, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (AT(img, W, r + 1, c) + AT(img, W, r - 1, c) - v2) * second_deriv_scale;
        const float dxy = (AT(img, W, r + 1, c + 1) - AT(img, W, r + 1, c - 1) - AT(img, W, r - 1, c + 1) +
                           AT(img, W, r - 1, c - 1)) * cross_deriv_scale;
        const float tr = dxx + dyy;
        const float det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * SIFT_EDGE >= (SIFT_EDGE + 1) * (SIFT_EDGE + 1) * det) return 0;
        *contr_o = contr;
    }
    *layer_io = layer;
    *r_io = r;
    *c_io = c;
    *xc_o = xc;
    *xr_o = xr;
    *xi_o = xi;
    return 1;
}

/* 36-bin orientation histogram (fixed-point accumulation), smoothed; returns the maximum */
static float orientation_hist(const float* img, int H, int W, int py, int px, int radius, float sigma, float* hist) {
    const int n = SIFT_ORI_HIST_BINS;
    int64_t acc[SIFT_ORI_HIST_BINS];
    memset(acc, 0, sizeof(acc));
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    for (int i = -radius; i <= radius; i++) {
        const int y = py + i;
        if (y <= 0 || y >= H - 1) continue;
        for (int j = -radius; j <= radius; j++) {
            const int x = px + j;
            if (x <= 0 || x >= W - 1) continue;
            const float dx = AT(img, W, y, x + 1) - AT(img, W, y, x - 1);
            const float dy = AT(img, W, y - 1, x) - AT(img, W, y + 1, x);
            const float w = sift_exp_det((float)(i * i + j * j) * expf_scale);
            const float ori = sift_fast_atan2(dy, dx);
            const float mag = sqrtf(fmaf(dx, dx, dy * dy));
            int bin = (int)rintf((n / 360.f) * ori);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
            acc[bin] += to_fix(w * mag);
        }
    }
    float t[SIFT_ORI_HIST_BINS + 4];
    for (int i = 0; i < n; ++i) t[i + 2] = from_fix(acc[i]);
    t[1] = t[n + 1];
    t[0] = t[n];
    t[n + 2] = t[2];
    t[n + 3] = t[3];
    float maxval = 0.f;
    for (int i = 0; i < n; i++) {
        hist[i] = (t[i] + t[i + 4]) * (1.f / 16.f) + (t[i + 1] + t[i + 3]) * (4.f / 16.f) + t[i + 2] * (6.f / 16.f);
        maxval = i == 0 ? hist[0] : fmaxf(maxval, hist[i]);
    }
    return maxval;
}

/* 4x4x8 SIFT descriptor of one keypoint (fixed-point trilinear accumulation) -> 128 u8-valued floats */
void sift_descriptor(const float* img, int H, int W, float ptx, float pty, float ori, float scl, float* dst) {
    const int d = 4, n = 8;
    const int px = (int)rintf(ptx), py = (int)rintf(pty);
    float sin_t, cos_t;
    sift_sincos_det(ori * (float)(3.14159265358979323846 / 180), &sin_t, &cos_t);
    const float bins_per_rad = n / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = SIFT_DESCR_SCL_FCTR * scl;
    int radius = (int)rintf(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    const int diag = (int)sqrt(((double)W) * W + ((double)H) * H);
    if (radius > diag) radius = diag;
    cos_t /= hist_width;
    sin_t /= hist_width;
    int64_t hist[(4 + 2) * (4 + 2) * (8 + 2)];
    memset(hist, 0, sizeof(hist));
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            float rbin = r_rot + d / 2 - 0.5f;
            float cbin = c_rot + d / 2 - 0.5f;
            const int r = py + i, c = px + j;
            if (!(rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < H - 1 && c > 0 && c < W - 1)) continue;
            const float dx = AT(img, W, r, c + 1) - AT(img, W, r, c - 1);
            const float dy = AT(img, W, r - 1, c) - AT(img, W, r + 1, c);
            const float wexp = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
            const float o = sift_fast_atan2(dy, dx);
            const float mag0 = sqrtf(fmaf(dx, dx, dy * dy));
            const float w = sift_exp_det(wexp);
            float obin = (o - ori) * bins_per_rad;
            const float mag = mag0 * w;
            const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
            int o0 = (int)floorf(obin);
            rbin -= r0;
            cbin -= c0;
            obin -= o0;
            if (o0 < 0) o0 += n;
            if (o0 >= n) o0 -= n;
            const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
            const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
            const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
            const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
            const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
            const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
            const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
            const int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
            hist[idx] += to_fix(v_rco000);
            hist[idx + 1] += to_fix(v_rco001);
            hist[idx + (n + 2)] += to_fix(v_rco010);
            hist[idx + (n + 3)] += to_fix(v_rco011);
            hist[idx + (d + 2) * (n + 2)] += to_fix(v_rco100);
            hist[idx + (d + 2) * (n + 2) + 1] += to_fix(v_rco101);
            hist[idx + (d + 3) * (n + 2)] += to_fix(v_rco110);
            hist[idx + (d + 3) * (n + 2) + 1] += to_fix(v_rco111);
        }
    for (int i = 0; i < d; i++)
        for (int j = 0; j < d; j++) {
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            float h[10];
            for (int k = 0; k < n + 2; ++k) h[k] = from_fix(hist[idx + k]);
            h[0] += h[n];
            h[1] += h[n + 1];
            for (int k = 0; k < n; k++) dst[(i * d + j) * n + k] = h[k];
        }
    const int len = d * d * n;
    float nrm2 = 0;
    for (int k = 0; k < len; k++) nrm2 += dst[k] * dst[k];
    const float thr = sqrtf(nrm2) * SIFT_DESCR_MAG_THR;
    nrm2 = 0;
    for (int i = 0; i < len; i++) {
        const float val = fminf(dst[i], thr);
        dst[i] = val;
        nrm2 += val * val;
    }
    nrm2 = SIFT_INT_DESCR_FCTR / fmaxf(sqrtf(nrm2), FLT_EPSILON);
    for (int k = 0; k < len; k++) {
        int v = (int)rintf(dst[k] * nrm2);
        dst[k] = (float)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
}

static int kp_cmp_topk(const void* a, const void* b) {
    const kp_t* x = (const kp_t*)a;
    const kp_t* y = (const kp_t*)b;
    if (x->response != y->response) return x->response > y->response ? -1 : 1;
    if (x->o != y->o) return x->o - y->o;
    if (x->layer != y->layer) return x->layer - y->layer;
    if (x->r != y->r) return x->r - y->r;
    if (x->c != y->c) return x->c - y->c;
    if (x->angle != y->angle) return x->angle < y->angle ? -1 : 1;
    return 0;
}

int sift_num_octaves(int H, int W) {
    const int m = 2 * (H < W ? H : W);
    int n = (int)lrint(log((double)m) / log(2.) - 2) + 1;
    if (n > MAX_OCTAVES) n = MAX_OCTAVES;
    return n;
}

/*
 * SIFT on one u8 gray image. Writes up to max_kpts keypoints (rows of 5 floats: x, y, size, angle, response; in
 * original-image pixels, descending response) and their 128-D descriptors. Returns the count kept;
 * *n_detected receives the number of keypoints before the top-k cut.
 */
/* mask (H0 x W0 u8, may be NULL): cv::SIFT::detectAndCompute(gray, mask) keeps a keypoint iff
 * mask[(int)(y + 0.5f)][(int)(x + 0.5f)] != 0 (KeyPointsFilter::runByPixelsMask), after detection and before the
 * caller's top-k (reference frontend/detector_descriptor/sift.py:47-56). n_detected counts the keypoints kept. */
int oracle_sift_detect_describe_masked(const uint8_t* gray, const uint8_t* mask, int H0, int W0, int max_kpts,
                                       float* kp_out, float* desc_out, int* n_detected) {
    pyr_t P;
    memset(&P, 0, sizeof(P));
    P.n_oct = sift_num_octaves(H0, W0);
    double sig[N_LAYERS + 3];
    sift_level_sigmas(sig);
    float ktab[N_LAYERS + 3][MAX_KTAPS];
    int krad[N_LAYERS + 3];
    const double sig_diff = sqrt(fmax(SIFT_SIGMA * SIFT_SIGMA - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4, 0.01));
    krad[0] = sift_gauss_kernel((double)(float)sig_diff, ktab[0]) / 2;
    for (int i = 1; i < N_LAYERS + 3; ++i) krad[i] = sift_gauss_kernel(sig[i], ktab[i]) / 2;
    int H = 2 * H0, W = 2 * W0;
    float* up = (float*)malloc(sizeof(float) * (size_t)H * W);
    float* tmp = (float*)malloc(sizeof(float) * (size_t)H * W);
    upsample2(gray, H0, W0, up);
    for (int o = 0; o < P.n_oct; ++o) {
        P.H[o] = H;
        P.W[o] = W;
        for (int i = 0; i < N_LAYERS + 3; ++i) P.g[o][i] = (float*)malloc(sizeof(float) * (size_t)H * W);
        if (o == 0) {
            blur(up, P.g[0][0], H, W, ktab[0], krad[0], tmp);
        } else {
            const float* src = P.g[o - 1][N_LAYERS];
            const int Ws = P.W[o - 1];
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x) P.g[o][0][(size_t)y * W + x] = src[(size_t)(2 * y) * Ws + 2 * x];
        }
        for (int i = 1; i < N_LAYERS + 3; ++i) blur(P.g[o][i - 1], P.g[o][i], H, W, ktab[i], krad[i], tmp);
        for (int i = 0; i < N_LAYERS + 2; ++i) {
            P.d[o][i] = (float*)malloc(sizeof(float) * (size_t)H * W);
            for (size_t k = 0; k < (size_t)H * W; ++k) P.d[o][i][k] = P.g[o][i + 1][k] - P.g[o][i][k];
        }
        H /= 2;
        W /= 2;
    }
    free(up);
    free(tmp);

    /* extrema, refinement, orientation */
    size_t cap = 4096, nk = 0;
    kp_t* kps = (kp_t*)malloc(sizeof(kp_t) * cap);
    const float threshold = floorf(0.5f * SIFT_CONTRAST / N_LAYERS * 255.f);
    for (int o = 0; o < P.n_oct; ++o) {
        const int Wo = P.W[o], Ho = P.H[o];
        /* locations already emitted (duplicates are identical: removeDuplicatedSorted) */
        uint8_t* seen = (uint8_t*)calloc((size_t)Wo * Ho * (N_LAYERS + 2), 1);
        for (int i = 1; i <= N_LAYERS; ++i) {
            const float* prev = P.d[o][i - 1];
            const float* img = P.d[o][i];
            const float* next = P.d[o][i + 1];
            for (int r = SIFT_IMG_BORDER; r < Ho - SIFT_IMG_BORDER; r++)
                for (int c = SIFT_IMG_BORDER; c < Wo - SIFT_IMG_BORDER; c++) {
                    const float val = AT(img, Wo, r, c);
                    if (!(fabsf(val) > threshold)) continue;
                    int ismax = val > 0, ismin = val < 0;
                    for (int dy = -1; dy <= 1 && (ismax || ismin); ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            const float a = AT(prev, Wo, r + dy, c + dx), b = AT(next, Wo, r + dy, c + dx);
                            const float m = AT(img, Wo, r + dy, c + dx);
                            if (ismax && !(val >= a && val >= b && val >= m)) ismax = 0;
                            if (ismin && !(val <= a && val <= b && val <= m)) ismin = 0;
                        }
                    if (!ismax && !ismin) continue;
                    int layer = i, rr = r, cc = c;
                    float xc, xr, xi, contr;
                    if (!adjust_local_extrema(&P, o, &layer, &rr, &cc, &xc, &xr, &xi, &contr)) continue;
                    const size_t loc = ((size_t)layer * Ho + rr) * Wo + cc;
                    if (seen[loc]) continue;
                    seen[loc] = 1;
                    const float size_oct = SIFT_SIGMA * sift_exp2_det(((float)layer + xi) / N_LAYERS);
                    const float scl_octv = size_oct; /* kpt.size*0.5/(1<<o) */
                    float hist[SIFT_ORI_HIST_BINS];
                    const float omax = orientation_hist(P.g[o][layer], Ho, Wo, rr, cc,
                                                        (int)rintf(SIFT_ORI_RADIUS * scl_octv),
                                                        SIFT_ORI_SIG_FCTR * scl_octv, hist);
                    const float mag_thr = omax * SIFT_ORI_PEAK_RATIO;
                    const int n = SIFT_ORI_HIST_BINS;
                    for (int j = 0; j < n; j++) {
                        const int l = j > 0 ? j - 1 : n - 1;
                        const int r2 = j < n - 1 ? j + 1 : 0;
                        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                            float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                            bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
                            float angle = 360.f - (360.f / n) * bin;
                            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
                            if (nk == cap) {
                                cap *= 2;
                                kps = (kp_t*)realloc(kps, sizeof(kp_t) * cap);
                            }
                            kp_t* k = &kps[nk++];
                            const float sc = (float)(1 << o) * 0.5f;
                            k->x = ((float)cc + xc) * sc;
                            k->y = ((float)rr + xr) * sc;
                            k->size = size_oct * (float)(1 << o) * 2.f * 0.5f;
                            k->angle = angle;
                            k->response = fabsf(contr);
                            k->o = o;
                            k->layer = layer;
                            k->r = rr;
                            k->c = cc;
                            k->xc = xc;
                            k->xr = xr;
                            k->xi = xi;
                            k->scl_octv = scl_octv;
                        }
                    }
                }
        }
        free(seen);
    }
    if (mask) {
        size_t w = 0;
        for (size_t k = 0; k < nk; ++k) {
            const int yy = (int)(kps[k].y + 0.5f), xx = (int)(kps[k].x + 0.5f);
            if (yy < 0 || yy >= H0 || xx < 0 || xx >= W0 || mask[(size_t)yy * W0 + xx] == 0) continue;
            kps[w++] = kps[k];
        }
        nk = w;
    }
    if (n_detected) *n_detected = (int)nk;
    qsort(kps, nk, sizeof(kp_t), kp_cmp_topk);
    const int nout = (int)(nk < (size_t)max_kpts ? nk : (size_t)max_kpts);
    for (int k = 0; k < nout; ++k) {
        const kp_t* kp = &kps[k];
        kp_out[5 * k + 0] = kp->x;
        kp_out[5 * k + 1] = kp->y;
        kp_out[5 * k + 2] = kp->size;
        kp_out[5 * k + 3] = kp->angle;
        kp_out[5 * k + 4] = kp->response;
        float angle = 360.f - kp->angle;
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        if (desc_out)
            sift_descriptor(P.g[kp->o][kp->layer], P.H[kp->o], P.W[kp->o], (float)kp->c + kp->xc,
                            (float)kp->r + kp->xr, angle, kp->scl_octv, desc_out + (size_t)128 * k);
    }
    free(kps);
    for (int o = 0; o < P.n_oct; ++o) {
        for (int i = 0; i < N_LAYERS + 3; ++i) free(P.g[o][i]);
        for (int i = 0; i < N_LAYERS + 2; ++i) free(P.d[o][i]);
    }
    return nout;
}

int oracle_sift_detect_describe(const uint8_t* gray, int H0, int W0, int max_kpts, float* kp_out, float* desc_out,
                                int* n_detected) {
    return oracle_sift_detect_describe_masked(gray, NULL, H0, W0, max_kpts, kp_out, desc_out, n_detected);
}

/* Debug / parity hook: the Gaussian level (o, i) of an image into out (size returned through H, W). */
int oracle_sift_pyramid_level(const uint8_t* gray, int H0, int W0, int o_want, int i_want, float* out, int* Ho,
                              int* Wo) {
    double sig[N_LAYERS + 3];
    sift_level_sigmas(sig);
    float ktab[N_LAYERS + 3][MAX_KTAPS];
    int krad[N_LAYERS + 3];
    const double sig_diff = sqrt(fmax(SIFT_SIGMA * SIFT_SIGMA - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4, 0.01));
    krad[0] = sift_gauss_kernel((double)(float)sig_diff, ktab[0]) / 2;
    for (int i = 1; i < N_LAYERS + 3; ++i) krad[i] = sift_gauss_kernel(sig[i], ktab[i]) / 2;
    int H = 2 * H0, W = 2 * W0;
    float* cur[N_LAYERS + 3];
    float* up = (float*)malloc(sizeof(float) * (size_t)H * W);
    float* tmp = (float*)malloc(sizeof(float) * (size_t)H * W);
    upsample2(gray, H0, W0, up);
    for (int i = 0; i < N_LAYERS + 3; ++i) cur[i] = (float*)malloc(sizeof(float) * (size_t)H * W);
    blur(up, cur[0], H, W, ktab[0], krad[0], tmp);
    for (int o = 0;; ++o) {
        for (int i = 1; i < N_LAYERS + 3; ++i) blur(cur[i - 1], cur[i], H, W, ktab[i], krad[i], tmp);
        if (o == o_want) {
            memcpy(out, cur[i_want], sizeof(float) * (size_t)H * W);
            *Ho = H;
            *Wo = W;
            break;
        }
        const int Hn = H / 2, Wn = W / 2;
        for (int y = 0; y < Hn; ++y)
            for (int x = 0; x < Wn; ++x) up[(size_t)y * Wn + x] = cur[N_LAYERS][(size_t)(2 * y) * W + 2 * x];
        memcpy(cur[0], up, sizeof(float) * (size_t)Hn * Wn);
        H = Hn;
        W = Wn;
    }
    for (int i = 0; i < N_LAYERS + 3; ++i) free(cur[i]);
    free(up);
    free(tmp);
    return 0;
}
