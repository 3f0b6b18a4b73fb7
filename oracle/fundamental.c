/*
 * ORACLE — test infrastructure only. CPU restatement of the reference's fundamental-matrix verifier path
 * (use_intrinsics_in_verification=False), the checker for the HIP F kernel. The product path never calls it.
 *
 * Reference path (/root/reference):
 *   gtsfm/frontend/verifier/opencv_verifier_base.py:61-99  verify(): M < 8 -> failure (verifier_base.py:14,39-44),
 *       estimate_F on pixel coordinates, E = K2^T F K1 (utils/verification.py:97-110), inlier idxs, inlier ratio,
 *       recover_relative_pose_from_essential_matrix (utils/verification.py:52-94: normalise the inliers with K,
 *       cv.recoverPose)
 *   gtsfm/frontend/verifier/ransac.py:84-111  cv2.findFundamentalMat(x1, x2, FM_RANSAC,
 *       ransacReprojThreshold = px, confidence = 0.999999, maxIters = 1000000)
 * Third-party algorithm restated (OpenCV, opencv-python>=4.5.4.58, environment_linux.yml:50; source absent here):
 *   - points are converted to float32 (findFundamentalMat converts its inputs to CV_32F);
 *   - FM_RANSAC with >= 15 points: RANSAC over 7-point samples, model count > max(best, 6) replaces the best,
 *     iteration bound RANSACUpdateNumIters(conf, 1 - best/M, 7, n); with 8..14 points: LMedS over 7-point
 *     samples (outlier ratio 0.45 for the iteration count, the model with the least median error wins,
 *     sigma = 2.5 * 1.4826 * (1 + 5 / (M - 7)) * sqrt(median), sigma >= 0.001, inliers err <= sigma^2);
 *   - sample check: no three collinear points in either image (FMEstimatorCallback::checkSubset, float test
 *     |dx2 dy1 - dy2 dx1| <= FLT_EPSILON (|dx1| + |dy1| + |dx2| + |dy2|), applied here to every triple);
 *   - 7-point solver (run7Point): 2-dim null space {f1, f2} of the 7x9 epipolar system, F = l (f1 - f2) + f2,
 *     det F = 0 as a cubic in l, one F per real root, scaled so F33 = 1 when |F33| > DBL_EPSILON. Restated with
 *     Hartley-normalised sample points (the same rank-2 pencil, better conditioned) and a Gauss-Jordan null space;
 *     cubic roots by bisection on the monotone pieces (no libm transcendental, so the GPU computes the same bits);
 *   - error (FMEstimatorCallback::computeError): max of the squared point-to-epipolar-line distances in the two
 *     images, in double, stored as float; inlier iff err <= (float)(thr^2).
 *   - final refit: normalised 8-point least squares (smallest eigenvector of A^T A by cyclic Jacobi, rank 2
 *     enforced as F (I - v3 v3^T)) on the inliers of the best minimal model, kept when it has at least as many
 *     inliers at the same threshold. Minimal 7-point models of near-critical configurations (the reference's
 *     two-plane verifier scene) fit every point to ~1e-7 px^2, so the choice among them is arbitrary; the refit
 *     over all inliers recovers the unique F (the reference's known answer needs it).
 * Deterministic sampling: splitmix64 counter hash of (seed, pair id, hypothesis, attempt, draw), shared with the
 * HIP kernel. Compiled with -ffp-contract=off; the HIP kernel disables contraction for this code too.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define F_BATCH 64
#define F_ATTEMPTS 4
#define F_DRAWS 16
#define F_MAX_SOL 3

static uint64_t fm_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int collinear3(float ax, float ay, float bx, float by, float cx, float cy) {
    const float dx1 = bx - ax, dy1 = by - ay, dx2 = cx - ax, dy2 = cy - ay;
    return fabsf(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabsf(dx1) + fabsf(dy1) + fabsf(dx2) + fabsf(dy2));
}

/* pts: M x 4 float (x1, y1, x2, y2) pixels. 7 distinct, non-degenerate indices for hypothesis h; 0 on failure. */
int oracle_sample7(uint64_t seed, int pair, int h, int M, const float* pts, int* idx) {
    const uint64_t key = fm_mix(seed ^ fm_mix((uint64_t)(uint32_t)pair));
    for (int a = 0; a < F_ATTEMPTS; ++a) {
        int n = 0;
        for (int d = 0; d < F_DRAWS && n < 7; ++d) {
            const uint64_t r = fm_mix(key + ((uint64_t)h * F_ATTEMPTS + (uint64_t)a) * F_DRAWS + (uint64_t)d);
            const int v = (int)(((r >> 32) * (uint64_t)(uint32_t)M) >> 32);
            int dup = 0;
            for (int k = 0; k < n; ++k) dup |= (idx[k] == v);
            if (!dup) idx[n++] = v;
        }
        if (n < 7) continue;
        int bad = 0;
        for (int i = 0; i < 7 && !bad; ++i)
            for (int j = i + 1; j < 7 && !bad; ++j)
                for (int k = j + 1; k < 7 && !bad; ++k) {
                    const float* p = pts + 4 * idx[i];
                    const float* q = pts + 4 * idx[j];
                    const float* r = pts + 4 * idx[k];
                    bad = collinear3(p[0], p[1], q[0], q[1], r[0], r[1]) || collinear3(p[2], p[3], q[2], q[3], r[2], r[3]);
                }
        if (!bad) return 1;
    }
    return 0;
}

/* real roots of c0 l^3 + c1 l^2 + c2 l + c3 (ascending, distinct), by bisection on monotone pieces */
static double fm_cubic_eval(const double* a, double x) { return ((x + a[0]) * x + a[1]) * x + a[2]; }

static int fm_bisect(const double* a, double lo, double hi, double* root) {
    double flo = fm_cubic_eval(a, lo), fhi = fm_cubic_eval(a, hi);
    if (flo == 0.0) { *root = lo; return 1; }
    if (fhi == 0.0) { *root = hi; return 1; }
    if ((flo < 0.0) == (fhi < 0.0)) return 0;
    for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (!(mid > lo && mid < hi)) break;
        const double fm = fm_cubic_eval(a, mid);
        if (fm == 0.0) { lo = hi = mid; break; }
        if ((fm < 0.0) == (flo < 0.0)) { lo = mid; flo = fm; } else { hi = mid; }
    }
    *root = 0.5 * (lo + hi);
    return 1;
}

static int fm_solve_cubic(const double* c, double* r) {
    const double m = fmax(fmax(fabs(c[0]), fabs(c[1])), fmax(fabs(c[2]), fabs(c[3])));
    if (!(m > 0.0)) return 0;
    if (fabs(c[0]) <= 1e-12 * m) { /* quadratic c1 l^2 + c2 l + c3 */
        if (fabs(c[1]) <= 1e-12 * m) {
            if (fabs(c[2]) <= 1e-12 * m) return 0;
            r[0] = -c[3] / c[2];
            return 1;
        }
        const double d = c[2] * c[2] - 4.0 * c[1] * c[3];
        if (d < 0.0) return 0;
        const double s = sqrt(d);
        const double x1 = (-c[2] - s) / (2.0 * c[1]), x2 = (-c[2] + s) / (2.0 * c[1]);
        r[0] = fmin(x1, x2);
        r[1] = fmax(x1, x2);
        return r[1] > r[0] ? 2 : 1;
    }
    const double a[3] = {c[1] / c[0], c[2] / c[0], c[3] / c[0]}; /* monic l^3 + a0 l^2 + a1 l + a2 */
    const double B = 1.0 + fmax(fabs(a[0]), fmax(fabs(a[1]), fabs(a[2])));
    const double disc = a[0] * a[0] - 3.0 * a[1];
    int n = 0;
    if (disc <= 0.0) {
        n += fm_bisect(a, -B, B, r + n);
        return n;
    }
    const double sd = sqrt(disc);
    double k1 = (-a[0] - sd) / 3.0, k2 = (-a[0] + sd) / 3.0;
    k1 = fmin(fmax(k1, -B), B);
    k2 = fmin(fmax(k2, -B), B);
    const double edges[4] = {-B, k1, k2, B};
    for (int s = 0; s < 3; ++s) {
        double x;
        if (!(edges[s + 1] >= edges[s])) continue;
        if (fm_bisect(a, edges[s], edges[s + 1], &x)) {
            if (n == 0 || x > r[n - 1]) r[n++] = x;
        }
    }
    return n;
}

/* 7-point solver on the sample idx (pixel pts, M x 4 float). Up to 3 F (row-major, F33 = 1 when possible). */
int oracle_seven_point(const float* pts, const int* idx, double* Fs) {
    double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
    for (int k = 0; k < 7; ++k) {
        const float* p = pts + 4 * idx[k];
        c1x += p[0]; c1y += p[1]; c2x += p[2]; c2y += p[3];
    }
    c1x /= 7.0; c1y /= 7.0; c2x /= 7.0; c2y /= 7.0;
    double d1 = 0.0, d2 = 0.0;
    for (int k = 0; k < 7; ++k) {
        const float* p = pts + 4 * idx[k];
        const double ax = p[0] - c1x, ay = p[1] - c1y, bx = p[2] - c2x, by = p[3] - c2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return 0;
    const double s1 = 1.4142135623730951 * 7.0 / d1, s2 = 1.4142135623730951 * 7.0 / d2;
    double A[7][9];
    for (int k = 0; k < 7; ++k) {
        const float* p = pts + 4 * idx[k];
        const double u1 = (p[0] - c1x) * s1, v1 = (p[1] - c1y) * s1;
        const double u2 = (p[2] - c2x) * s2, v2 = (p[3] - c2y) * s2;
        A[k][0] = u2 * u1; A[k][1] = u2 * v1; A[k][2] = u2;
        A[k][3] = v2 * u1; A[k][4] = v2 * v1; A[k][5] = v2;
        A[k][6] = u1; A[k][7] = v1; A[k][8] = 1.0;
    }
    /* Gauss-Jordan on columns 0..6 with partial (row) pivoting; columns 7, 8 are free */
    for (int c = 0; c < 7; ++c) {
        int pr = c;
        double best = fabs(A[c][c]);
        for (int r = c + 1; r < 7; ++r)
            if (fabs(A[r][c]) > best) { best = fabs(A[r][c]); pr = r; }
        if (!(best > 1e-10)) return 0;
        if (pr != c)
            for (int j = 0; j < 9; ++j) { const double t = A[c][j]; A[c][j] = A[pr][j]; A[pr][j] = t; }
        const double inv = 1.0 / A[c][c];
        for (int j = 0; j < 9; ++j) A[c][j] = A[c][j] * inv;
        for (int r = 0; r < 7; ++r) {
            if (r == c) continue;
            const double f = A[r][c];
            for (int j = 0; j < 9; ++j) A[r][j] = A[r][j] - f * A[c][j];
        }
    }
    double f1[9], f2[9];
    for (int r = 0; r < 7; ++r) { f1[r] = -A[r][7]; f2[r] = -A[r][8]; }
    f1[7] = 1.0; f1[8] = 0.0;
    f2[7] = 0.0; f2[8] = 1.0;
    for (int i = 0; i < 9; ++i) f1[i] = f1[i] - f2[i];
    /* det(l f1 + f2) = c0 l^3 + c1 l^2 + c2 l + c3 (run7Point's expansion) */
    double c[4];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    double roots[3];
    const int nr = fm_solve_cubic(c, roots);
    int ns = 0;
    for (int k = 0; k < nr; ++k) {
        double Fn[9], F[9];
        for (int i = 0; i < 9; ++i) Fn[i] = roots[k] * f1[i] + f2[i];
        /* F = T2^T Fn T1, T = [[s, 0, -s cx], [0, s, -s cy], [0, 0, 1]] */
        const double T1[9] = {s1, 0.0, -s1 * c1x, 0.0, s1, -s1 * c1y, 0.0, 0.0, 1.0};
        const double T2[9] = {s2, 0.0, -s2 * c2x, 0.0, s2, -s2 * c2y, 0.0, 0.0, 1.0};
        double G[9];
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc)
                G[3 * r + cc] = Fn[3 * r + 0] * T1[0 * 3 + cc] + Fn[3 * r + 1] * T1[1 * 3 + cc] + Fn[3 * r + 2] * T1[2 * 3 + cc];
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc)
                F[3 * r + cc] = T2[0 * 3 + r] * G[0 * 3 + cc] + T2[1 * 3 + r] * G[1 * 3 + cc] + T2[2 * 3 + r] * G[2 * 3 + cc];
        if (fabs(F[8]) > DBL_EPSILON) {
            const double inv = 1.0 / F[8];
            for (int i = 0; i < 8; ++i) F[i] = F[i] * inv;
            F[8] = 1.0;
        }
        memcpy(Fs + 9 * ns, F, sizeof(F));
        ++ns;
    }
    return ns;
}

/* FMEstimatorCallback::computeError for one correspondence */
float oracle_f_error(const double* F, const float* p) {
    const double x1 = p[0], y1 = p[1], x2 = p[2], y2 = p[3];
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1.0 / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1.0 / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    return (float)fmax(d1 * d1 * s1, d2 * d2 * s2);
}

static int fm_count(const double* F, const float* pts, int M, float thr2, uint8_t* mask) {
    int c = 0;
    for (int i = 0; i < M; ++i) {
        const int in = oracle_f_error(F, pts + 4 * i) <= thr2;
        if (mask) mask[i] = (uint8_t)in;
        c += in;
    }
    return c;
}

static int fm_update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmax(p, 0.0); p = fmin(p, 1.0);
    ep = fmax(ep, 0.0); ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - pow(1.0 - ep, (double)model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)lround(num / denom);
}

/* cyclic Jacobi on a symmetric n x n matrix (row-major, destroyed): eigenvalues w, eigenvectors in columns of V */
static void fm_jacobi(double* a, int n, double* w, double* V) {
    for (int i = 0; i < n * n; ++i) V[i] = 0.0;
    for (int i = 0; i < n; ++i) V[i * n + i] = 1.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
        if (!(off > 1e-300)) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                const double theta = (a[q * n + q] - a[p * n + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = c * akp - sn * akq;
                    a[k * n + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = a[p * n + k], aqk = a[q * n + k];
                    a[p * n + k] = c * apk - sn * aqk;
                    a[q * n + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - sn * vkq;
                    V[k * n + q] = sn * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

/* normalised 8-point on the masked correspondences (>= 8), rank 2, F33 = 1 when possible. 0 on failure. */
int oracle_eight_point(const float* pts, const uint8_t* mask, int M, double* F_out) {
    int n = 0;
    double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float* p = pts + 4 * i;
        c1x += p[0]; c1y += p[1]; c2x += p[2]; c2y += p[3];
        ++n;
    }
    if (n < 8) return 0;
    c1x /= n; c1y /= n; c2x /= n; c2y /= n;
    double d1 = 0.0, d2 = 0.0;
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float* p = pts + 4 * i;
        const double ax = p[0] - c1x, ay = p[1] - c1y, bx = p[2] - c2x, by = p[3] - c2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return 0;
    const double s1 = 1.4142135623730951 * n / d1, s2 = 1.4142135623730951 * n / d2;
    double AtA[81];
    memset(AtA, 0, sizeof(AtA));
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float* p = pts + 4 * i;
        const double u1 = (p[0] - c1x) * s1, v1 = (p[1] - c1y) * s1;
        const double u2 = (p[2] - c2x) * s2, v2 = (p[3] - c2y) * s2;
        const double r[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        for (int a = 0; a < 9; ++a)
            for (int b = a; b < 9; ++b) AtA[a * 9 + b] = AtA[a * 9 + b] + r[a] * r[b];
    }
    for (int a = 0; a < 9; ++a)
        for (int b = 0; b < a; ++b) AtA[a * 9 + b] = AtA[b * 9 + a];
    double w[9], V[81];
    fm_jacobi(AtA, 9, w, V);
    int kmin = 0;
    for (int k = 1; k < 9; ++k)
        if (w[k] < w[kmin]) kmin = k;
    double Fn[9];
    for (int e = 0; e < 9; ++e) Fn[e] = V[e * 9 + kmin];
    /* rank 2: Fn (I - v v^T), v = eigenvector of Fn^T Fn with the smallest eigenvalue */
    double FtF[9], w3[3], V3[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            FtF[a * 3 + b] = Fn[0 * 3 + a] * Fn[0 * 3 + b] + Fn[1 * 3 + a] * Fn[1 * 3 + b] + Fn[2 * 3 + a] * Fn[2 * 3 + b];
    fm_jacobi(FtF, 3, w3, V3);
    int k3 = 0;
    for (int k = 1; k < 3; ++k)
        if (w3[k] < w3[k3]) k3 = k;
    const double v[3] = {V3[0 * 3 + k3], V3[1 * 3 + k3], V3[2 * 3 + k3]};
    for (int r = 0; r < 3; ++r) {
        const double fv = Fn[3 * r] * v[0] + Fn[3 * r + 1] * v[1] + Fn[3 * r + 2] * v[2];
        for (int c = 0; c < 3; ++c) Fn[3 * r + c] = Fn[3 * r + c] - fv * v[c];
    }
    const double T1[9] = {s1, 0.0, -s1 * c1x, 0.0, s1, -s1 * c1y, 0.0, 0.0, 1.0};
    const double T2[9] = {s2, 0.0, -s2 * c2x, 0.0, s2, -s2 * c2y, 0.0, 0.0, 1.0};
    double G[9], F[9];
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc)
            G[3 * r + cc] = Fn[3 * r + 0] * T1[0 * 3 + cc] + Fn[3 * r + 1] * T1[1 * 3 + cc] + Fn[3 * r + 2] * T1[2 * 3 + cc];
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc)
            F[3 * r + cc] = T2[0 * 3 + r] * G[0 * 3 + cc] + T2[1 * 3 + r] * G[1 * 3 + cc] + T2[2 * 3 + r] * G[2 * 3 + cc];
    if (fabs(F[8]) > DBL_EPSILON) {
        const double inv = 1.0 / F[8];
        for (int i = 0; i < 8; ++i) F[i] = F[i] * inv;
        F[8] = 1.0;
    }
    memcpy(F_out, F, sizeof(F));
    return 1;
}

static int cmp_float(const void* a, const void* b) {
    const float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

/*
 * Estimates F from M pixel correspondences (x1, x2: M x 2 float32) with threshold thr_px.
 * Outputs F (9, row-major) and the inlier mask. Returns the inlier count, -1 when no model (or M < 8).
 * *n_hyp receives the number of hypotheses drawn (whole batches of 64).
 */
int oracle_ransac_F(const float* x1, const float* x2, int M, double thr_px, double prob, int max_iters, uint64_t seed,
                    int pair_id, double* F_out, uint8_t* mask_out, int* n_hyp) {
    if (n_hyp) *n_hyp = 0;
    if (M < 8) return -1;
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)M);
    float* err = (float*)malloc(sizeof(float) * (size_t)M);
    for (int i = 0; i < M; ++i) {
        pts[4 * i] = x1[2 * i];
        pts[4 * i + 1] = x1[2 * i + 1];
        pts[4 * i + 2] = x2[2 * i];
        pts[4 * i + 3] = x2[2 * i + 1];
    }
    const int lmeds = M < 15;
    int niters = lmeds ? fm_update_num_iters(prob, 0.45, 7, max_iters) : max_iters;
    if (niters < 1) niters = 1;
    int done = 0, best = -1, have = 0;
    float min_median = FLT_MAX;
    double bestF[9];
    while (done < niters) {
        for (int h = done; h < done + F_BATCH; ++h) {
            int idx[7];
            if (!oracle_sample7(seed, pair_id, h, M, pts, idx)) continue;
            double Fs[9 * F_MAX_SOL];
            const int ns = oracle_seven_point(pts, idx, Fs);
            for (int s = 0; s < ns; ++s) {
                const double* F = Fs + 9 * s;
                if (lmeds) {
                    for (int i = 0; i < M; ++i) err[i] = oracle_f_error(F, pts + 4 * i);
                    qsort(err, (size_t)M, sizeof(float), cmp_float);
                    const float med = err[M / 2];
                    if (med < min_median) {
                        min_median = med;
                        memcpy(bestF, F, sizeof(bestF));
                        have = 1;
                    }
                } else {
                    const int c = fm_count(F, pts, M, (float)(thr_px * thr_px), NULL);
                    if (c > (best > 6 ? best : 6)) {
                        best = c;
                        memcpy(bestF, F, sizeof(bestF));
                        have = 1;
                    }
                }
            }
        }
        done += F_BATCH;
        if (!lmeds && best > 0) {
            const int upd = fm_update_num_iters(prob, (double)(M - best) / M, 7, niters);
            if (upd < niters) niters = upd;
        }
    }
    if (n_hyp) *n_hyp = done;
    int cnt = -1;
    if (have) {
        double th = thr_px;
        if (lmeds) {
            th = 2.5 * 1.4826 * (1.0 + 5.0 / (M - 7)) * sqrt((double)min_median);
            if (th < 0.001) th = 0.001;
        }
        const float th2 = (float)(th * th);
        cnt = fm_count(bestF, pts, M, th2, mask_out);
        double Fr[9];
        if (cnt >= 8 && oracle_eight_point(pts, mask_out, M, Fr)) {
            const int cr = fm_count(Fr, pts, M, th2, NULL);
            if (cr >= cnt) {
                memcpy(bestF, Fr, sizeof(bestF));
                cnt = fm_count(bestF, pts, M, th2, mask_out);
            }
        }
        if (lmeds && cnt < 7) cnt = -1;
        memcpy(F_out, bestF, sizeof(bestF));
    }
    free(pts);
    free(err);
    return cnt;
}
