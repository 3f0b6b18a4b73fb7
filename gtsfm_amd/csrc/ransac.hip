// Batched essential-matrix verifier: 5-point RANSAC + iterative LO + recoverPose, one wavefront per image pair.
//
// Replaces, per pair (file:line in the reference):
//   gtsfm/frontend/verifier/opencv_verifier_base.py:45-109  verify(): M<5/M<6 failure, K-normalisation of the
//       putatives (utils/features.py:40-50), fx = max(fx1, fx2), threshold px/fx, inlier mask, inlier ratio
//   gtsfm/frontend/verifier/ransac.py:52-82  cv2.findEssentialMat(USAC_ACCURATE, prob 0.999999, maxIters 1000)
//   gtsfm/utils/verification.py:52-94  cv.recoverPose(E, x1n, x2n) on the verified correspondences
// The algorithm is the one restated in oracle/ransac.c (same sampling hash, same solver steps, same fp32 fmaf
// inlier test, same batch-wise termination, same LO and cheirality vote).
//
// Work mapping (wave64, gfx950):
//   * hypotheses are drawn in batches of 64: lane l solves hypothesis (batch*64 + l) with Nister's 5-point
//     solver in fp64 (private arrays; the 10x20 elimination lives in scratch);
//   * every candidate E of the batch is then scored by the whole wave, lanes striding over the putatives
//     (fp32 Sampson test, ballot+popcount), with an exact early exit once a candidate can no longer beat the
//     best count;
//   * after the loop one lane re-solves the winning hypothesis in fp64, the wave runs the LO refits (the 9x9
//     normal matrix is reduced through LDS in a fixed order) and the cheirality vote of recoverPose.
#include <math.h>

#include "common.hpp"

namespace {

constexpr int kBatch = 64;
constexpr int kMaxSol = 10;
constexpr int kLoSteps = 4;
constexpr int kLoIrls = 3;
constexpr double kLoMult = 6.0;

// ------------------------------------------------------------------ sampling (identical to the oracle)
__device__ __forceinline__ uint64_t sm_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ bool sample5(uint64_t seed, int pair, int h, int M, int* idx) {
    const uint64_t key = sm_mix(seed ^ sm_mix((uint64_t)(uint32_t)pair));
    int n = 0;
    for (int d = 0; d < 32 && n < 5; ++d) {
        const uint64_t r = sm_mix(key + (uint64_t)h * 32u + (uint64_t)d);
        const int v = (int)(((r >> 32) * (uint64_t)(uint32_t)M) >> 32);
        bool dup = false;
        for (int k = 0; k < n; ++k) dup |= (idx[k] == v);
        if (!dup) idx[n++] = v;
    }
    return n == 5;
}

// ------------------------------------------------------------------ polynomial algebra tables
// linear [x y z 1] x linear -> quadratic [xx yy xy xz yz zz x y z 1]
__constant__ int8_t kLL2Q[4][4] = {{0, 2, 3, 6}, {2, 1, 4, 7}, {3, 4, 5, 8}, {6, 7, 8, 9}};
// quadratic x linear -> cubic (Nister order)
// [xxx yyy xxy xyy xxz xx yyz yy xyz xy xzz xz x yzz yz y zzz zz z 1]
__constant__ int8_t kQL2C[10][4] = {{0, 2, 4, 5},     {3, 1, 6, 7},     {2, 3, 8, 9},     {4, 8, 10, 11},
                                    {8, 6, 13, 14},   {10, 13, 16, 17}, {5, 9, 11, 12},   {9, 7, 14, 15},
                                    {11, 14, 17, 18}, {12, 15, 18, 19}};

__device__ __forceinline__ void mul_ll(const double* a, const double* b, double* q) {
#pragma unroll
    for (int i = 0; i < 10; ++i) q[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) q[kLL2Q[i][j]] += a[i] * b[j];
}

__device__ __forceinline__ void addmul_ql(const double* q, const double* l, double s, double* c) {
#pragma unroll
    for (int i = 0; i < 10; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[kQL2C[i][j]] += s * (q[i] * l[j]);
}

__device__ __forceinline__ double peval(const double* p, int deg, double x) {
    double v = p[deg];
    for (int i = deg - 1; i >= 0; --i) v = v * x + p[i];
    return v;
}

__device__ int prem(const double* a, int da, const double* b, int db, double* r) {
    double t[11];
    for (int i = 0; i <= da; ++i) t[i] = a[i];
    for (int k = da; k >= db; --k) {
        const double f = t[k] / b[db];
        for (int i = 0; i <= db; ++i) t[k - db + i] -= f * b[i];
        t[k] = 0.0;
    }
    int dr = db - 1;
    double scale = 0.0;
    for (int i = 0; i <= da; ++i) scale = fmax(scale, fabs(a[i]));
    while (dr >= 0 && fabs(t[dr]) <= 1e-14 * scale) --dr;
    for (int i = 0; i <= dr; ++i) r[i] = t[i];
    return dr;
}

struct Sturm {
    double p[11][11];
    int deg[11];
    int n;
};

__device__ int sign_changes(const Sturm& s, double x) {
    int c = 0;
    double prev = 0.0;
    for (int k = 0; k < s.n; ++k) {
        const double v = peval(s.p[k], s.deg[k], x);
        if (v == 0.0) continue;
        if (prev != 0.0 && ((v < 0.0) != (prev < 0.0))) ++c;
        prev = v;
    }
    return c;
}

// Real roots (ascending) of a degree <= 10 polynomial: Sturm isolation + bisection.
__device__ int real_roots(const double* pin, int deg, double* roots) {
    double p[11];
    while (deg > 0 && fabs(pin[deg]) <= 1e-300) --deg;
    if (deg <= 0) return 0;
    for (int i = 0; i <= deg; ++i) p[i] = pin[i] / pin[deg];
    Sturm s;
    for (int i = 0; i <= deg; ++i) s.p[0][i] = p[i];
    s.deg[0] = deg;
    for (int i = 1; i <= deg; ++i) s.p[1][i - 1] = (double)i * p[i];
    s.deg[1] = deg - 1;
    s.n = 2;
    while (s.n < 11 && s.deg[s.n - 1] > 0) {
        double r[11];
        const int dr = prem(s.p[s.n - 2], s.deg[s.n - 2], s.p[s.n - 1], s.deg[s.n - 1], r);
        if (dr < 0) break;
        for (int i = 0; i <= dr; ++i) s.p[s.n][i] = -r[i];
        s.deg[s.n] = dr;
        s.n++;
    }
    double bound = 0.0;
    for (int i = 0; i < deg; ++i) bound = fmax(bound, fabs(p[i]));
    bound += 1.0;
    double st_a[48], st_b[48];
    int st_va[48], st_vb[48];
    int ns = 1, nr = 0, guard = 0;
    st_a[0] = -bound;
    st_b[0] = bound;
    st_va[0] = sign_changes(s, -bound);
    st_vb[0] = sign_changes(s, bound);
    while (ns > 0 && nr < kMaxSol && guard < 2000) {
        ++guard;
        --ns;
        const double a = st_a[ns], b = st_b[ns];
        const int va = st_va[ns], vb = st_vb[ns];
        const int cnt = va - vb;
        if (cnt <= 0) continue;
        if (cnt == 1 || b - a < 1e-10 * fmax(1.0, fabs(a))) {
            double lo = a, hi = b;
            double flo = peval(p, deg, lo);
            for (int it = 0; it < 80; ++it) {
                const double mid = 0.5 * (lo + hi);
                const double fm = peval(p, deg, mid);
                if ((fm < 0.0) == (flo < 0.0) && fm != 0.0) {
                    lo = mid;
                    flo = fm;
                } else {
                    hi = mid;
                }
            }
            roots[nr++] = 0.5 * (lo + hi);
            continue;
        }
        const double mid = 0.5 * (a + b);
        const int vm = sign_changes(s, mid);
        if (ns + 2 <= 48) {
            st_a[ns] = mid; st_b[ns] = b; st_va[ns] = vm; st_vb[ns] = vb; ++ns;
            st_a[ns] = a; st_b[ns] = mid; st_va[ns] = va; st_vb[ns] = vm; ++ns;
        }
    }
    return nr;
}

// ------------------------------------------------------------------ Nister 5-point (one lane)
__device__ bool nullspace_5x9(double q[5][9], double N[4][9]) {
    int col[9];
    for (int j = 0; j < 9; ++j) col[j] = j;
    for (int r = 0; r < 5; ++r) {
        int pr = r, pc = r;
        double best = -1.0;
        for (int i = r; i < 5; ++i)
            for (int j = r; j < 9; ++j)
                if (fabs(q[i][j]) > best) { best = fabs(q[i][j]); pr = i; pc = j; }
        if (best < 1e-12) return false;
        if (pr != r)
            for (int j = 0; j < 9; ++j) { const double t = q[r][j]; q[r][j] = q[pr][j]; q[pr][j] = t; }
        if (pc != r) {
            for (int i = 0; i < 5; ++i) { const double t = q[i][r]; q[i][r] = q[i][pc]; q[i][pc] = t; }
            const int t = col[r]; col[r] = col[pc]; col[pc] = t;
        }
        const double inv = 1.0 / q[r][r];
        for (int j = 0; j < 9; ++j) q[r][j] *= inv;
        for (int i = 0; i < 5; ++i) {
            if (i == r) continue;
            const double f = q[i][r];
            for (int j = 0; j < 9; ++j) q[i][j] -= f * q[r][j];
        }
    }
    for (int k = 0; k < 4; ++k) {
        double v[9];
        for (int j = 0; j < 9; ++j) v[j] = 0.0;
        v[col[5 + k]] = 1.0;
        for (int r = 0; r < 5; ++r) v[col[r]] = -q[r][5 + k];
        double nrm = 0.0;
        for (int j = 0; j < 9; ++j) nrm += v[j] * v[j];
        nrm = sqrt(nrm);
        for (int j = 0; j < 9; ++j) N[k][j] = v[j] / nrm;
    }
    return true;
}

// 5 correspondences (x1[i], x2[i]) -> up to 10 unit-norm E (row-major). Returns the count.
__device__ int five_point(const double* x1, const double* x2, double* Es) {
    double Q[5][9];
    for (int i = 0; i < 5; ++i) {
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        Q[i][0] = u2 * u1; Q[i][1] = u2 * v1; Q[i][2] = u2;
        Q[i][3] = v2 * u1; Q[i][4] = v2 * v1; Q[i][5] = v2;
        Q[i][6] = u1; Q[i][7] = v1; Q[i][8] = 1.0;
    }
    double N[4][9];
    if (!nullspace_5x9(Q, N)) return 0;
    double E[9][4];
    for (int e = 0; e < 9; ++e) {
        E[e][0] = N[0][e];
        E[e][1] = N[1][e];
        E[e][2] = N[2][e];
        E[e][3] = N[3][e];
    }
    double A[10][20];
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) A[r][c] = 0.0;
    {
        double q[10];
        mul_ll(E[4], E[8], q); addmul_ql(q, E[0], 1.0, A[0]);
        mul_ll(E[5], E[7], q); addmul_ql(q, E[0], -1.0, A[0]);
        mul_ll(E[3], E[8], q); addmul_ql(q, E[1], -1.0, A[0]);
        mul_ll(E[5], E[6], q); addmul_ql(q, E[1], 1.0, A[0]);
        mul_ll(E[3], E[7], q); addmul_ql(q, E[2], 1.0, A[0]);
        mul_ll(E[4], E[6], q); addmul_ql(q, E[2], -1.0, A[0]);
    }
    double EEt[3][3][10], tr[10], tmp[10];
    for (int i = 0; i < 3; ++i)
        for (int j = i; j < 3; ++j) {
            for (int m = 0; m < 10; ++m) EEt[i][j][m] = 0.0;
            for (int k = 0; k < 3; ++k) {
                mul_ll(E[3 * i + k], E[3 * j + k], tmp);
                for (int m = 0; m < 10; ++m) EEt[i][j][m] += tmp[m];
            }
            if (j != i)
                for (int m = 0; m < 10; ++m) EEt[j][i][m] = EEt[i][j][m];
        }
    for (int m = 0; m < 10; ++m) tr[m] = EEt[0][0][m] + EEt[1][1][m] + EEt[2][2][m];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double* row = A[1 + 3 * i + j];
            for (int k = 0; k < 3; ++k) addmul_ql(EEt[i][k], E[3 * k + j], 2.0, row);
            addmul_ql(tr, E[3 * i + j], -1.0, row);
        }
    for (int c = 0; c < 10; ++c) {
        int pr = c;
        double best = fabs(A[c][c]);
        for (int r = c + 1; r < 10; ++r)
            if (fabs(A[r][c]) > best) { best = fabs(A[r][c]); pr = r; }
        if (best < 1e-14) return 0;
        if (pr != c)
            for (int j = 0; j < 20; ++j) { const double t = A[c][j]; A[c][j] = A[pr][j]; A[pr][j] = t; }
        const double inv = 1.0 / A[c][c];
        for (int j = 0; j < 20; ++j) A[c][j] *= inv;
        for (int r = 0; r < 10; ++r) {
            if (r == c) continue;
            const double f = A[r][c];
            for (int j = 0; j < 20; ++j) A[r][j] -= f * A[c][j];
        }
    }
    double B[3][3][5];
    for (int r = 0; r < 3; ++r) {
        const double* e = A[4 + 2 * r];
        const double* f = A[5 + 2 * r];
        B[r][0][0] = e[12]; B[r][0][1] = e[11] - f[12]; B[r][0][2] = e[10] - f[11]; B[r][0][3] = -f[10]; B[r][0][4] = 0.0;
        B[r][1][0] = e[15]; B[r][1][1] = e[14] - f[15]; B[r][1][2] = e[13] - f[14]; B[r][1][3] = -f[13]; B[r][1][4] = 0.0;
        B[r][2][0] = e[19]; B[r][2][1] = e[18] - f[19]; B[r][2][2] = e[17] - f[18]; B[r][2][3] = e[16] - f[17];
        B[r][2][4] = -f[16];
    }
    double n[11];
    for (int i = 0; i < 11; ++i) n[i] = 0.0;
    {
        const int deg[3] = {3, 3, 4};
        for (int c = 0; c < 3; ++c) {
            const int c1 = (c + 1) % 3, c2 = (c + 2) % 3;
            double m[9];
            for (int i = 0; i < 9; ++i) m[i] = 0.0;
            for (int i = 0; i <= deg[c1]; ++i)
                for (int j = 0; j <= deg[c2]; ++j) m[i + j] += B[1][c1][i] * B[2][c2][j];
            for (int i = 0; i <= deg[c2]; ++i)
                for (int j = 0; j <= deg[c1]; ++j) m[i + j] -= B[1][c2][i] * B[2][c1][j];
            const int dm = deg[c1] + deg[c2];
            for (int i = 0; i <= deg[c]; ++i)
                for (int j = 0; j <= dm; ++j) n[i + j] += B[0][c][i] * m[j];
        }
    }
    double roots[kMaxSol];
    const int nroots = real_roots(n, 10, roots);
    int nsol = 0;
    for (int k = 0; k < nroots; ++k) {
        const double z = roots[k];
        double Bz[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Bz[r][c] = peval(B[r][c], c == 2 ? 4 : 3, z);
        double bx = 0, by = 0, bzz = 0, bn = -1.0;
        for (int a = 0; a < 3; ++a) {
            const int b = (a + 1) % 3;
            const double cx = Bz[a][1] * Bz[b][2] - Bz[a][2] * Bz[b][1];
            const double cy = Bz[a][2] * Bz[b][0] - Bz[a][0] * Bz[b][2];
            const double cz = Bz[a][0] * Bz[b][1] - Bz[a][1] * Bz[b][0];
            const double nn = cx * cx + cy * cy + cz * cz;
            if (nn > bn) { bn = nn; bx = cx; by = cy; bzz = cz; }
        }
        if (!(fabs(bzz) > 1e-300)) continue;
        const double x = bx / bzz, y = by / bzz;
        double* Eo = Es + 9 * nsol;
        double nrm = 0.0;
        for (int e = 0; e < 9; ++e) {
            Eo[e] = x * N[0][e] + y * N[1][e] + z * N[2][e] + N[3][e];
            nrm += Eo[e] * Eo[e];
        }
        nrm = sqrt(nrm);
        if (!(nrm > 0.0)) continue;
        for (int e = 0; e < 9; ++e) Eo[e] /= nrm;
        ++nsol;
    }
    return nsol;
}

// ------------------------------------------------------------------ scoring
__device__ __forceinline__ bool sampson_inlier(const float* E, float4 p, float thr2) {
    const float a0 = fmaf(E[1], p.y, fmaf(E[0], p.x, E[2]));
    const float a1 = fmaf(E[4], p.y, fmaf(E[3], p.x, E[5]));
    const float a2 = fmaf(E[7], p.y, fmaf(E[6], p.x, E[8]));
    const float b0 = fmaf(E[3], p.w, fmaf(E[0], p.z, E[6]));
    const float b1 = fmaf(E[4], p.w, fmaf(E[1], p.z, E[7]));
    const float num = fmaf(p.w, a1, fmaf(p.z, a0, a2));
    const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, __fmul_rn(a0, a0))));
    return __fmul_rn(num, num) <= __fmul_rn(thr2, den);
}

// Wave-wide inlier count of E over M points; stops early (exactly) once count + remaining <= floor.
__device__ int wave_count(const float* E, const float4* pts, int M, float thr2, int floor_count, int lane) {
    int c = 0;
    for (int base = 0; base < M; base += 64) {
        const int i = base + lane;
        bool in = false;
        if (i < M) in = sampson_inlier(E, pts[i], thr2);
        c += __popcll(__ballot(in));
        const int remaining = M - (base + 64);
        if (remaining > 0 && c + remaining <= floor_count) return -1;
    }
    return c;
}

// ------------------------------------------------------------------ small dense linear algebra (one lane / redundant)
__device__ void jacobi_eig(double* a, int n, double* w, double* V) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
        if (off < 1e-30) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                const double app = a[p * n + p], aqq = a[q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = c * akp - s * akq;
                    a[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = a[p * n + k], aqk = a[q * n + k];
                    a[p * n + k] = c * apk - s * aqk;
                    a[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

__device__ void svd3(const double* E, double* U, double* s, double* V) {
    double ata[9], w[3], Vt[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 3; ++k) acc += E[k * 3 + i] * E[k * 3 + j];
            ata[i * 3 + j] = acc;
        }
    jacobi_eig(ata, 3, w, Vt);
    int order[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (w[order[j]] > w[order[i]]) { const int t = order[i]; order[i] = order[j]; order[j] = t; }
    for (int c = 0; c < 3; ++c) {
        s[c] = sqrt(fmax(w[order[c]], 0.0));
        for (int r = 0; r < 3; ++r) V[r * 3 + c] = Vt[r * 3 + order[c]];
    }
    for (int c = 0; c < 2; ++c) {
        double u[3], nrm = 0.0;
        for (int r = 0; r < 3; ++r) {
            u[r] = E[r * 3 + 0] * V[0 * 3 + c] + E[r * 3 + 1] * V[1 * 3 + c] + E[r * 3 + 2] * V[2 * 3 + c];
            nrm += u[r] * u[r];
        }
        nrm = sqrt(nrm);
        for (int r = 0; r < 3; ++r) U[r * 3 + c] = nrm > 0 ? u[r] / nrm : (r == c ? 1.0 : 0.0);
    }
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
    const double v0 = V[3] * V[7] - V[6] * V[4], v1 = V[6] * V[1] - V[0] * V[7], v2 = V[0] * V[4] - V[3] * V[1];
    V[2] = v0;
    V[5] = v1;
    V[8] = v2;
}

__device__ __forceinline__ double sampson_sq(const double* E, double2 p1, double2 p2, double* den_out) {
    const double a0 = E[0] * p1.x + E[1] * p1.y + E[2];
    const double a1 = E[3] * p1.x + E[4] * p1.y + E[5];
    const double a2 = E[6] * p1.x + E[7] * p1.y + E[8];
    const double b0 = E[0] * p2.x + E[3] * p2.y + E[6];
    const double b1 = E[1] * p2.x + E[4] * p2.y + E[7];
    const double num = p2.x * a0 + p2.y * a1 + a2;
    const double den = a0 * a0 + a1 * a1 + b0 * b0 + b1 * b1;
    *den_out = den;
    return den > 0.0 ? num * num / den : 1e300;
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __shfl_xor((int)(u & 0xFFFFFFFFull), m), hi = __shfl_xor((int)(u >> 32), m);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Wave-cooperative Sampson-weighted 8-point refit (see oracle refit_essential). The 45 unique normal-matrix
// entries are summed per lane, then butterfly-reduced across the wave (fixed order: deterministic).
__device__ bool wave_refit(const double2* x1, const double2* x2, int M, const double* Esel, double th2,
                           const double* Ew, double* Eout, int lane) {
    double acc[45];
#pragma unroll
    for (int k = 0; k < 45; ++k) acc[k] = 0.0;
    int n = 0;
    for (int i = lane; i < M; i += 64) {
        double den;
        if (sampson_sq(Esel, x1[i], x2[i], &den) > th2) continue;
        double dw;
        sampson_sq(Ew, x1[i], x2[i], &dw);
        const double w2 = dw > 1e-300 ? 1.0 / dw : 0.0;
        const double u1 = x1[i].x, v1 = x1[i].y, u2 = x2[i].x, v2 = x2[i].y;
        const double r[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        int k = 0;
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
            for (int b = a; b < 9; ++b) acc[k++] += w2 * r[a] * r[b];
        ++n;
    }
    for (int m = 32; m >= 1; m >>= 1) n += __shfl_xor(n, m);
    if (n < 8) return false;
#pragma unroll
    for (int k = 0; k < 45; ++k)
        for (int m = 1; m < 64; m <<= 1) acc[k] += shfl_xor_d(acc[k], m);
    double ata[81];
    {
        int k = 0;
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
            for (int b = a; b < 9; ++b) {
                ata[a * 9 + b] = acc[k];
                ata[b * 9 + a] = acc[k];
                ++k;
            }
    }
    double w[9], V[81];
    jacobi_eig(ata, 9, w, V);
    int imin = 0;
    for (int i = 1; i < 9; ++i)
        if (w[i] < w[imin]) imin = i;
    double E[9];
    for (int k = 0; k < 9; ++k) E[k] = V[k * 9 + imin];
    double U[9], s[3], Vv[9];
    svd3(E, U, s, Vv);
    double nrm = 0.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            Eout[r * 3 + c] = U[r * 3 + 0] * Vv[c * 3 + 0] + U[r * 3 + 1] * Vv[c * 3 + 1];
            nrm += Eout[r * 3 + c] * Eout[r * 3 + c];
        }
    nrm = sqrt(nrm);
    for (int k = 0; k < 9; ++k) Eout[k] /= nrm;
    return true;
}

__device__ __forceinline__ double det3(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

__device__ int wave_cheirality(const double* R, const double* t, const double2* x1, const double2* x2,
                               const uint8_t* mask, int M, int lane) {
    int good = 0;
    for (int i = lane; i < M; i += 64) {
        if (!mask[i]) continue;
        const double p0 = x1[i].x, p1 = x1[i].y, q0 = x2[i].x, q1 = x2[i].y;
        const double a0 = R[0] * p0 + R[1] * p1 + R[2];
        const double a1 = R[3] * p0 + R[4] * p1 + R[5];
        const double a2 = R[6] * p0 + R[7] * p1 + R[8];
        const double aa = a0 * a0 + a1 * a1 + a2 * a2;
        const double aq = a0 * q0 + a1 * q1 + a2;
        const double qq = q0 * q0 + q1 * q1 + 1.0;
        const double at = a0 * t[0] + a1 * t[1] + a2 * t[2];
        const double qt = q0 * t[0] + q1 * t[1] + t[2];
        const double det = aa * qq - aq * aq;
        if (fabs(det) < 1e-18) continue;
        const double l1 = (-at * qq + aq * qt) / det;
        const double z2 = l1 * a2 + t[2];
        good += (l1 > 0.0 && l1 < 50.0 && z2 > 0.0 && z2 < 50.0) ? 1 : 0;
    }
    for (int m = 32; m >= 1; m >>= 1) good += __shfl_xor(good, m);
    return good;
}

__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmax(p, 0.0); p = fmin(p, 1.0);
    ep = fmax(ep, 0.0); ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - pow(1.0 - ep, (double)model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)llround(num / denom);
}

// ------------------------------------------------------------------ kernels
// Gather + normalise the putatives of every pair: x = (uv - (u0, v0)) / f per image (utils/features.py:40-50).
__global__ void normalize_putatives_kernel(const float* __restrict__ kp_xy, const double* __restrict__ intr, int kmax,
                                           const int* __restrict__ pairs, const uint32_t* __restrict__ match_idx,
                                           const int* __restrict__ match_count, int mcap,
                                           double2* __restrict__ x1n, double2* __restrict__ x2n,
                                           float4* __restrict__ pts) {
    const int p = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int M = match_count[p];
    if (i >= M) return;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const uint32_t a = match_idx[((size_t)p * mcap + i) * 2], b = match_idx[((size_t)p * mcap + i) * 2 + 1];
    const double f1 = intr[3 * i1], u1 = intr[3 * i1 + 1], v1 = intr[3 * i1 + 2];
    const double f2 = intr[3 * i2], u2 = intr[3 * i2 + 1], v2 = intr[3 * i2 + 2];
    const float* k1 = kp_xy + ((size_t)i1 * kmax + a) * 2;
    const float* k2 = kp_xy + ((size_t)i2 * kmax + b) * 2;
    const double2 n1 = make_double2(((double)k1[0] - u1) / f1, ((double)k1[1] - v1) / f1);
    const double2 n2 = make_double2(((double)k2[0] - u2) / f2, ((double)k2[1] - v2) / f2);
    const size_t o = (size_t)p * mcap + i;
    x1n[o] = n1;
    x2n[o] = n2;
    pts[o] = make_float4((float)n1.x, (float)n1.y, (float)n2.x, (float)n2.y);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

struct RansacOutputs {
    double* E;       // [P][9]
    double* R;       // [P][9]
    double* t;       // [P][3]
    int* n_inliers;  // [P]
    int* status;     // [P]: 0 ok, 1 too few putatives (M < 6), 2 no model
    int* n_hyp;      // [P] (may be null)
    uint8_t* mask;   // [P][mcap]
};

__global__ __launch_bounds__(64) void ransac_hypotheses_kernel(const int* __restrict__ pairs, const double* __restrict__ intr,
                                                      const int* __restrict__ match_count, int mcap,
                                                      const double2* __restrict__ x1n_all,
                                                      const double2* __restrict__ x2n_all,
                                                      const float4* __restrict__ pts_all, double thr_px, double prob,
                                                      int max_iters, uint64_t seed, int pair_id_base,
                                                      RansacOutputs out, int4* __restrict__ best_out) {
    __shared__ double bestE_sh[9];
    __shared__ float cand[kBatch][kMaxSol * 9 + 1];  // candidates of the batch, one padded row per lane
    __shared__ int nsol[kBatch];
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const int M = match_count[p];
    uint8_t* mask = out.mask + (size_t)p * mcap;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    if (M < 6) {  // opencv_verifier_base.py:69-78
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 1;
            if (out.n_hyp) out.n_hyp[p] = 0;
        }
        for (int i = lane; i < M; i += 64) mask[i] = 0;
        if (lane == 0) best_out[p] = make_int4(-1, -1, -1, 0);
        return;
    }
    const double fx = fmax(intr[3 * i1], intr[3 * i2]);  // opencv_verifier_base.py:86
    const double thr = thr_px / fx;
    const float thr2 = (float)(thr * thr);
    const double2* x1 = x1n_all + (size_t)p * mcap;
    const double2* x2 = x2n_all + (size_t)p * mcap;
    const float4* pts = pts_all + (size_t)p * mcap;
    const int pair_id = pair_id_base + p;

    int best = -1, best_h = -1, best_s = -1;
    int niters = max_iters, done = 0;
    while (done < niters) {
        // lane-per-hypothesis minimal solves; candidates go to this lane's LDS row
        int ns = 0;
        {
            const int h = done + lane;
            int idx[5];
            if (sample5(seed, pair_id, h, M, idx)) {
                double s1[10], s2[10], Es[9 * kMaxSol];
                for (int k = 0; k < 5; ++k) {
                    const double2 a = x1[idx[k]], b = x2[idx[k]];
                    s1[2 * k] = a.x; s1[2 * k + 1] = a.y;
                    s2[2 * k] = b.x; s2[2 * k + 1] = b.y;
                }
                ns = five_point(s1, s2, Es);
                for (int k = 0; k < 9 * ns; ++k) cand[lane][k] = (float)Es[k];
            }
            nsol[lane] = ns;
        }
        __syncthreads();
        // wave-cooperative scoring of every candidate, in (hypothesis, solution) order
        for (int hl = 0; hl < kBatch; ++hl) {
            const int nsh = nsol[hl];
            for (int s = 0; s < nsh; ++s) {
                float E[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) E[e] = cand[hl][9 * s + e];  // LDS broadcast
                const int c = wave_count(E, pts, M, thr2, best, lane);
                if (c > best) {
                    best = c;
                    best_h = done + hl;
                    best_s = s;
                }
            }
        }
        __syncthreads();  // cand/nsol are rewritten by the next batch
        done += kBatch;
        if (best > 0) {
            const int upd = update_num_iters(prob, (double)(M - best) / M, 5, niters);
            if (upd < niters) niters = upd;
        }
    }
    if (best <= 0) {
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 2;
            if (out.n_hyp) out.n_hyp[p] = done;
        }
        for (int i = lane; i < M; i += 64) mask[i] = 0;
    }
    if (lane == 0) best_out[p] = make_int4(best, best_h, best_s, done);
}

// Refinement of each pair's winning hypothesis: fp64 re-solve, iterative LO, final mask, recoverPose.
__global__ __launch_bounds__(64) void ransac_refine_kernel(const int* __restrict__ pairs,
                                                           const double* __restrict__ intr,
                                                           const int* __restrict__ match_count, int mcap,
                                                           const double2* __restrict__ x1n_all,
                                                           const double2* __restrict__ x2n_all,
                                                           const float4* __restrict__ pts_all, double thr_px,
                                                           uint64_t seed, int pair_id_base, RansacOutputs out,
                                                           const int4* __restrict__ best_in) {
    __shared__ double bestE_sh[9];
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const int M = match_count[p];
    const int4 bst = best_in[p];
    if (M < 6 || bst.x <= 0) return;  // status already written by ransac_hypotheses_kernel
    const int best_h = bst.y, best_s = bst.z, done = bst.w;
    uint8_t* mask = out.mask + (size_t)p * mcap;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const double fx = fmax(intr[3 * i1], intr[3 * i2]);
    const double thr = thr_px / fx;
    const float thr2 = (float)(thr * thr);
    const double2* x1 = x1n_all + (size_t)p * mcap;
    const double2* x2 = x2n_all + (size_t)p * mcap;
    const float4* pts = pts_all + (size_t)p * mcap;
    const int pair_id = pair_id_base + p;

    // re-solve the winning hypothesis in fp64 (deterministic) to recover its double-precision E
    if (lane == 0) {
        int idx[5];
        sample5(seed, pair_id, best_h, M, idx);
        double s1[10], s2[10], Es[9 * kMaxSol];
        for (int k = 0; k < 5; ++k) {
            const double2 a = x1[idx[k]], b = x2[idx[k]];
            s1[2 * k] = a.x; s1[2 * k + 1] = a.y;
            s2[2 * k] = b.x; s2[2 * k + 1] = b.y;
        }
        five_point(s1, s2, Es);
        for (int e = 0; e < 9; ++e) bestE_sh[e] = Es[9 * best_s + e];
    }
    __syncthreads();
    double bestE[9];
    for (int e = 0; e < 9; ++e) bestE[e] = bestE_sh[e];

    // iterative LO (oracle/ransac.c): thresholds kLoMult*thr -> thr, Sampson-weighted refits
    auto count_d = [&](const double* Ed) {
        float Ef[9];
        for (int e = 0; e < 9; ++e) Ef[e] = (float)Ed[e];
        return wave_count(Ef, pts, M, thr2, -1, lane);
    };
    int cur = count_d(bestE);
    {
        double E[9];
        for (int e = 0; e < 9; ++e) E[e] = bestE[e];
        for (int k = 0; k < kLoSteps; ++k) {
            const double th = thr * (kLoMult - (kLoMult - 1.0) * k / (kLoSteps - 1));
            double Esel[9], En[9];
            for (int e = 0; e < 9; ++e) Esel[e] = E[e];
            if (!wave_refit(x1, x2, M, Esel, th * th, Esel, En, lane)) break;
            bool ok = true;
            for (int r = 1; r < kLoIrls && ok; ++r) {
                double Et[9];
                ok = wave_refit(x1, x2, M, Esel, th * th, En, Et, lane);
                if (ok)
                    for (int e = 0; e < 9; ++e) En[e] = Et[e];
            }
            const int c = count_d(En);
            for (int e = 0; e < 9; ++e) E[e] = En[e];
            if (c >= cur) {
                cur = c;
                for (int e = 0; e < 9; ++e) bestE[e] = En[e];
            }
        }
    }
    // final inlier mask at thr
    {
        float Ef[9];
        for (int e = 0; e < 9; ++e) Ef[e] = (float)bestE[e];
        int c = 0;
        for (int i = lane; i < M; i += 64) {
            const bool in = sampson_inlier(Ef, pts[i], thr2);
            mask[i] = in ? 1 : 0;
            c += in ? 1 : 0;
        }
        for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
        cur = c;
    }
    __syncthreads();  // mask visible to every lane of the workgroup
    // recoverPose: decomposition (redundant per lane) + wave cheirality vote
    double U[9], s[3], V[9];
    svd3(bestE, U, s, V);
    if (det3(U) < 0)
        for (int k = 0; k < 9; ++k) U[k] = -U[k];
    if (det3(V) < 0)
        for (int k = 0; k < 9; ++k) V[k] = -V[k];
    double R1[9], R2[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            const double uw0 = -U[r * 3 + 1], uw1 = U[r * 3 + 0], uw2 = U[r * 3 + 2];
            const double uwt0 = U[r * 3 + 1], uwt1 = -U[r * 3 + 0], uwt2 = U[r * 3 + 2];
            R1[r * 3 + c] = uw0 * V[c * 3 + 0] + uw1 * V[c * 3 + 1] + uw2 * V[c * 3 + 2];
            R2[r * 3 + c] = uwt0 * V[c * 3 + 0] + uwt1 * V[c * 3 + 1] + uwt2 * V[c * 3 + 2];
        }
    const double tp[3] = {U[2], U[5], U[8]};
    const double tn[3] = {-U[2], -U[5], -U[8]};
    const int g1 = wave_cheirality(R1, tp, x1, x2, mask, M, lane);
    const int g2 = wave_cheirality(R2, tp, x1, x2, mask, M, lane);
    const int g3 = wave_cheirality(R1, tn, x1, x2, mask, M, lane);
    const int g4 = wave_cheirality(R2, tn, x1, x2, mask, M, lane);
    const double* Rs;
    const double* ts;
    if (g1 >= g2 && g1 >= g3 && g1 >= g4) { Rs = R1; ts = tp; }
    else if (g2 >= g1 && g2 >= g3 && g2 >= g4) { Rs = R2; ts = tp; }
    else if (g3 >= g1 && g3 >= g2 && g3 >= g4) { Rs = R1; ts = tn; }
    else { Rs = R2; ts = tn; }
    if (lane == 0) {
        for (int k = 0; k < 9; ++k) {
            out.E[9 * p + k] = bestE[k];
            out.R[9 * p + k] = Rs[k];
        }
        for (int k = 0; k < 3; ++k) out.t[3 * p + k] = ts[k];
        out.n_inliers[p] = cur;
        out.status[p] = 0;
        if (out.n_hyp) out.n_hyp[p] = done;
    }
}

}  // namespace

extern "C" {

size_t gtsfm_ransac_workspace_bytes(int n_pairs, int mcap) {
    if (n_pairs <= 0 || mcap <= 0) return 0;
    const size_t n = (size_t)n_pairs * mcap;
    return gtsfm_align_up(n * sizeof(double2), 256) * 2 + gtsfm_align_up(n * sizeof(float4), 256) +
           gtsfm_align_up((size_t)n_pairs * sizeof(int4), 256);
}

int gtsfm_ransac_E_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax, const int* d_pairs,
                           int n_pairs, const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                           double thr_px, double prob, int max_iters, uint64_t seed, int pair_id_base,
                           void* d_workspace, size_t workspace_bytes, double* d_E, double* d_R, double* d_t,
                           int* d_n_inliers, int* d_status, int* d_n_hyp, uint8_t* d_inlier_mask, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_kp_xy || !d_intrinsics || !d_pairs || !d_match_idx || !d_match_count || !d_E || !d_R || !d_t ||
        !d_n_inliers || !d_status || !d_inlier_mask || n_img <= 0 || kmax <= 0 || n_pairs < 0 || mcap <= 0 ||
        max_iters <= 0 || !(thr_px > 0.0))
        return GTSFM_ERR_ARG;
    if (workspace_bytes < gtsfm_ransac_workspace_bytes(n_pairs, mcap)) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    const size_t n = (size_t)n_pairs * mcap;
    double2* x1n = (double2*)ws;
    double2* x2n = (double2*)(ws + gtsfm_align_up(n * sizeof(double2), 256));
    float4* pts = (float4*)(ws + 2 * gtsfm_align_up(n * sizeof(double2), 256));
    hipLaunchKernelGGL(normalize_putatives_kernel, dim3((mcap + 255) / 256, n_pairs), dim3(256), 0, stream, d_kp_xy,
                       d_intrinsics, kmax, d_pairs, d_match_idx, d_match_count, mcap, x1n, x2n, pts);
    GTSFM_CHECK_HIP(hipGetLastError());
    int4* best = (int4*)(ws + 2 * gtsfm_align_up(n * sizeof(double2), 256) + gtsfm_align_up(n * sizeof(float4), 256));
    const RansacOutputs o{d_E, d_R, d_t, d_n_inliers, d_status, d_n_hyp, d_inlier_mask};
    hipLaunchKernelGGL(ransac_hypotheses_kernel, dim3(n_pairs), dim3(64), 0, stream, d_pairs, d_intrinsics,
                       d_match_count, mcap, x1n, x2n, pts, thr_px, prob, max_iters, seed, pair_id_base, o, best);
    GTSFM_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(ransac_refine_kernel, dim3(n_pairs), dim3(64), 0, stream, d_pairs, d_intrinsics, d_match_count,
                       mcap, x1n, x2n, pts, thr_px, seed, pair_id_base, o, best);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
