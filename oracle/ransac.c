/*
 * ORACLE — test infrastructure only. CPU restatement of the reference's E-matrix verifier, used as the checker
 * for the HIP verifier and as the CPU baseline. The product path never calls it.
 *
 * Reference path (/root/reference):
 *   gtsfm/frontend/verifier/opencv_verifier_base.py:45-109  verify(): M<5 / M<6 failure, normalise all keypoints
 *       with K (utils/features.py:40-50), fx = max(fx1, fx2), estimate_E, inlier idxs, inlier_ratio = mean(mask),
 *       recover_relative_pose_from_essential_matrix
 *   gtsfm/frontend/verifier/ransac.py:52-82  cv2.findEssentialMat(x1n, x2n, I3, USAC_ACCURATE,
 *       threshold = px / fx, prob = 0.999999)   (maxIters: OpenCV default 1000)
 *   gtsfm/utils/verification.py:52-94  cv.recoverPose(E, x1n, x2n)
 * Third-party algorithm restated (OpenCV, opencv-python>=4.5.4.58, environment_linux.yml:50; its USAC/GC-RANSAC
 * internals — graph-cut LO, SPRT, its RNG — are not reproducible without its source, so parity with OpenCV is
 * tolerance-based and pinned by the reference's known-answer verifier tests):
 *   - minimal solver: Nister's 5-point algorithm (TPAMI 2004): 4-dim null space of the 5x9 epipolar system,
 *     10 cubic constraints (det E = 0, 2EE^TE - tr(EE^T)E = 0) in 20 monomials, elimination to [I | C] (the rows
 *     B(z) reads), the 3x3
 *     polynomial matrix B(z), degree-10 det B(z); real roots by Sturm-sequence isolation + bisection.
 *   - inlier test: squared Sampson distance <= threshold^2 (OpenCV EMEstimatorCallback::computeError), written
 *     division-free: (x2'Ex1)^2 <= thr^2 * (|Ex1|_xy^2 + |E'x2|_xy^2), float32 with explicit fmaf.
 *   - RANSAC: hypotheses in batches of 64; the OpenCV iteration bound RANSACUpdateNumIters(p, 1-best/M, 5, n)
 *     is re-evaluated after each batch (best = the inlier count of the selected model); maxIters 1000.
 *     Model selection (`scoring`): 0 = RANSAC, most inliers (cv2 RANSAC); 1 = MSAC, as USAC_ACCURATE scores
 *     (truncated quadratic sum_i min(e_i, thr^2), lowest wins), with each term quantised to an integer so the
 *     sum is exact in any order: q_i = floor(e_i * 2^16 / thr^2) clamped to 65535 for an inlier, 65536 for an
 *     outlier, e_i = num^2 / den in float32. The first candidate wins ties in both modes.
 *   - local optimisation: for MSAC, GC-RANSAC's graph-cut LO (USAC_ACCURATE's LOCAL_OPTIM_GC; gc_label below);
 *     for RANSAC, the iterative LO of Lebeda et al. (BMVC 2012): 4 steps with the selection threshold shrinking
 *     from 6*thr to thr. Both refit with 3 rounds of Sampson-weighted (IRLS) linear 8-point on the selected points,
 *     projected onto the essential manifold; a refined model is kept when its score improves.
 *   - recoverPose: SVD decomposition into 4 (R,t), cheirality count (depth in (0, 50) in both cameras).
 * Deterministic sampling: splitmix64 counter hash of (seed, pair id, hypothesis, draw) — the HIP kernel draws the
 * same samples.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* isolation stack depth (== gtsfm_amd/csrc/ransac.hip kStack): the DFS holds at most one pending interval per
 * bisection level, so 24 separates roots down to 2 * bound / 2^23 apart; closer pairs are skipped */
#define ISO_STACK 24

#define NMONO 20
#define RANSAC_BATCH 64
#define MAX_SOL 10
#define LO_STEPS 4
#define LO_IRLS 3
#define LO_MULT 6.0
/* graph-cut LO (the MSAC path's LO, GC-RANSAC as USAC_ACCURATE configures it): at most GC_ITERS labelling + refit
 * rounds, grid cells of GC_CELL_THR inlier thresholds (50 px at sift_front_end.yaml's 4 px), spatial coherence
 * lambda = GC_LAM_NUM / GC_LAM_DEN; pairs with more than GC_MAX_M putatives keep the iterative LO (the device's sort
 * key holds a 15-bit index) */
#define GC_ITERS 10
#define GC_CELL_THR 12.5
#define GC_LAM_NUM 39
#define GC_LAM_DEN 40
#define GC_MAX_M 32768

/* ------------------------------------------------------------------ sampling */
static uint64_t sm_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* 5 distinct indices in [0, M) for hypothesis h of pair `pair`. Returns 0 if no distinct set in 32 draws. */
int oracle_sample5(uint64_t seed, int pair, int h, int M, int* idx) {
    const uint64_t key = sm_mix(seed ^ sm_mix((uint64_t)(uint32_t)pair));
    int n = 0;
    for (int d = 0; d < 32 && n < 5; ++d) {
        const uint64_t r = sm_mix(key + (uint64_t)h * 32u + (uint64_t)d);
        const int v = (int)(((r >> 32) * (uint64_t)(uint32_t)M) >> 32);
        int dup = 0;
        for (int k = 0; k < n; ++k) dup |= (idx[k] == v);
        if (!dup) idx[n++] = v;
    }
    return n == 5;
}

/* ------------------------------------------------------------------ polynomial algebra in (x, y, z) */
/* linear: [x, y, z, 1]; quadratic: [xx, yy, xy, xz, yz, zz, x, y, z, 1];
 * cubic (Nister order): [xxx, yyy, xxy, xyy, xxz, xx, yyz, yy, xyz, xy, xzz, xz, x, yzz, yz, y, zzz, zz, z, 1] */
static const int LIN_E[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
static const int QUAD_E[10][3] = {{2, 0, 0}, {0, 2, 0}, {1, 1, 0}, {1, 0, 1}, {0, 1, 1},
                                  {0, 0, 2}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
static const int CUB_E[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                                 {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                                 {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};

static int find_mono(const int (*tab)[3], int n, int a, int b, int c) {
    for (int i = 0; i < n; ++i)
        if (tab[i][0] == a && tab[i][1] == b && tab[i][2] == c) return i;
    return -1;
}

static int LL2Q[4][4], QL2C[10][4];
static int tables_ready = 0;
static void init_tables(void) {
    if (tables_ready) return;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            LL2Q[i][j] = find_mono(QUAD_E, 10, LIN_E[i][0] + LIN_E[j][0], LIN_E[i][1] + LIN_E[j][1],
                                   LIN_E[i][2] + LIN_E[j][2]);
    for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 4; ++j)
            QL2C[i][j] = find_mono(CUB_E, 20, QUAD_E[i][0] + LIN_E[j][0], QUAD_E[i][1] + LIN_E[j][1],
                                   QUAD_E[i][2] + LIN_E[j][2]);
    tables_ready = 1;
}

static void mul_ll(const double* a, const double* b, double* q) { /* q = a*b */
    memset(q, 0, 10 * sizeof(double));
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) q[LL2Q[i][j]] = fma(a[i], b[j], q[LL2Q[i][j]]);
}
/* c += s * q*l; s is 1, -1 or 2, so s * q[i] is exact and every term is one fused multiply-add */
static void addmul_ql(const double* q, const double* l, double s, double* c) {
    for (int i = 0; i < 10; ++i) {
        const double sq = s * q[i];
        for (int j = 0; j < 4; ++j) c[QL2C[i][j]] = fma(sq, l[j], c[QL2C[i][j]]);
    }
}

/* ------------------------------------------------------------------ univariate polynomials (ascending coeffs) */
static double peval(const double* p, int deg, double x) {
    double v = p[deg];
    for (int i = deg - 1; i >= 0; --i) v = fma(v, x, p[i]);
    return v;
}

/* r = a mod b (deg_a >= deg_b), returns degree of r (-1 if zero) */
static int prem(const double* a, int da, const double* b, int db, double* r) {
    double t[11];
    for (int i = 0; i <= da; ++i) t[i] = a[i];
    for (int k = da; k >= db; --k) {
        const double f = t[k] / b[db];
        for (int i = 0; i <= db; ++i) t[k - db + i] = fma(-f, b[i], t[k - db + i]);
        t[k] = 0.0;
    }
    int dr = db - 1;
    double scale = 0.0;
    for (int i = 0; i <= da; ++i) scale = fmax(scale, fabs(a[i]));
    while (dr >= 0 && fabs(t[dr]) <= 1e-14 * scale) --dr;
    for (int i = 0; i <= dr; ++i) r[i] = t[i];
    return dr;
}

typedef struct {
    double p[11][11];
    int deg[11];
    int n; /* number of polynomials in the chain */
} sturm_t;

static int sign_changes(const sturm_t* s, double x) {
    int c = 0;
    double prev = 0.0;
    for (int k = 0; k < s->n; ++k) {
        const double v = peval(s->p[k], s->deg[k], x);
        if (v == 0.0) continue;
        if (prev != 0.0 && ((v < 0.0) != (prev < 0.0))) ++c;
        prev = v;
    }
    return c;
}

/* Real roots of p (degree <= 10) in ascending order. Returns the count. */
/* Root-magnitude bound of a monic polynomial (Fujiwara: |z| <= 2 max_k |p[deg-k]|^(1/k), the constant term halved),
   rounded up to a power of two with exact exponent arithmetic (frexp), so CPU and GPU agree bit for bit. */
static double root_bound_pow2(const double* p, int deg) {
    int emax = -2000;
    for (int k = 1; k <= deg; ++k) {
        double m = fabs(p[deg - k]);
        if (k == deg) m *= 0.5;
        if (m == 0.0) continue;
        int x;
        frexp(m, &x); /* m < 2^x */
        const int c = x >= 0 ? (x + k - 1) / k : -((-x) / k); /* ceil(x / k) */
        if (c > emax) emax = c;
    }
    if (emax == -2000) emax = 0;
    return ldexp(1.0, emax + 1);
}

static int real_roots(const double* pin, int deg, double* roots) {
    double p[11];
    while (deg > 0 && fabs(pin[deg]) <= 1e-300) --deg;
    if (deg <= 0) return 0;
    for (int i = 0; i <= deg; ++i) p[i] = pin[i] / pin[deg];
    sturm_t s;
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
    const double bound = root_bound_pow2(p, deg);
    /* isolation by bisection with Sturm counts */
    double st_a[ISO_STACK], st_b[ISO_STACK];
    int st_va[ISO_STACK], st_vb[ISO_STACK], ns = 0, nr = 0;
    st_a[0] = -bound;
    st_b[0] = bound;
    st_va[0] = sign_changes(&s, -bound);
    st_vb[0] = sign_changes(&s, bound);
    ns = 1;
    int guard = 0;
    while (ns > 0 && nr < MAX_SOL && guard < 2000) {
        ++guard;
        --ns;
        const double a = st_a[ns], b = st_b[ns];
        const int va = st_va[ns], vb = st_vb[ns];
        const int cnt = va - vb;
        if (cnt <= 0) continue;
        if (cnt == 1 || b - a < 1e-10 * fmax(1.0, fabs(a))) {
            /* refine: bisection down to a relative width of 2^-20, then 4 safeguarded Newton steps (p' is Sturm
             * row 1; a step landing on a bracket end is kept, so a root within rounding of an end is reached) */
            double lo = a, hi = b;
            double flo = peval(p, deg, lo);
            for (int it = 0; it < 80; ++it) {
                if (hi - lo <= 0x1p-20 * fmax(1.0, fmax(fabs(lo), fabs(hi)))) break;
                const double mid = 0.5 * (lo + hi);
                const double fm = peval(p, deg, mid);
                if ((fm < 0.0) == (flo < 0.0) && fm != 0.0) {
                    lo = mid;
                    flo = fm;
                } else {
                    hi = mid;
                }
            }
            double x = 0.5 * (lo + hi);
            for (int it = 0; it < 4; ++it) {
                const double fx = peval(p, deg, x), dfx = peval(s.p[1], s.deg[1], x);
                if (fx == 0.0) break;
                if ((fx < 0.0) == (flo < 0.0)) {
                    lo = x;
                    flo = fx;
                } else {
                    hi = x;
                }
                const double xn = x - fx / dfx;
                x = (xn >= lo && xn <= hi) ? xn : 0.5 * (lo + hi);
            }
            roots[nr++] = x;
            continue;
        }
        const double mid = 0.5 * (a + b);
        const int vm = sign_changes(&s, mid);
        if (ns + 2 <= ISO_STACK) {
            /* push right then left so that the left interval is processed first (ascending roots) */
            st_a[ns] = mid; st_b[ns] = b; st_va[ns] = vm; st_vb[ns] = vb; ++ns;
            st_a[ns] = a; st_b[ns] = mid; st_va[ns] = va; st_vb[ns] = vm; ++ns;
        }
    }
    return nr;
}

/* ------------------------------------------------------------------ 5-point solver */
/* Null space of the 5 x 9 epipolar system: Householder QR of its transpose, M^T (9 x 5) = H_0 H_1 ... H_4 [R; 0],
 * H_k = I - beta_k v_k v_k^T acting on entries k..8; columns 5..8 of H_0 ... H_4 (each built by applying H_4 first)
 * are an orthonormal basis of null(M). Every index is static, so the device keeps the whole factorisation in
 * registers (gtsfm_amd/csrc/ransac.hip nullspace_5x9, the same operations). Returns 0 when a column's remaining norm
 * is below 1e-12 (rank < 5: a degenerate sample). */
static int nullspace_5x9(const double q[5][9], double N[4][9]) {
    double a[5][9], v[5][9], beta[5];
    memcpy(a, q, sizeof(a)); /* a[c][r] = M^T[r][c]: column c of M^T is row c of M */
    for (int k = 0; k < 5; ++k) {
        double s = 0.0;
        for (int r = k; r < 9; ++r) s = fma(a[k][r], a[k][r], s);
        const double nrm = sqrt(s);
        if (nrm < 1e-12) return 0;
        const double alpha = a[k][k] >= 0.0 ? -nrm : nrm;
        for (int r = k; r < 9; ++r) v[k][r] = a[k][r];
        v[k][k] = v[k][k] - alpha;
        double vv = 0.0;
        for (int r = k; r < 9; ++r) vv = fma(v[k][r], v[k][r], vv);
        beta[k] = 2.0 / vv;
        for (int c = k + 1; c < 5; ++c) {
            double d = 0.0;
            for (int r = k; r < 9; ++r) d = fma(v[k][r], a[c][r], d);
            d = d * beta[k];
            for (int r = k; r < 9; ++r) a[c][r] = fma(-d, v[k][r], a[c][r]);
        }
    }
    for (int n = 0; n < 4; ++n) {
        double y[9] = {0};
        y[5 + n] = 1.0;
        for (int k = 4; k >= 0; --k) {
            double d = 0.0;
            for (int r = k; r < 9; ++r) d = fma(v[k][r], y[r], d);
            d = d * beta[k];
            for (int r = k; r < 9; ++r) y[r] = fma(-d, v[k][r], y[r]);
        }
        for (int j = 0; j < 9; ++j) N[n][j] = y[j];
    }
    return 1;
}

/* The 10 x 20 constraint rows of Nister's 5-point for E = sum N_k (x, y, z, 1)_k: row 0 det(E), rows 1..9
 * 2 EE^T E - tr(EE^T) E (cubic coefficients in the Nister order above). */
static void build_rows(const double E[9][4], double A[10][NMONO]) {
    memset(A, 0, 10 * NMONO * sizeof(double));
    {
        double q[10];
        mul_ll(E[4], E[8], q); addmul_ql(q, E[0], 1.0, A[0]);
        mul_ll(E[5], E[7], q); addmul_ql(q, E[0], -1.0, A[0]);
        mul_ll(E[3], E[8], q); addmul_ql(q, E[1], -1.0, A[0]);
        mul_ll(E[5], E[6], q); addmul_ql(q, E[1], 1.0, A[0]);
        mul_ll(E[3], E[7], q); addmul_ql(q, E[2], 1.0, A[0]);
        mul_ll(E[4], E[6], q); addmul_ql(q, E[2], -1.0, A[0]);
    }
    /* EE^T (quadratic, symmetric), trace */
    double EEt[3][3][10], tr[10], tmp[10];
    for (int i = 0; i < 3; ++i)
        for (int j = i; j < 3; ++j) {
            memset(EEt[i][j], 0, sizeof(tmp));
            for (int k = 0; k < 3; ++k) {
                mul_ll(E[3 * i + k], E[3 * j + k], tmp);
                for (int m = 0; m < 10; ++m) EEt[i][j][m] += tmp[m];
            }
            if (j != i) memcpy(EEt[j][i], EEt[i][j], sizeof(tmp));
        }
    for (int m = 0; m < 10; ++m) tr[m] = EEt[0][0][m] + EEt[1][1][m] + EEt[2][2][m];
    /* 2 EE^T E - tr(EE^T) E */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double* row = A[1 + 3 * i + j];
            for (int k = 0; k < 3; ++k) addmul_ql(EEt[i][k], E[3 * k + j], 2.0, row);
            addmul_ql(tr, E[3 * i + j], -1.0, row);
        }
}

/* Nister 5-point: x1, x2 are 5 normalized points (x,y). Writes up to 10 E (row-major, unit Frobenius norm). */
int oracle_five_point(const double* x1, const double* x2, double* Es) {
    init_tables();
    double Q[5][9];
    for (int i = 0; i < 5; ++i) {
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        const double row[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        memcpy(Q[i], row, sizeof(row));
    }
    double N[4][9];
    if (!nullspace_5x9(Q, N)) return 0;
    /* E_ij as linear polynomial [x, y, z, 1] with X = N0, Y = N1, Z = N2, W = N3 */
    double E[9][4];
    for (int e = 0; e < 9; ++e) {
        E[e][0] = N[0][e];
        E[e][1] = N[1][e];
        E[e][2] = N[2][e];
        E[e][3] = N[3][e];
    }
    double A[10][NMONO];
    build_rows(E, A);
    /* Columns 10..19 come from the rows of the renamed E. Read homogeneously in (x, y, z, w = 1), columns 0..9 are
     * the cubic monomials with at least two factors from {x, y}, columns 10..19 those with at least two from {z, w};
     * the renaming (x, y, z, w) -> (z, w, x, y) maps the second set onto the first, so columns 0..9 of the renamed
     * rows are columns 10..19 of these (same values up to rounding, the summation order being the renamed one). This
     * is the construction the device uses: each lane of a pair builds only its own ten columns with the same code
     * (gtsfm_amd/csrc/ransac.hip five_point_stage1, kHiCol). */
    {
        static const int HI_COL[10] = {16, 19, 17, 18, 10, 13, 12, 15, 11, 14};
        double Er[9][4], Ar[10][NMONO];
        for (int e = 0; e < 9; ++e) {
            Er[e][0] = E[e][2];
            Er[e][1] = E[e][3];
            Er[e][2] = E[e][0];
            Er[e][3] = E[e][1];
        }
        build_rows(Er, Ar);
        for (int r = 0; r < 10; ++r)
            for (int k = 0; k < 10; ++k) A[r][HI_COL[k]] = Ar[r][k];
    }

    /* Gaussian elimination with partial pivoting on columns 0..9 (each pivot row scaled to a unit pivot), then
     * back-substitution of rows 4..9 only -> rows 4..9 of [I | C], all that B(z) reads. The pivots are Gauss-Jordan's;
     * rows 0..3 are not reduced above their pivots (the device's order: ransac.hip five_point_stage1). */
    for (int c = 0; c < 10; ++c) {
        int pr = c;
        double best = fabs(A[c][c]);
        for (int r = c + 1; r < 10; ++r)
            if (fabs(A[r][c]) > best) { best = fabs(A[r][c]); pr = r; }
        if (best < 1e-14) return 0;
        if (pr != c)
            for (int j = 0; j < NMONO; ++j) { double t = A[c][j]; A[c][j] = A[pr][j]; A[pr][j] = t; }
        const double inv = 1.0 / A[c][c];
        for (int j = 0; j < NMONO; ++j) A[c][j] *= inv;
        for (int r = c + 1; r < 10; ++r) {
            const double f = A[r][c];
            for (int j = 0; j < NMONO; ++j) A[r][j] = fma(-f, A[c][j], A[r][j]);
        }
    }
    for (int c = 9; c >= 5; --c)
        for (int r = 4; r < c; ++r) {
            const double f = A[r][c];
            for (int j = 0; j < NMONO; ++j) A[r][j] = fma(-f, A[c][j], A[r][j]);
        }
    /* B(z): rows k = e - z f, l = g - z h, m = i - z j (rows 4..9); columns [x-coef(deg3), y-coef(deg3), 1(deg4)] */
    /* trailing columns: 10 xzz, 11 xz, 12 x, 13 yzz, 14 yz, 15 y, 16 zzz, 17 zz, 18 z, 19 one */
    double B[3][3][5];
    memset(B, 0, sizeof(B));
    for (int r = 0; r < 3; ++r) {
        const double* e = A[4 + 2 * r];
        const double* f = A[5 + 2 * r];
        /* x coefficient: e.xzz z^2 + e.xz z + e.x - z (f.xzz z^2 + f.xz z + f.x) */
        B[r][0][0] = e[12];
        B[r][0][1] = e[11] - f[12];
        B[r][0][2] = e[10] - f[11];
        B[r][0][3] = -f[10];
        B[r][1][0] = e[15];
        B[r][1][1] = e[14] - f[15];
        B[r][1][2] = e[13] - f[14];
        B[r][1][3] = -f[13];
        B[r][2][0] = e[19];
        B[r][2][1] = e[18] - f[19];
        B[r][2][2] = e[17] - f[18];
        B[r][2][3] = e[16] - f[17];
        B[r][2][4] = -f[16];
    }
    /* n(z) = det B(z), degree 10: sum over cyclic (c, c1, c2) of B0c * (B1c1 B2c2 - B1c2 B2c1) */
    double n[11];
    memset(n, 0, sizeof(n));
    {
        const int deg[3] = {3, 3, 4};
        for (int c = 0; c < 3; ++c) {
            const int c1 = (c + 1) % 3, c2 = (c + 2) % 3;
            double m[9];
            memset(m, 0, sizeof(m));
            for (int i = 0; i <= deg[c1]; ++i)
                for (int j = 0; j <= deg[c2]; ++j) m[i + j] = fma(B[1][c1][i], B[2][c2][j], m[i + j]);
            for (int i = 0; i <= deg[c2]; ++i)
                for (int j = 0; j <= deg[c1]; ++j) m[i + j] = fma(-B[1][c2][i], B[2][c1][j], m[i + j]);
            const int dm = deg[c1] + deg[c2];
            for (int i = 0; i <= deg[c]; ++i)
                for (int j = 0; j <= dm; ++j) n[i + j] = fma(B[0][c][i], m[j], n[i + j]);
        }
    }
    double roots[MAX_SOL];
    const int nroots = real_roots(n, 10, roots);
    int nsol = 0;
    for (int k = 0; k < nroots; ++k) {
        const double z = roots[k];
        double Bz[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Bz[r][c] = peval(B[r][c], c == 2 ? 4 : 3, z);
        /* null vector of Bz: the largest of the three row cross products */
        double best[3] = {0, 0, 0}, bn = -1.0;
        for (int a = 0; a < 3; ++a) {
            const int b = (a + 1) % 3;
            const double cx = Bz[a][1] * Bz[b][2] - Bz[a][2] * Bz[b][1];
            const double cy = Bz[a][2] * Bz[b][0] - Bz[a][0] * Bz[b][2];
            const double cz = Bz[a][0] * Bz[b][1] - Bz[a][1] * Bz[b][0];
            const double nn = cx * cx + cy * cy + cz * cz;
            if (nn > bn) { bn = nn; best[0] = cx; best[1] = cy; best[2] = cz; }
        }
        if (!(fabs(best[2]) > 1e-300)) continue;
        const double x = best[0] / best[2], y = best[1] / best[2];
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

/* ------------------------------------------------------------------ scoring (float32, explicit fma) */
static int sampson_inlier(const float* E, float x1, float y1, float x2, float y2, float thr2) {
    const float a0 = fmaf(E[1], y1, fmaf(E[0], x1, E[2]));
    const float a1 = fmaf(E[4], y1, fmaf(E[3], x1, E[5]));
    const float a2 = fmaf(E[7], y1, fmaf(E[6], x1, E[8]));
    const float b0 = fmaf(E[3], y2, fmaf(E[0], x2, E[6]));
    const float b1 = fmaf(E[4], y2, fmaf(E[1], x2, E[7]));
    const float num = fmaf(y2, a1, fmaf(x2, a0, a2));
    const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, a0 * a0)));
    return num * num <= thr2 * den;
}

/* MSAC term of one correspondence (see the header): the inlier test of sampson_inlier, then the quantised error */
static uint32_t msac_cost(const float* E, float x1, float y1, float x2, float y2, float thr2, float scale, int* in) {
    const float a0 = fmaf(E[1], y1, fmaf(E[0], x1, E[2]));
    const float a1 = fmaf(E[4], y1, fmaf(E[3], x1, E[5]));
    const float a2 = fmaf(E[7], y1, fmaf(E[6], x1, E[8]));
    const float b0 = fmaf(E[3], y2, fmaf(E[0], x2, E[6]));
    const float b1 = fmaf(E[4], y2, fmaf(E[1], x2, E[7]));
    const float num = fmaf(y2, a1, fmaf(x2, a0, a2));
    const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, a0 * a0)));
    const float nn = num * num;
    *in = nn <= thr2 * den;
    if (!*in) return 65536u;
    const float r = den > 0.0f ? nn / den : 0.0f;
    const float q = r * scale;
    return q < 65535.0f ? (uint32_t)q : 65535u;
}

/* MSAC score of E (and its inlier count in *count, mask when non-NULL) */
static uint32_t msac_score(const double* Ed, const float* pts, int M, float thr2, int* count, uint8_t* mask) {
    float E[9];
    for (int k = 0; k < 9; ++k) E[k] = (float)Ed[k];
    const float scale = 65536.0f / thr2;
    uint32_t s = 0;
    int c = 0;
    for (int i = 0; i < M; ++i) {
        int in;
        s += msac_cost(E, pts[4 * i], pts[4 * i + 1], pts[4 * i + 2], pts[4 * i + 3], thr2, scale, &in);
        if (mask) mask[i] = (uint8_t)in;
        c += in;
    }
    *count = c;
    return s;
}

static int count_inliers(const double* Ed, const float* pts, int M, float thr2, uint8_t* mask) {
    float E[9];
    for (int k = 0; k < 9; ++k) E[k] = (float)Ed[k];
    int c = 0;
    for (int i = 0; i < M; ++i) {
        const int in = sampson_inlier(E, pts[4 * i], pts[4 * i + 1], pts[4 * i + 2], pts[4 * i + 3], thr2);
        if (mask) mask[i] = (uint8_t)in;
        c += in;
    }
    return c;
}

/* ------------------------------------------------------------------ small symmetric eigen / SVD helpers */
/* Cyclic Jacobi on a symmetric n x n matrix (n <= 9). Eigenvalues in w, eigenvectors in columns of V. */
static void jacobi_eig(double* a, int n, double* w, double* V) {
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

/* SVD of 3x3 E = U diag(s) V^T, s descending, via eigen of E^T E. U completed to a rotation-compatible basis. */
static void svd3(const double* E, double* U, double* s, double* V) {
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
            if (w[order[j]] > w[order[i]]) { int t = order[i]; order[i] = order[j]; order[j] = t; }
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
    /* third columns: cross products (rank-2 E) */
    U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
    U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
    U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
    double v3[3] = {V[1 * 3 + 0] * V[2 * 3 + 1] - V[2 * 3 + 0] * V[1 * 3 + 1],
                    V[2 * 3 + 0] * V[0 * 3 + 1] - V[0 * 3 + 0] * V[2 * 3 + 1],
                    V[0 * 3 + 0] * V[1 * 3 + 1] - V[1 * 3 + 0] * V[0 * 3 + 1]};
    for (int r = 0; r < 3; ++r) V[r * 3 + 2] = v3[r];
}

/* Sampson denominator |Ex1|_xy^2 + |E'x2|_xy^2 and squared Sampson error of one correspondence (double). */
static double sampson_sq(const double* E, const double* p1, const double* p2, double* den_out) {
    const double a0 = fma(E[1], p1[1], fma(E[0], p1[0], E[2]));
    const double a1 = fma(E[4], p1[1], fma(E[3], p1[0], E[5]));
    const double a2 = fma(E[7], p1[1], fma(E[6], p1[0], E[8]));
    const double b0 = fma(E[3], p2[1], fma(E[0], p2[0], E[6]));
    const double b1 = fma(E[4], p2[1], fma(E[1], p2[0], E[7]));
    const double num = fma(p2[1], a1, fma(p2[0], a0, a2));
    const double den = fma(b1, b1, fma(b0, b0, fma(a1, a1, a0 * a0)));
    *den_out = den;
    return den > 0.0 ? num * num / den : 1e300;
}

/* Sum of 64 per-lane partial sums in the order of the device's wave reduction (gtsfm_amd/csrc/ransac.hip
 * wave_sum_f64): a Hillis-Steele scan inside each row of 16 lanes (lane i adds lane i - 1, i - 2, i - 4, i - 8 of its
 * row, or +0.0 past the row start), then rows 1 and 3 add lane 15 of the row below, rows 2 and 3 add lane 31; the
 * total is lane 63. Fixed order, so the CPU and the GPU round identically. */
static double wave_sum_order(const double* in) {
    double v[64], t[64];
    memcpy(v, in, sizeof(v));
    for (int n = 1; n <= 8; n <<= 1) {
        memcpy(t, v, sizeof(t));
        for (int i = 0; i < 64; ++i) v[i] = t[i] + ((i & 15) >= n ? t[i - n] : 0.0);
    }
    memcpy(t, v, sizeof(t));
    for (int i = 0; i < 64; ++i) {
        const int r = i >> 4;
        v[i] = t[i] + ((r == 1 || r == 3) ? t[16 * r - 1] : 0.0);
    }
    memcpy(t, v, sizeof(t));
    for (int i = 0; i < 64; ++i) v[i] = t[i] + ((i >> 4) >= 2 ? t[31] : 0.0);
    return v[63];
}

/* Sampson-weighted linear 8-point fit (rows scaled by 1/sqrt(den under E_w)) on the points whose squared Sampson
 * error under E_sel is <= th2, projected onto the essential manifold. Returns 0 if fewer than 8 points.
 * The 45 normal-matrix sums are formed as the device forms them (point i into partial sum i mod 64, in index order,
 * then wave_sum_order). The smallest eigenvector is found by shifted inverse iteration on the Cholesky factor
 * (shift 1e-12 trace, 8 iterations from the all-ones vector, the factor's diagonal stored as reciprocals), with the
 * cyclic Jacobi as the fallback when the factor breaks down; both are the device's operations in its order. */
static int refit_essential(const double* x1, const double* x2, int M, const double* E_sel, double th2,
                           const uint8_t* sel, const double* E_w, double* Eout) {
    static __thread double part[64][45];
    memset(part, 0, sizeof(part));
    int n = 0;
    for (int i = 0; i < M; ++i) {
        double den;
        if (sel ? !sel[i] : sampson_sq(E_sel, x1 + 2 * i, x2 + 2 * i, &den) > th2) continue;
        double dw;
        sampson_sq(E_w, x1 + 2 * i, x2 + 2 * i, &dw);
        const double w2 = dw > 1e-300 ? 1.0 / dw : 0.0;
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        const double r[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        double* acc = part[i & 63];
        int k = 0;
        for (int a = 0; a < 9; ++a) {
            const double wa = w2 * r[a];
            for (int b = a; b < 9; ++b, ++k) acc[k] = fma(wa, r[b], acc[k]);
        }
        ++n;
    }
    if (n < 8) return 0;
    double ata[45], col[64];
    for (int k = 0; k < 45; ++k) {
        for (int l = 0; l < 64; ++l) col[l] = part[l][k];
        ata[k] = wave_sum_order(col);
    }
#define ATA(i, j) ata[((i) < (j) ? (i) : (j)) * 9 - ((i) < (j) ? (i) : (j)) * (((i) < (j) ? (i) : (j)) - 1) / 2 + \
                      (((i) < (j) ? (j) : (i)) - ((i) < (j) ? (i) : (j)))]
    double E[9];
    double tr = 0.0;
    for (int i = 0; i < 9; ++i) tr += ATA(i, i);
    const double shift = 1e-12 * tr;
    double L[45]; /* packed lower triangle, row i at i (i + 1) / 2; the diagonal holds 1 / L_ii */
    int ok = tr > 0.0;
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j <= i; ++j) {
            double v = ATA(i, j) + (i == j ? shift : 0.0);
            for (int k = 0; k < j; ++k) v = fma(-L[i * (i + 1) / 2 + k], L[j * (j + 1) / 2 + k], v);
            if (i == j) {
                ok = ok && v > 0.0;
                L[i * (i + 1) / 2 + i] = 1.0 / sqrt(fmax(v, 1e-300));
            } else {
                L[i * (i + 1) / 2 + j] = v * L[j * (j + 1) / 2 + j];
            }
        }
    if (ok) {
        double x[9];
        for (int i = 0; i < 9; ++i) x[i] = 1.0;
        for (int it = 0; it < 8; ++it) {
            for (int i = 0; i < 9; ++i) { /* L y = x */
                double v = x[i];
                for (int k = 0; k < i; ++k) v = fma(-L[i * (i + 1) / 2 + k], x[k], v);
                x[i] = v * L[i * (i + 1) / 2 + i];
            }
            for (int i = 8; i >= 0; --i) { /* L^T z = y */
                double v = x[i];
                for (int k = i + 1; k < 9; ++k) v = fma(-L[k * (k + 1) / 2 + i], x[k], v);
                x[i] = v * L[i * (i + 1) / 2 + i];
            }
            double nrm = 0.0;
            for (int i = 0; i < 9; ++i) nrm = fma(x[i], x[i], nrm);
            nrm = 1.0 / sqrt(nrm);
            for (int i = 0; i < 9; ++i) x[i] *= nrm;
        }
        for (int k = 0; k < 9; ++k) E[k] = x[k];
    } else {
        double a[81], w[9], V[81];
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) a[i * 9 + j] = ATA(i, j);
        jacobi_eig(a, 9, w, V);
        int imin = 0;
        for (int i = 1; i < 9; ++i)
            if (w[i] < w[imin]) imin = i;
        for (int k = 0; k < 9; ++k) E[k] = V[k * 9 + imin];
    }
#undef ATA
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
    return 1;
}

/* ------------------------------------------------------------------ graph-cut labelling (GC-RANSAC LO) */
/* GC-RANSAC's local optimisation labels the points inlier / outlier by a minimum s-t cut of
 *   E(L) = (1 - lambda) sum_i D_i(L_i) + lambda sum_{i~j} V_ij(L_i, L_j)
 * (Barath & Matas, CVPR 2018; OpenCV USAC LOCAL_OPTIM_GC), here with the truncated quadratic of the MSAC term as
 * the data cost: with q_i the point's MSAC term (integer, Q = 65536 for an outlier), D_i(in) = q_i, D_i(out) = Q - q_i,
 * and the pairwise cost V(in, in) = (q_i + q_j) / 2, V(out, out) = Q - (q_i + q_j) / 2, V(in, out) = Q (submodular:
 * V(in,in) + V(out,out) = Q <= 2Q). Neighbours are the points sharing a cell of a 4-D grid over (x1, y1, x2, y2)
 * (cell side `cell` in normalised units), so the graph falls apart into one clique per cell and the minimum cut of
 * each clique is found exactly without a flow: for a fixed number m of inliers in a cell of k points the energy
 * only depends on which points through sum_S q with a positive coefficient, so the best S is the m points of lowest
 * q (ties: lower index), and 2 * E(m) is an integer evaluated for every m from prefix sums. The smallest m reaching
 * the minimum is taken (the minimal source set), so the labelling is unique and the kernel reproduces it bit for bit.
 * lambda = lam_num / lam_den. Returns the number of points labelled inlier. */
typedef struct {
    int64_t key;
    uint32_t q;
    int idx;
} gc_item;

static int gc_cmp(const void* a, const void* b) {
    const gc_item* x = (const gc_item*)a;
    const gc_item* y = (const gc_item*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    if (x->q != y->q) return x->q < y->q ? -1 : 1;
    return x->idx - y->idx;
}

/* 4-D grid cell of a correspondence: (x1, y1, x2, y2) / cell, floored, offset by 128 and kept to 8 bits each (exact
 * for |coordinate| < 127 cells: 6350 px at 50-px cells) */
static int64_t gc_cell_key(const float* p, double inv_cell) {
    uint32_t k = 0;
    for (int d = 0; d < 4; ++d) {
        const uint32_t c = (uint32_t)((int)floor((double)p[d] * inv_cell) + 128) & 0xFFu;
        k = (k << 8) | c;
    }
    return (int64_t)k;
}

/* The labelling of M points given their MSAC terms q and cell keys (exported for tests). */
int oracle_gc_label_q(const uint32_t* q, const int64_t* key, int M, int64_t lam_num, int64_t lam_den, uint8_t* lab) {
    const int64_t Q = 65536;
    gc_item* it = (gc_item*)malloc(sizeof(gc_item) * (size_t)(M > 0 ? M : 1));
    for (int i = 0; i < M; ++i) {
        it[i].q = q[i];
        it[i].key = key[i];
        it[i].idx = i;
        lab[i] = 0;
    }
    qsort(it, (size_t)M, sizeof(gc_item), gc_cmp);
    int n_in = 0;
    for (int a = 0; a < M;) {
        int b = a;
        int64_t sum = 0;
        while (b < M && it[b].key == it[a].key) sum += it[b++].q;
        const int64_t k = b - a;
        int64_t best = INT64_MAX, pre = 0;
        int best_m = 0;
        for (int64_t m = 0; m <= k; ++m) {  /* 2 E(m): m lowest-q points inliers, the other t outliers */
            if (m > 0) pre += it[a + m - 1].q;
            const int64_t t = k - m, post = sum - pre;
            const int64_t U = 2 * pre + 2 * (t * Q - post);
            const int64_t P = (m > 0 ? (m - 1) * pre : 0) + t * (t - 1) * Q - (t > 0 ? (t - 1) * post : 0) +
                              2 * m * t * Q;
            const int64_t e = (lam_den - lam_num) * U + lam_num * P;
            if (e < best) { best = e; best_m = (int)m; }
        }
        for (int m = 0; m < best_m; ++m) lab[it[a + m].idx] = 1;
        n_in += best_m;
        a = b;
    }
    free(it);
    return n_in;
}

static int gc_label(const double* Ed, const float* pts, int M, float thr2, double cell, int64_t lam_num,
                    int64_t lam_den, uint8_t* lab) {
    float E[9];
    for (int k = 0; k < 9; ++k) E[k] = (float)Ed[k];
    const float scale = 65536.0f / thr2;
    uint32_t* q = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(M > 0 ? M : 1));
    int64_t* key = (int64_t*)malloc(sizeof(int64_t) * (size_t)(M > 0 ? M : 1));
    const double inv_cell = 1.0 / cell;
    for (int i = 0; i < M; ++i) {
        int in;
        q[i] = msac_cost(E, pts[4 * i], pts[4 * i + 1], pts[4 * i + 2], pts[4 * i + 3], thr2, scale, &in);
        key[i] = gc_cell_key(pts + 4 * i, inv_cell);
    }
    const int n = oracle_gc_label_q(q, key, M, lam_num, lam_den, lab);
    free(q);
    free(key);
    return n;
}

/* ------------------------------------------------------------------ recoverPose */
static double det3(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

static int cheirality_count(const double* R, const double* t, const double* x1, const double* x2,
                            const uint8_t* mask, int M) {
    const double dist = 50.0;
    int good = 0;
    for (int i = 0; i < M; ++i) {
        if (mask && !mask[i]) continue;
        const double p[3] = {x1[2 * i], x1[2 * i + 1], 1.0};
        const double q[3] = {x2[2 * i], x2[2 * i + 1], 1.0};
        double a[3];
        for (int r = 0; r < 3; ++r) a[r] = R[r * 3 + 0] * p[0] + R[r * 3 + 1] * p[1] + R[r * 3 + 2] * p[2];
        /* min || l1 a - l2 q + t ||: [a, -q] [l1 l2]^T = -t */
        const double aa = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
        const double aq = a[0] * q[0] + a[1] * q[1] + a[2] * q[2];
        const double qq = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
        const double at = a[0] * t[0] + a[1] * t[1] + a[2] * t[2];
        const double qt = q[0] * t[0] + q[1] * t[1] + q[2] * t[2];
        const double det = aa * qq - aq * aq;
        if (fabs(det) < 1e-18) continue;
        const double l1 = (-at * qq + aq * qt) / det;
        const double z2 = l1 * a[2] + t[2];
        if (l1 > 0.0 && l1 < dist && z2 > 0.0 && z2 < dist) ++good;
    }
    return good;
}

/* E -> (R, t) with the cheirality vote over the masked points (OpenCV recoverPose order of preference). */
int oracle_recover_pose(const double* E, const double* x1, const double* x2, const uint8_t* mask, int M, double* R,
                        double* t) {
    double U[9], s[3], V[9];
    svd3(E, U, s, V);
    if (det3(U) < 0)
        for (int k = 0; k < 9; ++k) U[k] = -U[k];
    if (det3(V) < 0)
        for (int k = 0; k < 9; ++k) V[k] = -V[k];
    /* R1 = U W V^T, R2 = U W^T V^T with W = [[0,1,0],[-1,0,0],[0,0,1]]; t = U[:,2] */
    double R1[9], R2[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            /* (U W)[r][k]: W cols: col0 = (0,-1,0), col1 = (1,0,0), col2 = (0,0,1) */
            const double uw0 = -U[r * 3 + 1], uw1 = U[r * 3 + 0], uw2 = U[r * 3 + 2];
            const double uwt0 = U[r * 3 + 1], uwt1 = -U[r * 3 + 0], uwt2 = U[r * 3 + 2];
            R1[r * 3 + c] = uw0 * V[c * 3 + 0] + uw1 * V[c * 3 + 1] + uw2 * V[c * 3 + 2];
            R2[r * 3 + c] = uwt0 * V[c * 3 + 0] + uwt1 * V[c * 3 + 1] + uwt2 * V[c * 3 + 2];
        }
    const double tp[3] = {U[2], U[5], U[8]};
    const double tn[3] = {-U[2], -U[5], -U[8]};
    const int g1 = cheirality_count(R1, tp, x1, x2, mask, M);
    const int g2 = cheirality_count(R2, tp, x1, x2, mask, M);
    const int g3 = cheirality_count(R1, tn, x1, x2, mask, M);
    const int g4 = cheirality_count(R2, tn, x1, x2, mask, M);
    const double* Rs;
    const double* ts;
    int good;
    if (g1 >= g2 && g1 >= g3 && g1 >= g4) { Rs = R1; ts = tp; good = g1; }
    else if (g2 >= g1 && g2 >= g3 && g2 >= g4) { Rs = R2; ts = tp; good = g2; }
    else if (g3 >= g1 && g3 >= g2 && g3 >= g4) { Rs = R1; ts = tn; good = g3; }
    else { Rs = R2; ts = tn; good = g4; }
    memcpy(R, Rs, 9 * sizeof(double));
    memcpy(t, ts, 3 * sizeof(double));
    return good;
}

/* ------------------------------------------------------------------ RANSAC driver */
static int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmax(p, 0.0); p = fmin(p, 1.0);
    ep = fmax(ep, 0.0); ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - pow(1.0 - ep, (double)model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)lround(num / denom);
}

/*
 * Estimates E from M normalized correspondences (x1n, x2n: M x 2 double) with threshold `thr` (normalized units).
 * Outputs E (9), the inlier mask (M bytes), R (9), t (3). Returns the inlier count, or -1 when no model was found.
 * *n_hyp receives the number of hypotheses evaluated.
 */
int oracle_ransac_E_gc(const double* x1n, const double* x2n, int M, double thr, double prob, int max_iters,
                       uint64_t seed, int pair_id, int scoring, int gc_iters, double gc_cell, int gc_lam_num,
                       int gc_lam_den, double* E_out, uint8_t* mask_out, double* R_out, double* t_out, int* n_hyp) {
    init_tables();
    if (M < 6) return -1;
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)M);
    for (int i = 0; i < M; ++i) {
        pts[4 * i] = (float)x1n[2 * i];
        pts[4 * i + 1] = (float)x1n[2 * i + 1];
        pts[4 * i + 2] = (float)x2n[2 * i];
        pts[4 * i + 3] = (float)x2n[2 * i + 1];
    }
    const float thr2 = (float)(thr * thr);
    int best = -1, best_h = -1, best_s = -1;
    uint32_t best_score = 0xFFFFFFFFu;
    double bestE[9];
    int niters = max_iters, done = 0;
    while (done < niters) {
        for (int h = done; h < done + RANSAC_BATCH; ++h) {
            int idx[5];
            if (!oracle_sample5(seed, pair_id, h, M, idx)) continue;
            double s1[10], s2[10], Es[9 * MAX_SOL];
            for (int k = 0; k < 5; ++k) {
                s1[2 * k] = x1n[2 * idx[k]];
                s1[2 * k + 1] = x1n[2 * idx[k] + 1];
                s2[2 * k] = x2n[2 * idx[k]];
                s2[2 * k + 1] = x2n[2 * idx[k] + 1];
            }
            const int ns = oracle_five_point(s1, s2, Es);
            for (int s = 0; s < ns; ++s) {
                int c;
                if (scoring) {
                    const uint32_t sc = msac_score(Es + 9 * s, pts, M, thr2, &c, NULL);
                    if (sc >= best_score) continue;
                    best_score = sc;
                } else {
                    c = count_inliers(Es + 9 * s, pts, M, thr2, NULL);
                    if (c <= best) continue;
                }
                best = c;
                best_h = h;
                best_s = s;
                memcpy(bestE, Es + 9 * s, sizeof(bestE));
            }
        }
        done += RANSAC_BATCH;
        if (best > 0) {
            const int upd = update_num_iters(prob, (double)(M - best) / M, 5, niters);
            if (upd < niters) niters = upd;
        }
    }
    if (n_hyp) *n_hyp = done;
    (void)best_h;
    (void)best_s;
    if (best <= 0) {
        free(pts);
        return -1;
    }
    /* local optimisation (iterative LO): 4 steps with the selection threshold shrinking linearly from
     * LO_MULT*thr to thr; each step = 3 rounds of Sampson-weighted 8-point on the selected points; a refined
     * model replaces the best one when it has at least as many inliers at thr (RANSAC) / a score no higher (MSAC) */
    int cur = count_inliers(bestE, pts, M, thr2, NULL);
    uint32_t cur_score = 0;
    if (scoring) cur_score = msac_score(bestE, pts, M, thr2, &cur, NULL);
    const int gc_only = gc_iters < 0;  /* gc_iters < 0: the graph-cut LO replaces the iterative LO (USAC_ACCURATE) */
    if (gc_only) gc_iters = -gc_iters;
    if (!gc_only) {
        double E[9];
        memcpy(E, bestE, sizeof(E));
        for (int k = 0; k < LO_STEPS; ++k) {
            const double th = thr * (LO_MULT - (LO_MULT - 1.0) * k / (LO_STEPS - 1));
            double Esel[9], En[9];
            memcpy(Esel, E, sizeof(Esel));
            if (!refit_essential(x1n, x2n, M, Esel, th * th, NULL, Esel, En)) break;
            for (int r = 1; r < LO_IRLS; ++r) {
                double Et[9];
                if (!refit_essential(x1n, x2n, M, Esel, th * th, NULL, En, Et)) break;
                memcpy(En, Et, sizeof(En));
            }
            int c;
            int better;
            if (scoring) {
                const uint32_t sc = msac_score(En, pts, M, thr2, &c, NULL);
                better = sc <= cur_score;
                if (better) cur_score = sc;
            } else {
                c = count_inliers(En, pts, M, thr2, NULL);
                better = c >= cur;
            }
            memcpy(E, En, sizeof(E));
            if (better) {
                cur = c;
                memcpy(bestE, En, sizeof(bestE));
            }
        }
    }
    /* graph-cut LO (GC-RANSAC, MSAC only): label by the minimum cut under the best model, refit on the labelled
     * points (Sampson-weighted 8-point, LO_IRLS rounds), keep the refit while its MSAC score drops */
    if (gc_iters > 0 && scoring) {
        uint8_t* lab = (uint8_t*)malloc((size_t)M);
        for (int g = 0; g < gc_iters; ++g) {
            if (gc_label(bestE, pts, M, thr2, gc_cell, gc_lam_num, gc_lam_den, lab) < 8) break;
            double En[9];
            if (!refit_essential(x1n, x2n, M, NULL, 0.0, lab, bestE, En)) break;
            for (int r = 1; r < LO_IRLS; ++r) {
                double Et[9];
                if (!refit_essential(x1n, x2n, M, NULL, 0.0, lab, En, Et)) break;
                memcpy(En, Et, sizeof(En));
            }
            int c;
            const uint32_t sc = msac_score(En, pts, M, thr2, &c, NULL);
            if (sc >= cur_score) break;
            cur_score = sc;
            cur = c;
            memcpy(bestE, En, sizeof(bestE));
        }
        free(lab);
    }
    uint8_t* mask = mask_out;
    cur = count_inliers(bestE, pts, M, thr2, mask);
    memcpy(E_out, bestE, sizeof(bestE));
    oracle_recover_pose(bestE, x1n, x2n, mask, M, R_out, t_out);
    free(pts);
    return cur;
}

/* The verifier as the product runs it: MSAC with the graph-cut LO (GC-RANSAC) in place of the iterative LO;
 * inlier-count selection (RANSAC) with the iterative LO. */
int oracle_ransac_E(const double* x1n, const double* x2n, int M, double thr, double prob, int max_iters,
                    uint64_t seed, int pair_id, int scoring, double* E_out, uint8_t* mask_out, double* R_out,
                    double* t_out, int* n_hyp) {
    const int gc = scoring && M <= GC_MAX_M;
    return oracle_ransac_E_gc(x1n, x2n, M, thr, prob, max_iters, seed, pair_id, scoring, gc ? -GC_ITERS : 0,
                              GC_CELL_THR * thr, GC_LAM_NUM, GC_LAM_DEN, E_out, mask_out, R_out, t_out, n_hyp);
}

/* Squared Sampson distances of n correspondences under F (row-major 3x3) -- reference
 * gtsfm/utils/verification.py:170-214. precision 0: double (the reference's numpy arithmetic); 1: the float32 FMA
 * expression sampson_inlier() thresholds (num^2 / den evaluated from the same float terms). */
void oracle_sampson_sq(const double* F, const double* x1, const double* x2, int n, int precision, double* out) {
    for (int i = 0; i < n; ++i) {
        if (precision == 0) {
            double den;
            const double d = sampson_sq(F, x1 + 2 * i, x2 + 2 * i, &den);
            const double a0 = F[0] * x1[2 * i] + F[1] * x1[2 * i + 1] + F[2];
            const double a1 = F[3] * x1[2 * i] + F[4] * x1[2 * i + 1] + F[5];
            const double a2 = F[6] * x1[2 * i] + F[7] * x1[2 * i + 1] + F[8];
            const double num = x2[2 * i] * a0 + x2[2 * i + 1] * a1 + a2;
            out[i] = den > 0.0 ? d : num * num / den;
        } else {
            float E[9];
            for (int k = 0; k < 9; ++k) E[k] = (float)F[k];
            const float px = (float)x1[2 * i], py = (float)x1[2 * i + 1];
            const float pz = (float)x2[2 * i], pw = (float)x2[2 * i + 1];
            const float a0 = fmaf(E[1], py, fmaf(E[0], px, E[2]));
            const float a1 = fmaf(E[4], py, fmaf(E[3], px, E[5]));
            const float a2 = fmaf(E[7], py, fmaf(E[6], px, E[8]));
            const float b0 = fmaf(E[3], pw, fmaf(E[0], pz, E[6]));
            const float b1 = fmaf(E[4], pw, fmaf(E[1], pz, E[7]));
            const float num = fmaf(pw, a1, fmaf(pz, a0, a2));
            const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, a0 * a0)));
            out[i] = (double)(num * num) / (double)den;
        }
    }
}
