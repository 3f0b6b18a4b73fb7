/* ORACLE — test infrastructure only. CPU restatement of the reference's two-view triangulation + bundle adjustment
 * (gtsfm/two_view_estimator.py:101-208 bundle_adjust, :311-337 the run_2view branch that calls it).
 *
 * The reference hands the arithmetic to GTSAM 4.2 (environment_linux.yml:55; not in this image):
 *   - gtsam.triangulatePoint3(cameras, measurements, rank_tol=1e-9, optimize=True) per verified correspondence
 *     (data_association/point3d_initializer.py:225-290, TriangulationSamplingMode.NO_RANSAC,
 *     reproj_error_threshold 100 from sift_front_end.yaml): linear DLT (SVD null vector of the 4x4 system, rank >= 3)
 *     -> Levenberg-Marquardt refinement of the point on two TriangulationFactors (unit noise; GTSAM's
 *     triangulation.h optimize(): lambdaInitial 1, lambdaFactor 10, maxIterations 100, absoluteErrorTol 1.0)
 *     -> cheirality (point in front of both cameras) and per-measurement reprojection error < 100 px.
 *   - BundleAdjustmentOptimizer.run_ba (bundle/bundle_adjustment.py:119-419) on that 2-view scene: poses X0 (the i1
 *     camera, identity) and X1 (= i2Ti1^-1), one Point3 per track, GeneralSFMFactor2 reprojection factors with a
 *     Huber(1.345) robust model on sigma 1 px, PriorFactorPose3 on X0 (sigma 0.1) and PriorFactorPoint3 on the first
 *     track (sigma 0.1); gtsam.LevenbergMarquardtOptimizer with default parameters and maxIterations 100
 *     (bundle_adjust_2view_maxiters); then filter_landmarks(0.5 px) (common/gtsfm_data.py:389-427).
 *   The calibrations, which the reference keeps as variables under a sigma 1e-5 prior (bundle_adjustment.py:89),
 *   are held fixed here (k1 = k2 = 0 on this path; the prior pins them to ~1e-10 relative).
 *
 * GTSAM's Levenberg-Marquardt loop is restated from its published algorithm (LevenbergMarquardtOptimizer::tryLambda /
 * iterate, NonlinearOptimizer::defaultOptimize, checkConvergence): isotropic damping lambda * I on every variable,
 * model fidelity = nonlinear cost change / linearized cost change > 1e-3 accepts a step and divides lambda by 10,
 * otherwise lambda *= 10 until 1e5; convergence when the error decrease is <= relativeErrorTol * error or <=
 * absoluteErrorTol. Poses retract as X * Exp(xi), xi = (omega, v) (GTSAM_POSE3_EXPMAP). The linear system is solved
 * through the Schur complement on the points (12 x 12 Cholesky), the same solution GTSAM's elimination computes.
 * Parity to GTSAM itself is unpinned (the library is absent); the reference's own 2-view test (5pointExample1,
 * tests/test_two_view_estimator.py:52-94, <= 1 degree) needs GTSAM's example data and is restated on synthetic scenes.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double R[9]; /* wRc row-major */
    double t[3]; /* wtc */
} pose_t;

#define HUBER_K 1.345
#define BA_PI 3.14159265358979323846
#define LM_MIN_FIDELITY 1e-3
#define LM_LAMBDA_UPPER 1e5

static void skew3(const double* w, double* S) {
    S[0] = 0; S[1] = -w[2]; S[2] = w[1];
    S[3] = w[2]; S[4] = 0; S[5] = -w[0];
    S[6] = -w[1]; S[7] = w[0]; S[8] = 0;
}

static void mm3(const double* A, const double* B, double* C) { /* C = A B */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

static void mtv3(const double* A, const double* v, double* o) { /* o = A^T v */
    for (int j = 0; j < 3; ++j) o[j] = A[j] * v[0] + A[3 + j] * v[1] + A[6 + j] * v[2];
}

static void mv3(const double* A, const double* v, double* o) {
    for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}

/* Rot3::Expmap (Rodrigues) */
static void so3_exp(const double* w, double* R) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double W[9], W2[9];
    skew3(w, W);
    mm3(W, W, W2);
    double a, b;
    if (th2 < 1e-16) {
        a = 1.0 - th2 / 6.0;
        b = 0.5 - th2 / 24.0;
    } else {
        const double th = sqrt(th2);
        a = sin(th) / th;
        b = (1.0 - cos(th)) / th2;
    }
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * W[k] + b * W2[k];
}

/* Rot3::Logmap */
static void so3_log(const double* R, double* w) {
    const double tr = R[0] + R[4] + R[8];
    double c = 0.5 * (tr - 1.0);
    if (c > 1.0) c = 1.0;
    if (c < -1.0) c = -1.0;
    const double th = acos(c);
    const double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (th < 1e-8) {
        for (int k = 0; k < 3; ++k) w[k] = 0.5 * v[k];
    } else if (BA_PI - th < 1e-6) {
        /* near pi: axis from the diagonal */
        int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        double ax[3];
        ax[i] = sqrt(fmax(0.0, (R[4 * i] + 1.0) * 0.5));
        for (int j = 0; j < 3; ++j)
            if (j != i) ax[j] = (R[3 * i + j] + R[3 * j + i]) / (4.0 * ax[i]);
        const double n = sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
        for (int k = 0; k < 3; ++k) w[k] = th * ax[k] / n;
    } else {
        const double s = th / (2.0 * sin(th));
        for (int k = 0; k < 3; ++k) w[k] = s * v[k];
    }
}

/* X * Exp(xi), xi = (omega, v): R' = R Exp(omega), t' = t + R (Jl(omega) v) */
static void pose_retract(const pose_t* X, const double* xi, pose_t* out) {
    double dR[9], tv[3];
    so3_exp(xi, dR);
    const double* w = xi;
    const double* v = xi + 3;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double W[9], W2[9];
    skew3(w, W);
    mm3(W, W, W2);
    double a, b;
    if (th2 < 1e-16) {
        a = 0.5 - th2 / 24.0;
        b = 1.0 / 6.0 - th2 / 120.0;
    } else {
        const double th = sqrt(th2);
        a = (1.0 - cos(th)) / th2;
        b = (th - sin(th)) / (th2 * th);
    }
    for (int i = 0; i < 3; ++i)
        tv[i] = v[i] + a * (W[3 * i] * v[0] + W[3 * i + 1] * v[1] + W[3 * i + 2] * v[2]) +
                b * (W2[3 * i] * v[0] + W2[3 * i + 1] * v[1] + W2[3 * i + 2] * v[2]);
    pose_t o;
    mm3(X->R, dR, o.R);
    double Rt[3];
    mv3(X->R, tv, Rt);
    for (int i = 0; i < 3; ++i) o.t[i] = X->t[i] + Rt[i];
    *out = o;
}

/* Pose3::Logmap of T (GTSAM_POSE3_EXPMAP) */
static void pose_log(const pose_t* T, double* xi) {
    double w[3];
    so3_log(T->R, w);
    const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    xi[0] = w[0]; xi[1] = w[1]; xi[2] = w[2];
    if (th < 1e-10) {
        for (int k = 0; k < 3; ++k) xi[3 + k] = T->t[k];
        return;
    }
    double W[9], Wt[3], WWt[3];
    const double wn[3] = {w[0] / th, w[1] / th, w[2] / th};
    skew3(wn, W);
    mv3(W, T->t, Wt);
    mv3(W, Wt, WWt);
    const double tn = tan(0.5 * th);
    for (int k = 0; k < 3; ++k) xi[3 + k] = T->t[k] - (0.5 * th) * Wt[k] + (1.0 - th / (2.0 * tn)) * WWt[k];
}

/* ------------------------------------------------------------------ relative-pose prior
 * BetweenFactorPose3(X0, X1, m, Diagonal.Sigmas(sigmas)) with m = i2Ti1_prior.value.inverse()
 * (bundle_adjustment.py:136-152; two_view_estimator.py:165,192 passes the prior). GTSAM's error is
 * e = Pose3::Logmap(m^-1 * X0^-1 * X1) (Local of the Expmap chart), whitened by 1 / sigma. With X_c <- X_c Exp(d_c):
 * de/dd1 = Jr^-1(e), de/dd0 = -Jr^-1(e) Ad(hx^-1), hx = X0^-1 X1, with the closed-form Jr^-1 of se3_jr_inv
 * (GTSAM's BetweenFactor H1/H2 through Pose3::LogmapDerivative); Ad((R, t)) = [[R, 0], [t^ R, R]]. */
typedef struct {
    int on;
    pose_t minv;    /* m^-1 = i2Ti1_prior (the prior's value itself) */
    double isig[6]; /* 1 / sigma, GTSAM tangent order (rotation, translation) */
} between_t;

static void pose_mul(const pose_t* A, const pose_t* B, pose_t* C) {
    pose_t o;
    mm3(A->R, B->R, o.R);
    mv3(A->R, B->t, o.t);
    for (int k = 0; k < 3; ++k) o.t[k] += A->t[k];
    *C = o;
}

static void pose_inv(const pose_t* A, pose_t* C) {
    pose_t o;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o.R[3 * i + j] = A->R[3 * j + i];
    mtv3(A->R, A->t, o.t);
    for (int k = 0; k < 3; ++k) o.t[k] = -o.t[k];
    *C = o;
}

/* unwhitened residual e (6) and hx = X0^-1 X1 */
static void between_residual(const between_t* f, const pose_t* X, double* e, pose_t* hx) {
    pose_t x0i, E0;
    pose_inv(&X[0], &x0i);
    pose_mul(&x0i, &X[1], hx);
    pose_mul(&f->minv, hx, &E0);
    pose_log(&E0, e);
}

static double between_error(const between_t* f, const pose_t* X) {
    if (!f->on) return 0.0;
    double e[6];
    pose_t hx;
    between_residual(f, X, e, &hx);
    double s = 0;
    for (int k = 0; k < 6; ++k) s += (e[k] * f->isig[k]) * (e[k] * f->isig[k]);
    return 0.5 * s;
}

/* exact inverse right Jacobian of SE(3) at e = (w, v), rotation first (GTSAM Pose3::LogmapDerivative):
 * Jr(e) = [[Jw, 0], [Q, Jw]] so Jr^-1 = [[A, 0], [-A Q A, A]] with A = Jw^-1 = I + W/2 + c W^2,
 * c = 1/th^2 - 1/(2 th tan(th/2)), and Q the right-Jacobian coupling block (Barfoot & Furgale 2014, eq. 102,
 * evaluated at -e): Q = -P/2 + c1 (WP + PW - WPW) - c2 (WWP + PWW - 3 WPW) + c3 (WPWW + WWPW), W = w^, P = v^,
 * c1 = (th - sin th) / th^3, c2 = (th^2 + 2 cos th - 2) / (2 th^4), c3 = (2 th - 3 sin th + th cos th) / (2 th^5);
 * below th = 1e-2 the coefficients use their Taylor series to th^2. */
static void se3_jr_inv(const double* e, double* Ji) {
    const double* w = e;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double c, c1, c2, c3;
    if (th2 < 1e-4) {
        c = 1.0 / 12.0 + th2 / 720.0;
        c1 = 1.0 / 6.0 - th2 / 120.0;
        c2 = 1.0 / 24.0 - th2 / 720.0;
        c3 = 1.0 / 120.0 - th2 / 2520.0;
    } else {
        const double th = sqrt(th2), s = sin(th), co = cos(th);
        c = 1.0 / th2 - 1.0 / (2.0 * th * tan(0.5 * th));
        c1 = (th - s) / (th2 * th);
        c2 = (th2 + 2.0 * co - 2.0) / (2.0 * th2 * th2);
        c3 = (2.0 * th - 3.0 * s + th * co) / (2.0 * th2 * th2 * th);
    }
    double W[9], P[9], W2[9], WP[9], PW[9], WPW[9], W2P[9], PW2[9], WPW2[9], W2PW[9], A[9], Q[9], AQ[9], B[9];
    skew3(w, W);
    skew3(e + 3, P);
    mm3(W, W, W2);
    mm3(W, P, WP);
    mm3(P, W, PW);
    mm3(WP, W, WPW);
    mm3(W, WP, W2P);
    mm3(PW, W, PW2);
    mm3(WPW, W, WPW2);
    mm3(W, WPW, W2PW);
    for (int k = 0; k < 9; ++k) {
        A[k] = (k % 4 == 0 ? 1.0 : 0.0) + 0.5 * W[k] + c * W2[k];
        Q[k] = -0.5 * P[k] + c1 * (WP[k] + PW[k] - WPW[k]) - c2 * (W2P[k] + PW2[k] - 3.0 * WPW[k]) +
               c3 * (WPW2[k] + W2PW[k]);
    }
    mm3(A, Q, AQ);
    mm3(AQ, A, B);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Ji[6 * i + j] = A[3 * i + j];
            Ji[6 * i + 3 + j] = 0.0;
            Ji[6 * (3 + i) + j] = -B[3 * i + j];
            Ji[6 * (3 + i) + 3 + j] = A[3 * i + j];
        }
}

/* whitened residual r (6) and Jacobian J (6 x 12, columns: X0 then X1) at X */
static void between_linearize(const between_t* f, const pose_t* X, double* r, double* J) {
    double e[6];
    pose_t hx, hi;
    between_residual(f, X, e, &hx);
    double Ji[36], Ad[36];
    se3_jr_inv(e, Ji);
    pose_inv(&hx, &hi);
    memset(Ad, 0, sizeof(Ad));
    double T[9], TR[9];
    skew3(hi.t, T);
    mm3(T, hi.R, TR);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Ad[6 * i + j] = hi.R[3 * i + j];
            Ad[6 * (3 + i) + 3 + j] = hi.R[3 * i + j];
            Ad[6 * (3 + i) + j] = TR[3 * i + j];
        }
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) {
            double a = 0;
            for (int k = 0; k < 6; ++k) a += Ji[6 * i + k] * Ad[6 * k + j];
            J[12 * i + j] = -a * f->isig[i];
            J[12 * i + 6 + j] = Ji[6 * i + j] * f->isig[i];
        }
        r[i] = e[i] * f->isig[i];
    }
}

/* camera (pose X, calibration f,u0,v0, k1 = k2 = 0) projection; 0 on cheirality failure (z <= 0) */
static int project(const pose_t* X, const double* K, const double* p, double* pc, double* uv) {
    const double d[3] = {p[0] - X->t[0], p[1] - X->t[1], p[2] - X->t[2]};
    mtv3(X->R, d, pc);
    if (pc[2] <= 0.0) return 0;
    const double xn = pc[0] / pc[2], yn = pc[1] / pc[2];
    uv[0] = K[1] + K[0] * xn;
    uv[1] = K[2] + K[0] * yn;
    return 1;
}

/* Jacobians of uv w.r.t. the point (2x3) and the pose (2x6, right perturbation (omega, v)) at pc */
static void project_jac(const pose_t* X, const double* K, const double* pc, double* Jp, double* Jx) {
    const double iz = 1.0 / pc[2], xn = pc[0] * iz, yn = pc[1] * iz, f = K[0];
    const double D[6] = {f * iz, 0.0, -f * xn * iz, 0.0, f * iz, -f * yn * iz}; /* duv / dpc */
    /* dpc/dp = R^T ; dpc/domega = [pc]x ; dpc/dv = -I */
    for (int r = 0; r < 2; ++r) {
        for (int j = 0; j < 3; ++j)
            Jp[3 * r + j] = D[3 * r] * X->R[3 * j] + D[3 * r + 1] * X->R[3 * j + 1] + D[3 * r + 2] * X->R[3 * j + 2];
        const double* d = D + 3 * r;
        /* [pc]x rows: (0,-z,y), (z,0,-x), (-y,x,0); d^T [pc]x */
        Jx[6 * r + 0] = d[1] * pc[2] - d[2] * pc[1];
        Jx[6 * r + 1] = -d[0] * pc[2] + d[2] * pc[0];
        Jx[6 * r + 2] = d[0] * pc[1] - d[1] * pc[0];
        Jx[6 * r + 3] = -d[0];
        Jx[6 * r + 4] = -d[1];
        Jx[6 * r + 5] = -d[2];
    }
}

static double huber_loss(double d) { return d <= HUBER_K ? 0.5 * d * d : HUBER_K * d - 0.5 * HUBER_K * HUBER_K; }
static double huber_weight(double d) { return d <= HUBER_K ? 1.0 : HUBER_K / d; }

/* Cholesky solve of an n x n SPD system (row-major a, overwritten); 0 if not positive definite */
static int chol_solve(double* a, double* b, int n) {
    for (int j = 0; j < n; ++j) {
        double s = a[j * n + j];
        for (int k = 0; k < j; ++k) s -= a[j * n + k] * a[j * n + k];
        if (!(s > 0.0)) return 0;
        const double d = sqrt(s);
        a[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double v = a[i * n + j];
            for (int k = 0; k < j; ++k) v -= a[i * n + k] * a[j * n + k];
            a[i * n + j] = v / d;
        }
    }
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= a[i * n + k] * b[k];
        b[i] = v / a[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < n; ++k) v -= a[k * n + i] * b[k];
        b[i] = v / a[i * n + i];
    }
    return 1;
}

/* symmetric 3x3 inverse; 0 if singular */
static int inv3_sym(const double* A, double* I) {
    const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    if (!(fabs(det) > 0.0) || !isfinite(det)) return 0;
    const double id = 1.0 / det;
    I[0] = c00 * id;
    I[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    I[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    I[3] = c01 * id;
    I[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    I[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    I[6] = c02 * id;
    I[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    I[8] = (A[0] * A[4] - A[1] * A[3]) * id;
    return 1;
}

/* ------------------------------------------------------------------ triangulation (triangulatePoint3) */

/* null vector of the 4x4 DLT system by one-sided Jacobi SVD; returns the rank (singular values > rank_tol) */
static int dlt_null_vector(const double* A_in, double rank_tol, double* v_out) {
    double U[16], V[16];
    memcpy(U, A_in, sizeof(U));
    for (int k = 0; k < 16; ++k) V[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 4; ++i) {
                    al += U[4 * i + p] * U[4 * i + p];
                    be += U[4 * i + q] * U[4 * i + q];
                    ga += U[4 * i + p] * U[4 * i + q];
                }
                if (fabs(ga) <= 1e-15 * sqrt(al * be) || ga == 0.0) continue;
                rotated = 1;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 4; ++i) {
                    const double up = U[4 * i + p], uq = U[4 * i + q];
                    U[4 * i + p] = c * up - s * uq;
                    U[4 * i + q] = s * up + c * uq;
                    const double vp = V[4 * i + p], vq = V[4 * i + q];
                    V[4 * i + p] = c * vp - s * vq;
                    V[4 * i + q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    int rank = 0, jmin = 0;
    double smin = INFINITY;
    for (int j = 0; j < 4; ++j) {
        double s = 0;
        for (int i = 0; i < 4; ++i) s += U[4 * i + j] * U[4 * i + j];
        s = sqrt(s);
        if (s > rank_tol) ++rank;
        if (s < smin) { smin = s; jmin = j; }
    }
    for (int i = 0; i < 4; ++i) v_out[i] = V[4 * i + jmin];
    return rank;
}

/* TriangulationFactor error of one camera: projection - measured, or (2f, 2f) on cheirality failure (Jacobian 0) */
static double tri_factor(const pose_t* X, const double* K, const double* p, const double* uv, double* e, double* Jp) {
    double pc[3], pr[2], Jx[12];
    if (!project(X, K, p, pc, pr)) {
        e[0] = e[1] = 2.0 * K[0];
        memset(Jp, 0, 6 * sizeof(double));
    } else {
        e[0] = pr[0] - uv[0];
        e[1] = pr[1] - uv[1];
        project_jac(X, K, pc, Jp, Jx);
    }
    return 0.5 * (e[0] * e[0] + e[1] * e[1]);
}

/* gtsam::triangulatePoint3(cameras, measurements, 1e-9, optimize=true) + the reference's checks; 1 = track kept */
int oracle_triangulate2(const pose_t* X0, const pose_t* X1, const double* K1, const double* K2, const double* uv1,
                        const double* uv2, double tri_thresh, double* p_out) {
    const pose_t* X[2] = {X0, X1};
    const double* K[2] = {K1, K2};
    const double* uv[2] = {uv1, uv2};
    double A[16];
    for (int c = 0; c < 2; ++c) {
        /* P = K [R^T | -R^T t] */
        double P[12];
        for (int r = 0; r < 3; ++r) {
            const double* Rc = X[c]->R;
            const double row[3] = {Rc[r], Rc[3 + r], Rc[6 + r]}; /* row r of R^T */
            const double tr = -(row[0] * X[c]->t[0] + row[1] * X[c]->t[1] + row[2] * X[c]->t[2]);
            P[4 * r + 0] = row[0]; P[4 * r + 1] = row[1]; P[4 * r + 2] = row[2]; P[4 * r + 3] = tr;
        }
        double KP[12];
        for (int j = 0; j < 4; ++j) {
            KP[j] = K[c][0] * P[j] + K[c][1] * P[8 + j];
            KP[4 + j] = K[c][0] * P[4 + j] + K[c][2] * P[8 + j];
            KP[8 + j] = P[8 + j];
        }
        for (int j = 0; j < 4; ++j) {
            A[4 * (2 * c) + j] = uv[c][0] * KP[8 + j] - KP[j];
            A[4 * (2 * c + 1) + j] = uv[c][1] * KP[8 + j] - KP[4 + j];
        }
    }
    double v[4];
    if (dlt_null_vector(A, 1e-9, v) < 3) return 0; /* TriangulationUnderconstrainedException */
    double p[3] = {v[0] / v[3], v[1] / v[3], v[2] / v[3]};
    /* triangulateNonlinear: LM on the point, lambdaInitial 1, factor 10, maxIterations 100, absoluteErrorTol 1 */
    double e[2], J[6], err = 0;
    for (int c = 0; c < 2; ++c) err += tri_factor(X[c], K[c], p, uv[c], e, J);
    double lambda = 1.0;
    int iters = 0;
    if (isfinite(err) && err > 0.0) {
        for (;;) {
            const double cur = err;
            /* linearize */
            double H[9] = {0}, g[3] = {0}, bb = 0;
            double Js[2][6], es[2][2];
            for (int c = 0; c < 2; ++c) {
                tri_factor(X[c], K[c], p, uv[c], es[c], Js[c]);
                for (int r = 0; r < 2; ++r) {
                    for (int i = 0; i < 3; ++i) {
                        g[i] += Js[c][3 * r + i] * (-es[c][r]);
                        for (int j = 0; j < 3; ++j) H[3 * i + j] += Js[c][3 * r + i] * Js[c][3 * r + j];
                    }
                    bb += es[c][r] * es[c][r];
                }
            }
            for (;;) {
                double Hd[9], d[3] = {g[0], g[1], g[2]};
                memcpy(Hd, H, sizeof(Hd));
                for (int i = 0; i < 3; ++i) Hd[4 * i] += lambda;
                int success = 0, stop = 0;
                double newp[3], newErr = INFINITY;
                if (chol_solve(Hd, d, 3)) {
                    double nl = 0;
                    for (int c = 0; c < 2; ++c)
                        for (int r = 0; r < 2; ++r) {
                            const double a = Js[c][3 * r] * d[0] + Js[c][3 * r + 1] * d[1] + Js[c][3 * r + 2] * d[2];
                            const double rr = a + es[c][r];
                            nl += rr * rr;
                        }
                    const double oldLin = 0.5 * bb, newLin = 0.5 * nl, linChange = oldLin - newLin;
                    if (linChange >= 0) {
                        for (int i = 0; i < 3; ++i) newp[i] = p[i] + d[i];
                        newErr = 0;
                        for (int c = 0; c < 2; ++c) newErr += tri_factor(X[c], K[c], newp, uv[c], e, J);
                        const double costChange = err - newErr;
                        if (linChange > DBL_EPSILON * oldLin) success = costChange / linChange > LM_MIN_FIDELITY;
                        else success = 1;
                        if (fabs(costChange) < 1e-5 * err) stop = 1;
                    }
                }
                if (success) {
                    memcpy(p, newp, sizeof(p));
                    err = newErr;
                    lambda /= 10.0;
                    ++iters;
                    break;
                }
                if (stop) break;
                lambda *= 10.0;
                if (lambda >= LM_LAMBDA_UPPER) break;
            }
            const double dec = cur - err;
            if (iters >= 100 || dec / cur <= 1e-5 || dec <= 1.0 || !isfinite(cur)) break;
        }
    }
    /* cheirality (GTSAM_THROW_CHEIRALITY_EXCEPTION) and the reprojection threshold */
    for (int c = 0; c < 2; ++c) {
        double pc[3], pr[2];
        if (!project(X[c], K[c], p, pc, pr)) return 0;
        const double dx = pr[0] - uv[c][0], dy = pr[1] - uv[c][1];
        if (!(sqrt(dx * dx + dy * dy) < tri_thresh)) return 0;
    }
    memcpy(p_out, p, sizeof(p));
    return 1;
}

/* ------------------------------------------------------------------ bundle adjustment */

/* total nonlinear error: Huber reprojection losses + X0 prior + P0 prior */
static double ba_error(const pose_t* X, const double* K1, const double* K2, const double* P, const double* uv1,
                       const double* uv2, int n, const double* P0_prior, const between_t* bf) {
    const double* K[2] = {K1, K2};
    double err = 0;
    for (int j = 0; j < n; ++j) {
        for (int c = 0; c < 2; ++c) {
            double pc[3], pr[2];
            if (!project(&X[c], K[c], P + 3 * j, pc, pr)) continue; /* GeneralSFMFactor: zero error */
            const double* uv = c ? uv2 + 2 * j : uv1 + 2 * j;
            const double dx = pr[0] - uv[0], dy = pr[1] - uv[1];
            err += huber_loss(sqrt(dx * dx + dy * dy));
        }
    }
    double xi[6];
    pose_log(&X[0], xi); /* prior is the identity */
    double s = 0;
    for (int k = 0; k < 6; ++k) s += xi[k] * xi[k];
    err += 0.5 * s / 0.01;
    s = 0;
    for (int k = 0; k < 3; ++k) s += (P[k] - P0_prior[k]) * (P[k] - P0_prior[k]);
    err += 0.5 * s / 0.01;
    return err + between_error(bf, X);
}

/* one point's whitened, Huber-reweighted factor blocks at the current values */
typedef struct {
    double Jx[2][12]; /* [camera][2x6] */
    double Jp[2][6];  /* [camera][2x3] */
    double b[2][2];   /* -sqrt(w) e */
    int ok[2];
} pt_lin_t;

static void linearize_point(const pose_t* X, const double* K1, const double* K2, const double* p, const double* uv1,
                            const double* uv2, pt_lin_t* L) {
    const double* K[2] = {K1, K2};
    const double* uv[2] = {uv1, uv2};
    for (int c = 0; c < 2; ++c) {
        double pc[3], pr[2];
        L->ok[c] = project(&X[c], K[c], p, pc, pr);
        if (!L->ok[c]) {
            memset(L->Jx[c], 0, sizeof(L->Jx[c]));
            memset(L->Jp[c], 0, sizeof(L->Jp[c]));
            L->b[c][0] = L->b[c][1] = 0;
            continue;
        }
        project_jac(&X[c], K[c], pc, L->Jp[c], L->Jx[c]);
        const double e0 = pr[0] - uv[c][0], e1 = pr[1] - uv[c][1];
        const double sw = sqrt(huber_weight(sqrt(e0 * e0 + e1 * e1)));
        for (int k = 0; k < 12; ++k) L->Jx[c][k] *= sw;
        for (int k = 0; k < 6; ++k) L->Jp[c][k] *= sw;
        L->b[c][0] = -sw * e0;
        L->b[c][1] = -sw * e1;
    }
}

/* Returns 0 (BA ran, >= 1 valid track), 1 (no triangulated track), 2 (no track valid after the 0.5 px filter).
 * R_in / t_in: i2Ri1 and the unit i2ti1 of the verifier. R_out / t_out: i2Ri1 and unit i2ti1 after BA (the input
 * pose for statuses 1 and 2). valid[j]: correspondence j survives triangulation + BA + filtering. */
/* test hook: the between factor (prior value prior_Rt = [R | t] row-major 3x4, isig 6) at cameras X = [R0 | t0, R1 | t1]
 * (2 x 12) each retracted by d (12, may be NULL): whitened residual r (6) and, when J != NULL, its Jacobian (6 x 12) */
void oracle_between_eval(const double* prior_Rt, const double* isig, const double* Xrt, const double* d, double* r,
                         double* J) {
    between_t f;
    f.on = 1;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) f.minv.R[3 * i + j] = prior_Rt[4 * i + j];
        f.minv.t[i] = prior_Rt[4 * i + 3];
    }
    for (int k = 0; k < 6; ++k) f.isig[k] = isig[k];
    pose_t X[2];
    for (int c = 0; c < 2; ++c) {
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) X[c].R[3 * i + j] = Xrt[12 * c + 4 * i + j];
            X[c].t[i] = Xrt[12 * c + 4 * i + 3];
        }
        if (d) pose_retract(&X[c], d + 6 * c, &X[c]);
    }
    if (J) {
        between_linearize(&f, X, r, J);
    } else {
        double e[6];
        pose_t hx;
        between_residual(&f, X, e, &hx);
        for (int k = 0; k < 6; ++k) r[k] = e[k] * f.isig[k];
    }
}

int oracle_ba2(const double* uv1, const double* uv2, int n, const double* K1, const double* K2, const double* R_in,
               const double* t_in, int max_iters, double reproj_thresh, double tri_thresh, const double* prior_Rt,
               const double* prior_sigmas, double* R_out, double* t_out, uint8_t* valid, int* iters_out,
               double* error_out) {
    memcpy(R_out, R_in, 9 * sizeof(double));
    memcpy(t_out, t_in, 3 * sizeof(double));
    memset(valid, 0, (size_t)n);
    if (iters_out) *iters_out = 0;
    /* relative-pose prior i2Ti1_prior = (R, t) (prior_Rt: R row-major then t; NULL = none): it initialises the
     * second camera instead of the verifier's pose (two_view_estimator.py:165-171) and adds the between factor */
    between_t bf;
    memset(&bf, 0, sizeof(bf));
    const double* Ri = R_in;
    const double* ti = t_in;
    if (prior_Rt && prior_sigmas) {
        bf.on = 1;
        memcpy(bf.minv.R, prior_Rt, 9 * sizeof(double));
        memcpy(bf.minv.t, prior_Rt + 9, 3 * sizeof(double));
        for (int k = 0; k < 6; ++k) bf.isig[k] = 1.0 / prior_sigmas[k];
        Ri = prior_Rt;
        ti = prior_Rt + 9;
        /* no track: the reference returns the initial pose, i.e. the prior's (two_view_estimator.py:186-187) */
        memcpy(R_out, Ri, 9 * sizeof(double));
        const double nt = sqrt(ti[0] * ti[0] + ti[1] * ti[1] + ti[2] * ti[2]);
        for (int k = 0; k < 3; ++k) t_out[k] = ti[k] / nt;
    }
    pose_t X[2];
    memset(&X[0], 0, sizeof(pose_t));
    X[0].R[0] = X[0].R[4] = X[0].R[8] = 1.0;
    /* X1 = i2Ti1^-1: R^T, -R^T t */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) X[1].R[3 * i + j] = Ri[3 * j + i];
    mtv3(Ri, ti, X[1].t);
    for (int i = 0; i < 3; ++i) X[1].t[i] = -X[1].t[i];
    /* triangulate every correspondence */
    int* tri = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    double* P = (double*)malloc(sizeof(double) * 3 * (size_t)(n > 0 ? n : 1));
    double* u1 = (double*)malloc(sizeof(double) * 2 * (size_t)(n > 0 ? n : 1));
    double* u2 = (double*)malloc(sizeof(double) * 2 * (size_t)(n > 0 ? n : 1));
    int m = 0;
    for (int j = 0; j < n; ++j) {
        if (oracle_triangulate2(&X[0], &X[1], K1, K2, uv1 + 2 * j, uv2 + 2 * j, tri_thresh, P + 3 * m)) {
            tri[m] = j;
            memcpy(u1 + 2 * m, uv1 + 2 * j, 2 * sizeof(double));
            memcpy(u2 + 2 * m, uv2 + 2 * j, 2 * sizeof(double));
            ++m;
        }
    }
    if (m == 0) {
        free(tri); free(P); free(u1); free(u2);
        return 1;
    }
    const double P0_prior[3] = {P[0], P[1], P[2]};
    double* Pn = (double*)malloc(sizeof(double) * 3 * (size_t)m);
    pt_lin_t* lin = (pt_lin_t*)malloc(sizeof(pt_lin_t) * (size_t)m);
    double err = ba_error(X, K1, K2, P, u1, u2, m, P0_prior, &bf);
    double lambda = 1e-5;
    int iters = 0;
    if (err > 0.0) {
        for (;;) {
            const double cur = err;
            /* linearize at the current values */
            for (int j = 0; j < m; ++j) linearize_point(X, K1, K2, P + 3 * j, u1 + 2 * j, u2 + 2 * j, &lin[j]);
            double xi0[6];
            pose_log(&X[0], xi0);
            double oldLin = 0;
            for (int j = 0; j < m; ++j)
                for (int c = 0; c < 2; ++c) oldLin += lin[j].b[c][0] * lin[j].b[c][0] + lin[j].b[c][1] * lin[j].b[c][1];
            for (int k = 0; k < 6; ++k) oldLin += xi0[k] * xi0[k] / 0.01;
            for (int k = 0; k < 3; ++k) oldLin += (P[k] - P0_prior[k]) * (P[k] - P0_prior[k]) / 0.01;
            double br[6] = {0, 0, 0, 0, 0, 0}, bJ[72];
            if (bf.on) {
                between_linearize(&bf, X, br, bJ);
                for (int k = 0; k < 6; ++k) oldLin += br[k] * br[k];
            }
            oldLin *= 0.5;
            for (;;) {
                /* reduced camera system S dc = s (Schur complement on the points) */
                double S[144], s[12];
                memset(S, 0, sizeof(S));
                memset(s, 0, sizeof(s));
                for (int k = 0; k < 12; ++k) S[13 * k] = lambda;
                for (int k = 0; k < 6; ++k) { /* X0 prior: A = I / 0.1, b = -xi0 / 0.1 (Jacobian ~ identity) */
                    S[13 * k] += 100.0;
                    s[k] += -xi0[k] * 100.0;
                }
                if (bf.on) /* between factor: A = J, b = -r */
                    for (int a = 0; a < 12; ++a) {
                        for (int b2 = 0; b2 < 12; ++b2) {
                            double v = 0;
                            for (int k = 0; k < 6; ++k) v += bJ[12 * k + a] * bJ[12 * k + b2];
                            S[12 * a + b2] += v;
                        }
                        double v = 0;
                        for (int k = 0; k < 6; ++k) v += bJ[12 * k + a] * br[k];
                        s[a] -= v;
                    }
                int ok = 1;
                for (int j = 0; j < m && ok; ++j) {
                    const pt_lin_t* L = &lin[j];
                    double Hpp[9] = {lambda, 0, 0, 0, lambda, 0, 0, 0, lambda}, rp[3] = {0, 0, 0};
                    double B[36]; /* H_cp: 12 x 3 */
                    memset(B, 0, sizeof(B));
                    if (j == 0)
                        for (int k = 0; k < 3; ++k) {
                            Hpp[4 * k] += 100.0;
                            rp[k] += -(P[k] - P0_prior[k]) * 100.0;
                        }
                    for (int c = 0; c < 2; ++c) {
                        if (!L->ok[c]) continue;
                        for (int r = 0; r < 2; ++r) {
                            const double* jx = L->Jx[c] + 6 * r;
                            const double* jp = L->Jp[c] + 3 * r;
                            const double br = L->b[c][r];
                            for (int a = 0; a < 6; ++a) {
                                s[6 * c + a] += jx[a] * br;
                                for (int b2 = 0; b2 < 6; ++b2) S[(6 * c + a) * 12 + 6 * c + b2] += jx[a] * jx[b2];
                                for (int k = 0; k < 3; ++k) B[(6 * c + a) * 3 + k] += jx[a] * jp[k];
                            }
                            for (int k = 0; k < 3; ++k) {
                                rp[k] += jp[k] * br;
                                for (int l = 0; l < 3; ++l) Hpp[3 * k + l] += jp[k] * jp[l];
                            }
                        }
                    }
                    double M[9];
                    if (!inv3_sym(Hpp, M)) { ok = 0; break; }
                    double BM[36], Mr[3];
                    for (int a = 0; a < 12; ++a)
                        for (int k = 0; k < 3; ++k)
                            BM[3 * a + k] = B[3 * a] * M[k] + B[3 * a + 1] * M[3 + k] + B[3 * a + 2] * M[6 + k];
                    mv3(M, rp, Mr);
                    for (int a = 0; a < 12; ++a) {
                        s[a] -= B[3 * a] * Mr[0] + B[3 * a + 1] * Mr[1] + B[3 * a + 2] * Mr[2];
                        for (int b2 = 0; b2 < 12; ++b2)
                            S[12 * a + b2] -= BM[3 * a] * B[3 * b2] + BM[3 * a + 1] * B[3 * b2 + 1] + BM[3 * a + 2] * B[3 * b2 + 2];
                    }
                }
                int success = 0, stop = 0;
                double newErr = INFINITY;
                pose_t Xn[2];
                if (ok && chol_solve(S, s, 12)) {
                    /* back-substitution, linearized and nonlinear errors of the step */
                    double newLin = 0;
                    for (int j = 0; j < m; ++j) {
                        const pt_lin_t* L = &lin[j];
                        double Hpp[9] = {lambda, 0, 0, 0, lambda, 0, 0, 0, lambda}, rp[3] = {0, 0, 0};
                        double B[36];
                        memset(B, 0, sizeof(B));
                        if (j == 0)
                            for (int k = 0; k < 3; ++k) {
                                Hpp[4 * k] += 100.0;
                                rp[k] += -(P[k] - P0_prior[k]) * 100.0;
                            }
                        for (int c = 0; c < 2; ++c) {
                            if (!L->ok[c]) continue;
                            for (int r = 0; r < 2; ++r) {
                                const double* jx = L->Jx[c] + 6 * r;
                                const double* jp = L->Jp[c] + 3 * r;
                                for (int a = 0; a < 6; ++a)
                                    for (int k = 0; k < 3; ++k) B[(6 * c + a) * 3 + k] += jx[a] * jp[k];
                                for (int k = 0; k < 3; ++k) {
                                    rp[k] += jp[k] * L->b[c][r];
                                    for (int l = 0; l < 3; ++l) Hpp[3 * k + l] += jp[k] * jp[l];
                                }
                            }
                        }
                        double M[9], q[3];
                        inv3_sym(Hpp, M);
                        for (int k = 0; k < 3; ++k) {
                            q[k] = rp[k];
                            for (int a = 0; a < 12; ++a) q[k] -= B[3 * a + k] * s[a];
                        }
                        double dp[3];
                        mv3(M, q, dp);
                        for (int k = 0; k < 3; ++k) Pn[3 * j + k] = P[3 * j + k] + dp[k];
                        for (int c = 0; c < 2; ++c)
                            for (int r = 0; r < 2; ++r) {
                                const double* jx = L->Jx[c] + 6 * r;
                                const double* jp = L->Jp[c] + 3 * r;
                                double a = -L->b[c][r];
                                for (int k = 0; k < 6; ++k) a += jx[k] * s[6 * c + k];
                                for (int k = 0; k < 3; ++k) a += jp[k] * dp[k];
                                newLin += a * a;
                            }
                        if (j == 0)
                            for (int k = 0; k < 3; ++k) {
                                const double a = (dp[k] + (P[k] - P0_prior[k])) * 10.0;
                                newLin += a * a;
                            }
                    }
                    for (int k = 0; k < 6; ++k) {
                        const double a = (s[k] + xi0[k]) * 10.0;
                        newLin += a * a;
                    }
                    if (bf.on)
                        for (int k = 0; k < 6; ++k) {
                            double a = br[k];
                            for (int c = 0; c < 12; ++c) a += bJ[12 * k + c] * s[c];
                            newLin += a * a;
                        }
                    newLin *= 0.5;
                    const double linChange = oldLin - newLin;
                    if (linChange >= 0) {
                        pose_retract(&X[0], s, &Xn[0]);
                        pose_retract(&X[1], s + 6, &Xn[1]);
                        newErr = ba_error(Xn, K1, K2, Pn, u1, u2, m, P0_prior, &bf);
                        const double costChange = err - newErr;
                        if (linChange > DBL_EPSILON * oldLin) success = costChange / linChange > LM_MIN_FIDELITY;
                        else success = 1;
                        if (fabs(costChange) < 1e-5 * err) stop = 1;
                    }
                }
                if (success) {
                    X[0] = Xn[0];
                    X[1] = Xn[1];
                    memcpy(P, Pn, sizeof(double) * 3 * (size_t)m);
                    err = newErr;
                    lambda /= 10.0;
                    ++iters;
                    break;
                }
                if (stop) break;
                lambda *= 10.0;
                if (lambda >= LM_LAMBDA_UPPER) break;
            }
            const double dec = cur - err;
            if (iters >= max_iters || dec / cur <= 1e-5 || dec <= 1e-5 || !isfinite(cur)) break;
        }
    }
    if (iters_out) *iters_out = iters;
    if (error_out) *error_out = err;
    /* filter_landmarks(reproj_thresh): every measurement projects in front and within the threshold */
    int n_valid = 0;
    for (int j = 0; j < m; ++j) {
        int good = 1;
        /* reproj_error_thresh None (infinite): no filter, every track valid (bundle_adjustment.py:346-355) */
        for (int c = 0; c < 2 && good && isfinite(reproj_thresh); ++c) {
            double pc[3], pr[2];
            const double* uv = c ? u2 + 2 * j : u1 + 2 * j;
            if (!project(&X[c], c ? K2 : K1, P + 3 * j, pc, pr)) { good = 0; break; }
            const double dx = pr[0] - uv[0], dy = pr[1] - uv[1];
            if (!(sqrt(dx * dx + dy * dy) < reproj_thresh)) good = 0;
        }
        if (good) {
            valid[tri[j]] = 1;
            ++n_valid;
        }
    }
    free(tri); free(P); free(u1); free(u2); free(Pn); free(lin);
    if (n_valid == 0) { /* no camera keeps a landmark: the verifier's pose (two_view_estimator.py:199-202) */
        memcpy(R_out, R_in, 9 * sizeof(double));
        memcpy(t_out, t_in, 3 * sizeof(double));
        return 2;
    }
    /* i2Ti1 = wTi2^-1 wTi1 */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R_out[3 * i + j] = X[1].R[i] * X[0].R[j] + X[1].R[3 + i] * X[0].R[3 + j] + X[1].R[6 + i] * X[0].R[6 + j];
    const double d[3] = {X[0].t[0] - X[1].t[0], X[0].t[1] - X[1].t[1], X[0].t[2] - X[1].t[2]};
    mtv3(X[1].R, d, t_out);
    const double nt = sqrt(t_out[0] * t_out[0] + t_out[1] * t_out[1] + t_out[2] * t_out[2]);
    for (int k = 0; k < 3; ++k) t_out[k] /= nt;
    return 0;
}
