// Two-view triangulation + bundle adjustment of every verified pair, one wavefront per pair.
//
// Reference: gtsfm/two_view_estimator.py:101-208 (triangulate_two_view_correspondences, bundle_adjust) and :311-337
// (run_2view's BA branch), on GTSAM 4.2 (triangulatePoint3 + LevenbergMarquardtOptimizer; not in this image). The
// arithmetic is oracle/ba2.c's restatement, performed in fp64 in the same order per track; the sums over tracks are
// wave reductions here (sequential there), so results agree to rounding, not bit for bit. Per pair:
//   1. cameras X0 = identity (i1), X1 = i2Ti1^-1 from the verifier's R, unit t;
//   2. lane-parallel triangulation of the verified correspondences (matcher order): DLT null vector by one-sided
//      Jacobi SVD (rank >= 3), LM refinement of the point on two unit-noise reprojection factors (lambda 1, factor
//      10, <= 100 iterations, absolute tolerance 1), cheirality and < tri_thresh px reprojection checks; the kept
//      tracks are compacted in order (the first one carries the scale prior);
//   3. Levenberg-Marquardt on (X0, X1, points): Huber(1.345) reprojection factors, X0 prior sigma 0.1, first-point
//      prior sigma 0.1, isotropic damping, GTSAM's accept / lambda schedule and convergence tests. Each trial step
//      builds the 12 x 12 reduced camera system: every lane adds its tracks' Schur contributions into a private LDS
//      column, a 64-way reduction sums them, lane 0 solves it (Cholesky), and a second pass back-substitutes the
//      points and evaluates the linearized and nonlinear costs of the step;
//   4. filter_landmarks(reproj_thresh): tracks whose two reprojections are in front and within the threshold; an
//      infinite reproj_thresh (the reference's reproj_error_thresh None) keeps every triangulated track.
// Calibration is held fixed: the reference also optimises one Cal3Bundler (f, k1, k2) variable per camera under a
// 1e-5 prior (GeneralSFMFactor2Cal3Bundler + PriorFactorCal3Bundler, bundle_adjustment.py:106-136,180-200). Holding
// K at its prior value with k1 = k2 = 0 is the limit of that prior; the host refuses non-zero k1 / k2
// (geometry.calibration_params), so the approximation is the prior's 1e-5 freedom in f only.
// Relative-pose priors (optional, per pair): the prior's i2Ti1 initialises the second camera and a BetweenFactorPose3
// joins the LM (two_view_estimator.py:165,192; bundle_adjustment.py:136-152), as oracle/ba2.c.
// Outputs per pair: status (0 BA ok, 1 no track triangulated, 2 no track valid, 3 not run: verification failed or
// fewer than min_inliers verified rows -- the reference's guard at :312), R / unit t (the verifier's for statuses 1-3),
// the post-BA mask over the putatives (the pre-BA mask when not run), its count and the LM iterations.
#include "common.hpp"

namespace {

constexpr double kHuberK = 1.345;
constexpr double kMinFidelity = 1e-3;
constexpr double kLambdaUpper = 1e5;
constexpr double kDblEps = 2.220446049250313e-16;
constexpr int kAcc = 90;  // 78 entries of the upper triangle of the 12 x 12 reduced system + 12 right-hand sides
constexpr int kInnerMax = 64;

struct Pose {
    double R[9];  // wRc row-major
    double t[3];  // wtc
};

__device__ __forceinline__ void skew3(const double* w, double* S) {
    S[0] = 0; S[1] = -w[2]; S[2] = w[1];
    S[3] = w[2]; S[4] = 0; S[5] = -w[0];
    S[6] = -w[1]; S[7] = w[0]; S[8] = 0;
}

__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

__device__ __forceinline__ void mtv3(const double* A, const double* v, double* o) {
#pragma unroll
    for (int j = 0; j < 3; ++j) o[j] = A[j] * v[0] + A[3 + j] * v[1] + A[6 + j] * v[2];
}

__device__ __forceinline__ void mv3(const double* A, const double* v, double* o) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}

__device__ void so3_exp(const double* w, double* R) {
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
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * W[k] + b * W2[k];
}

__device__ void so3_log(const double* R, double* w) {
    double c = 0.5 * (R[0] + R[4] + R[8] - 1.0);
    c = fmin(1.0, fmax(-1.0, c));
    const double th = acos(c);
    const double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (th < 1e-8) {
        for (int k = 0; k < 3; ++k) w[k] = 0.5 * v[k];
    } else if (3.14159265358979323846 - th < 1e-6) {
        const int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
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

__device__ void pose_retract(const Pose& X, const double* xi, Pose& o) {
    double dR[9], tv[3], W[9], W2[9];
    so3_exp(xi, dR);
    const double* w = xi;
    const double* v = xi + 3;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
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
    mm3(X.R, dR, o.R);
    double Rt[3];
    mv3(X.R, tv, Rt);
    for (int i = 0; i < 3; ++i) o.t[i] = X.t[i] + Rt[i];
}

__device__ void pose_log(const Pose& T, double* xi) {
    double w[3];
    so3_log(T.R, w);
    const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    xi[0] = w[0]; xi[1] = w[1]; xi[2] = w[2];
    if (th < 1e-10) {
        for (int k = 0; k < 3; ++k) xi[3 + k] = T.t[k];
        return;
    }
    double W[9], Wt[3], WWt[3];
    const double wn[3] = {w[0] / th, w[1] / th, w[2] / th};
    skew3(wn, W);
    mv3(W, T.t, Wt);
    mv3(W, Wt, WWt);
    const double tn = tan(0.5 * th);
    for (int k = 0; k < 3; ++k) xi[3 + k] = T.t[k] - (0.5 * th) * Wt[k] + (1.0 - th / (2.0 * tn)) * WWt[k];
}

// ------------------------------------------------------------------ relative-pose prior (oracle/ba2.c between_t)
// BetweenFactorPose3(X0, X1, m = i2Ti1_prior^-1, Diagonal.Sigmas) (bundle_adjustment.py:136-152): whitened
// e = Logmap(m^-1 X0^-1 X1) / sigma; d e / d X1 = Jr^-1(e), d e / d X0 = -Jr^-1(e) Ad(hx^-1), hx = X0^-1 X1, with
// the closed-form Jr^-1 of se3_jr_inv. Same operations as the oracle; computed redundantly by every lane.
struct Between {
    bool on;
    Pose minv;       // the prior's value i2Ti1 (= m^-1)
    double isig[6];  // 1 / sigma, rotation first
};

__device__ void pose_mul(const Pose& A, const Pose& B, Pose& C) {
    Pose o;
    mm3(A.R, B.R, o.R);
    mv3(A.R, B.t, o.t);
    for (int k = 0; k < 3; ++k) o.t[k] += A.t[k];
    C = o;
}

__device__ void pose_inv(const Pose& A, Pose& C) {
    Pose o;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o.R[3 * i + j] = A.R[3 * j + i];
    mtv3(A.R, A.t, o.t);
    for (int k = 0; k < 3; ++k) o.t[k] = -o.t[k];
    C = o;
}

__device__ void between_residual(const Between& f, const Pose* X, double* e, Pose& hx) {
    Pose x0i, E0;
    pose_inv(X[0], x0i);
    pose_mul(x0i, X[1], hx);
    pose_mul(f.minv, hx, E0);
    pose_log(E0, e);
}

__device__ double between_error(const Between& f, const Pose* X) {
    if (!f.on) return 0.0;
    double e[6];
    Pose hx;
    between_residual(f, X, e, hx);
    double s = 0;
    for (int k = 0; k < 6; ++k) s += (e[k] * f.isig[k]) * (e[k] * f.isig[k]);
    return 0.5 * s;
}

// exact inverse right Jacobian of SE(3) at e = (w, v), rotation first (GTSAM Pose3::LogmapDerivative):
// Jr(e) = [[Jw, 0], [Q, Jw]] so Jr^-1 = [[A, 0], [-A Q A, A]] with A = Jw^-1 = I + W/2 + c W^2,
// c = 1/th^2 - 1/(2 th tan(th/2)), and Q the right-Jacobian coupling block (Barfoot & Furgale 2014, eq. 102,
// evaluated at -e): Q = -P/2 + c1 (WP + PW - WPW) - c2 (WWP + PWW - 3 WPW) + c3 (WPWW + WWPW), W = w^, P = v^,
// c1 = (th - sin th) / th^3, c2 = (th^2 + 2 cos th - 2) / (2 th^4), c3 = (2 th - 3 sin th + th cos th) / (2 th^5);
// below th = 1e-2 the coefficients use their Taylor series to th^2.
__device__ void se3_jr_inv(const double* e, double* Ji) {
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

__device__ void between_linearize(const Between& f, const Pose* X, double* r, double* J) {
    double e[6];
    Pose hx, hi;
    between_residual(f, X, e, hx);
    double Ji[36], Ad[36];
    se3_jr_inv(e, Ji);
    pose_inv(hx, hi);
    for (int k = 0; k < 36; ++k) Ad[k] = 0.0;
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
            J[12 * i + j] = -a * f.isig[i];
            J[12 * i + 6 + j] = Ji[6 * i + j] * f.isig[i];
        }
        r[i] = e[i] * f.isig[i];
    }
}

__device__ __forceinline__ bool project(const Pose& X, const double* K, const double* p, double* pc, double* uv) {
    const double d[3] = {p[0] - X.t[0], p[1] - X.t[1], p[2] - X.t[2]};
    mtv3(X.R, d, pc);
    if (pc[2] <= 0.0) return false;
    uv[0] = K[1] + K[0] * (pc[0] / pc[2]);
    uv[1] = K[2] + K[0] * (pc[1] / pc[2]);
    return true;
}

__device__ __forceinline__ void project_jac(const Pose& X, const double* K, const double* pc, double* Jp, double* Jx) {
    const double iz = 1.0 / pc[2], xn = pc[0] * iz, yn = pc[1] * iz, f = K[0];
    const double D[6] = {f * iz, 0.0, -f * xn * iz, 0.0, f * iz, -f * yn * iz};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
            Jp[3 * r + j] = D[3 * r] * X.R[3 * j] + D[3 * r + 1] * X.R[3 * j + 1] + D[3 * r + 2] * X.R[3 * j + 2];
        const double* d = D + 3 * r;
        Jx[6 * r + 0] = d[1] * pc[2] - d[2] * pc[1];
        Jx[6 * r + 1] = -d[0] * pc[2] + d[2] * pc[0];
        Jx[6 * r + 2] = d[0] * pc[1] - d[1] * pc[0];
        Jx[6 * r + 3] = -d[0];
        Jx[6 * r + 4] = -d[1];
        Jx[6 * r + 5] = -d[2];
    }
}

__device__ __forceinline__ double huber_loss(double d) {
    return d <= kHuberK ? 0.5 * d * d : kHuberK * d - 0.5 * kHuberK * kHuberK;
}
__device__ __forceinline__ double huber_weight(double d) { return d <= kHuberK ? 1.0 : kHuberK / d; }

__device__ bool inv3(const double* A, double* I) {
    const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    if (!(fabs(det) > 0.0) || !isfinite(det)) return false;
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
    return true;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------------------------ triangulation (one lane per correspondence)
__device__ double tri_factor(const Pose& X, const double* K, const double* p, const double* uv, double* e,
                             double* Jp) {
    double pc[3], pr[2], Jx[12];
    if (!project(X, K, p, pc, pr)) {
        e[0] = e[1] = 2.0 * K[0];
        for (int k = 0; k < 6; ++k) Jp[k] = 0.0;
    } else {
        e[0] = pr[0] - uv[0];
        e[1] = pr[1] - uv[1];
        project_jac(X, K, pc, Jp, Jx);
    }
    return 0.5 * (e[0] * e[0] + e[1] * e[1]);
}

__device__ bool chol3_solve(double* a, double* b) {
    for (int j = 0; j < 3; ++j) {
        double s = a[4 * j];
        for (int k = 0; k < j; ++k) s -= a[3 * j + k] * a[3 * j + k];
        if (!(s > 0.0)) return false;
        const double d = sqrt(s);
        a[4 * j] = d;
        for (int i = j + 1; i < 3; ++i) {
            double v = a[3 * i + j];
            for (int k = 0; k < j; ++k) v -= a[3 * i + k] * a[3 * j + k];
            a[3 * i + j] = v / d;
        }
    }
    for (int i = 0; i < 3; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= a[3 * i + k] * b[k];
        b[i] = v / a[4 * i];
    }
    for (int i = 2; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < 3; ++k) v -= a[3 * k + i] * b[k];
        b[i] = v / a[4 * i];
    }
    return true;
}

__device__ bool triangulate2(const Pose* X, const double* K1, const double* K2, const double* uv1, const double* uv2,
                             double tri_thresh, double* p_out) {
    const double* Ks[2] = {K1, K2};
    const double* uvs[2] = {uv1, uv2};
    double U[16], V[16];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const double* Rc = X[c].R;
        double P[12];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double row[3] = {Rc[r], Rc[3 + r], Rc[6 + r]};
            P[4 * r] = row[0]; P[4 * r + 1] = row[1]; P[4 * r + 2] = row[2];
            P[4 * r + 3] = -(row[0] * X[c].t[0] + row[1] * X[c].t[1] + row[2] * X[c].t[2]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double kp0 = Ks[c][0] * P[j] + Ks[c][1] * P[8 + j];
            const double kp1 = Ks[c][0] * P[4 + j] + Ks[c][2] * P[8 + j];
            U[4 * (2 * c) + j] = uvs[c][0] * P[8 + j] - kp0;
            U[4 * (2 * c + 1) + j] = uvs[c][1] * P[8 + j] - kp1;
        }
    }
    for (int k = 0; k < 16; ++k) V[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    al += U[4 * i + p] * U[4 * i + p];
                    be += U[4 * i + q] * U[4 * i + q];
                    ga += U[4 * i + p] * U[4 * i + q];
                }
                if (fabs(ga) <= 1e-15 * sqrt(al * be) || ga == 0.0) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double up = U[4 * i + p], uq = U[4 * i + q];
                    U[4 * i + p] = cs * up - sn * uq;
                    U[4 * i + q] = sn * up + cs * uq;
                    const double vp = V[4 * i + p], vq = V[4 * i + q];
                    V[4 * i + p] = cs * vp - sn * vq;
                    V[4 * i + q] = sn * vp + cs * vq;
                }
            }
        if (!rotated) break;
    }
    int rank = 0;
    double smin = INFINITY, vmin[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += U[4 * i + j] * U[4 * i + j];
        s = sqrt(s);
        if (s > 1e-9) ++rank;
        if (s < smin) {
            smin = s;
#pragma unroll
            for (int i = 0; i < 4; ++i) vmin[i] = V[4 * i + j];
        }
    }
    if (rank < 3) return false;
    double p[3] = {vmin[0] / vmin[3], vmin[1] / vmin[3], vmin[2] / vmin[3]};
    double e[2], J[6], err = 0;
    for (int c = 0; c < 2; ++c) err += tri_factor(X[c], Ks[c], p, uvs[c], e, J);
    double lambda = 1.0;
    int iters = 0;
    if (isfinite(err) && err > 0.0) {
        for (int outer = 0; outer < 200; ++outer) {
            const double cur = err;
            double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, bb = 0;
            double Js[2][6], es[2][2];
            for (int c = 0; c < 2; ++c) {
                tri_factor(X[c], Ks[c], p, uvs[c], es[c], Js[c]);
                for (int r = 0; r < 2; ++r) {
                    for (int i = 0; i < 3; ++i) {
                        g[i] += Js[c][3 * r + i] * (-es[c][r]);
                        for (int j = 0; j < 3; ++j) H[3 * i + j] += Js[c][3 * r + i] * Js[c][3 * r + j];
                    }
                    bb += es[c][r] * es[c][r];
                }
            }
            for (int inner = 0; inner < kInnerMax; ++inner) {
                double Hd[9], d[3] = {g[0], g[1], g[2]};
                for (int k = 0; k < 9; ++k) Hd[k] = H[k];
                for (int i = 0; i < 3; ++i) Hd[4 * i] += lambda;
                bool success = false, stop = false;
                double newp[3], newErr = INFINITY;
                if (chol3_solve(Hd, d)) {
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
                        for (int c = 0; c < 2; ++c) newErr += tri_factor(X[c], Ks[c], newp, uvs[c], e, J);
                        const double costChange = err - newErr;
                        if (linChange > kDblEps * oldLin) success = costChange / linChange > kMinFidelity;
                        else success = true;
                        if (fabs(costChange) < 1e-5 * err) stop = true;
                    }
                }
                if (success) {
                    for (int i = 0; i < 3; ++i) p[i] = newp[i];
                    err = newErr;
                    lambda /= 10.0;
                    ++iters;
                    break;
                }
                if (stop) break;
                lambda *= 10.0;
                if (lambda >= kLambdaUpper) break;
            }
            const double dec = cur - err;
            if (iters >= 100 || dec / cur <= 1e-5 || dec <= 1.0 || !isfinite(cur)) break;
        }
    }
    for (int c = 0; c < 2; ++c) {
        double pc[3], pr[2];
        if (!project(X[c], Ks[c], p, pc, pr)) return false;
        const double dx = pr[0] - uvs[c][0], dy = pr[1] - uvs[c][1];
        if (!(sqrt(dx * dx + dy * dy) < tri_thresh)) return false;
    }
    p_out[0] = p[0]; p_out[1] = p[1]; p_out[2] = p[2];
    return true;
}

// ------------------------------------------------------------------ bundle adjustment pieces (one track)
struct TrackLin {
    double Jx[2][12];
    double Jp[2][6];
    double b[2][2];
    bool ok[2];
};

__device__ __forceinline__ void linearize_track(const Pose* X, const double* K1, const double* K2, const double* p,
                                                const double* uv, TrackLin& L) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const double* K = c ? K2 : K1;
        double pc[3], pr[2];
        L.ok[c] = project(X[c], K, p, pc, pr);
        if (!L.ok[c]) {
            for (int k = 0; k < 12; ++k) L.Jx[c][k] = 0.0;
            for (int k = 0; k < 6; ++k) L.Jp[c][k] = 0.0;
            L.b[c][0] = L.b[c][1] = 0.0;
            continue;
        }
        project_jac(X[c], K, pc, L.Jp[c], L.Jx[c]);
        const double e0 = pr[0] - uv[2 * c], e1 = pr[1] - uv[2 * c + 1];
        const double sw = sqrt(huber_weight(sqrt(e0 * e0 + e1 * e1)));
        for (int k = 0; k < 12; ++k) L.Jx[c][k] *= sw;
        for (int k = 0; k < 6; ++k) L.Jp[c][k] *= sw;
        L.b[c][0] = -sw * e0;
        L.b[c][1] = -sw * e1;
    }
}

// H_pp (+ damping, + the scale prior for track 0), its inverse, the point right-hand side and B = H_cp (12 x 3)
__device__ __forceinline__ bool point_block(const TrackLin& L, double lambda, bool first, const double* p,
                                            const double* prior, double* M, double* rp, double* B) {
    double Hpp[9] = {lambda, 0, 0, 0, lambda, 0, 0, 0, lambda};
    rp[0] = rp[1] = rp[2] = 0.0;
    for (int k = 0; k < 36; ++k) B[k] = 0.0;
    if (first)
        for (int k = 0; k < 3; ++k) {
            Hpp[4 * k] += 100.0;
            rp[k] += -(p[k] - prior[k]) * 100.0;
        }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (!L.ok[c]) continue;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double* jx = L.Jx[c] + 6 * r;
            const double* jp = L.Jp[c] + 3 * r;
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) B[(6 * c + a) * 3 + k] += jx[a] * jp[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                rp[k] += jp[k] * L.b[c][r];
#pragma unroll
                for (int l = 0; l < 3; ++l) Hpp[3 * k + l] += jp[k] * jp[l];
            }
        }
    }
    return inv3(Hpp, M);
}

__device__ double track_error(const Pose* X, const double* K1, const double* K2, const double* p, const double* uv) {
    double e = 0;
    for (int c = 0; c < 2; ++c) {
        double pc[3], pr[2];
        if (!project(X[c], c ? K2 : K1, p, pc, pr)) continue;
        const double dx = pr[0] - uv[2 * c], dy = pr[1] - uv[2 * c + 1];
        e += huber_loss(sqrt(dx * dx + dy * dy));
    }
    return e;
}

__device__ double pose_prior_error(const Pose& X0) {
    double xi[6];
    pose_log(X0, xi);
    double s = 0;
    for (int k = 0; k < 6; ++k) s += xi[k] * xi[k];
    return 0.5 * s / 0.01;
}

struct Ba2Args {
    const float* kp_xy;
    const double* intr;
    int kmax;
    const int* pairs;
    const uint2* match_idx;
    const int* match_count;
    int mcap;
    const uint8_t* in_mask;
    const double* R_in;
    const double* t_in;
    const int* status_in;
    const double* prior_Rt;   // [pair][12] i2Ti1_prior (R row-major, t) or null
    const double* prior_sig;  // [pair][6] its sigmas; sigma[0] <= 0: no prior for the pair
    int min_inliers, max_iters;
    double reproj_thresh, tri_thresh;
    double* P;    // [pair][mcap][3]
    double* Pn;   // [pair][mcap][3]
    double* UV;   // [pair][mcap][4]
    int* list;    // [pair][mcap]: putative index of each track
    double* R_out;
    double* t_out;
    uint8_t* out_mask;
    int* n_out;
    int* status_out;
    int* iters_out;
};

__global__ __launch_bounds__(64) void ba2_kernel(Ba2Args a) {
    __shared__ double acc[kAcc * 64];
    __shared__ double sys[144 + 12];
    __shared__ double sh_dc[12];
    __shared__ int sh_ok;
    const int p = blockIdx.x, lane = threadIdx.x;
    const int M = a.match_count[p];
    const uint8_t* in_mask = a.in_mask + (size_t)p * a.mcap;
    uint8_t* out_mask = a.out_mask + (size_t)p * a.mcap;
    int n_in = 0;
    for (int j0 = 0; j0 < M; j0 += 64) n_in += __popcll(__ballot(j0 + lane < M && in_mask[j0 + lane] != 0));
    auto copy_input = [&](int status) {
        for (int j = lane; j < M; j += 64) out_mask[j] = in_mask[j];
        if (lane == 0) {
            for (int k = 0; k < 9; ++k) a.R_out[9 * p + k] = a.R_in[9 * p + k];
            for (int k = 0; k < 3; ++k) a.t_out[3 * p + k] = a.t_in[3 * p + k];
            a.n_out[p] = n_in;
            a.status_out[p] = status;
            if (a.iters_out) a.iters_out[p] = 0;
        }
    };
    if (a.status_in[p] != 0 || n_in < a.min_inliers) {
        copy_input(3);
        return;
    }
    const int i1 = a.pairs[2 * p], i2 = a.pairs[2 * p + 1];
    const double K1[3] = {a.intr[3 * i1], a.intr[3 * i1 + 1], a.intr[3 * i1 + 2]};
    const double K2[3] = {a.intr[3 * i2], a.intr[3 * i2 + 1], a.intr[3 * i2 + 2]};
    const double* Rin = a.R_in + 9 * p;
    const double* tin = a.t_in + 3 * p;
    // a relative-pose prior initialises the second camera (two_view_estimator.py:165-171) and adds the between factor
    Between bf;
    bf.on = a.prior_Rt != nullptr && a.prior_sig != nullptr && a.prior_sig[6 * p] > 0.0;
    if (bf.on) {
        for (int k = 0; k < 9; ++k) bf.minv.R[k] = a.prior_Rt[12 * p + k];
        for (int k = 0; k < 3; ++k) bf.minv.t[k] = a.prior_Rt[12 * p + 9 + k];
        for (int k = 0; k < 6; ++k) bf.isig[k] = 1.0 / a.prior_sig[6 * p + k];
        Rin = a.prior_Rt + 12 * p;
        tin = a.prior_Rt + 12 * p + 9;
    }
    Pose X[2];
    for (int k = 0; k < 9; ++k) X[0].R[k] = (k % 4 == 0) ? 1.0 : 0.0;
    X[0].t[0] = X[0].t[1] = X[0].t[2] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) X[1].R[3 * i + j] = Rin[3 * j + i];
    mtv3(Rin, tin, X[1].t);
    for (int i = 0; i < 3; ++i) X[1].t[i] = -X[1].t[i];
    double* P = a.P + (size_t)p * a.mcap * 3;
    double* Pn = a.Pn + (size_t)p * a.mcap * 3;
    double* UV = a.UV + (size_t)p * a.mcap * 4;
    int* list = a.list + (size_t)p * a.mcap;
    const uint2* mi = a.match_idx + (size_t)p * a.mcap;
    const float* kp1 = a.kp_xy + (size_t)i1 * a.kmax * 2;
    const float* kp2 = a.kp_xy + (size_t)i2 * a.kmax * 2;
    // triangulation of the verified rows, compacted in order
    int m = 0;
    for (int j0 = 0; j0 < M; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        double pt[3], uv[4];
        if (j < M && in_mask[j] != 0) {
            const uint2 r = mi[j];
            uv[0] = kp1[2 * r.x]; uv[1] = kp1[2 * r.x + 1];
            uv[2] = kp2[2 * r.y]; uv[3] = kp2[2 * r.y + 1];
            ok = triangulate2(X, K1, K2, uv, uv + 2, a.tri_thresh, pt);
        }
        const unsigned long long bal = __ballot(ok);
        const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
        if (ok) {
            const int s = m + rank;
            list[s] = j;
            for (int k = 0; k < 3; ++k) P[3 * s + k] = pt[k];
            for (int k = 0; k < 4; ++k) UV[4 * s + k] = uv[k];
        }
        m += __popcll(bal);
    }
    for (int j = lane; j < M; j += 64) out_mask[j] = 0;
    if (m == 0) {  // the initial pose: the prior's when given (two_view_estimator.py:186-187), unit translation
        if (lane == 0) {
            const double nt = sqrt(tin[0] * tin[0] + tin[1] * tin[1] + tin[2] * tin[2]);
            for (int k = 0; k < 9; ++k) a.R_out[9 * p + k] = Rin[k];
            for (int k = 0; k < 3; ++k) a.t_out[3 * p + k] = tin[k] / nt;
            a.n_out[p] = 0;
            a.status_out[p] = 1;
            if (a.iters_out) a.iters_out[p] = 0;
        }
        return;
    }
    __syncthreads();
    const double prior[3] = {P[0], P[1], P[2]};
    // initial nonlinear error
    double err;
    {
        double e = 0;
        for (int j = lane; j < m; j += 64) e += track_error(X, K1, K2, P + 3 * j, UV + 4 * j);
        err = wave_sum(e) + pose_prior_error(X[0]) + between_error(bf, X);  // the point prior is 0 at the start
    }
    double lambda = 1e-5;
    int iters = 0;
    if (err > 0.0) {
        for (;;) {  // ends: every outer step either accepts (iters <= max_iters) or leaves err unchanged (dec = 0)
            const double cur = err;
            double xi0[6];
            pose_log(X[0], xi0);
            double br[6] = {0, 0, 0, 0, 0, 0}, bJ[72];
            if (bf.on) between_linearize(bf, X, br, bJ);
            bool accepted = false;
            for (int inner = 0; inner < kInnerMax; ++inner) {
                // pass 1: reduced camera system, lane-private LDS columns
                for (int e = 0; e < kAcc; ++e) acc[e * 64 + lane] = 0.0;
                double oldLin_l = 0.0;
                int bad = 0;
                for (int j = lane; j < m; j += 64) {
                    TrackLin L;
                    linearize_track(X, K1, K2, P + 3 * j, UV + 4 * j, L);
                    double Mi[9], rp[3], B[36];
                    if (!point_block(L, lambda, j == 0, P + 3 * j, prior, Mi, rp, B)) bad = 1;
                    for (int c = 0; c < 2; ++c)
                        oldLin_l += L.b[c][0] * L.b[c][0] + L.b[c][1] * L.b[c][1];
                    if (j == 0)
                        for (int k = 0; k < 3; ++k) oldLin_l += (P[k] - prior[k]) * (P[k] - prior[k]) * 100.0;
                    double BM[36], Mr[3];
#pragma unroll
                    for (int r = 0; r < 12; ++r)
#pragma unroll
                        for (int k = 0; k < 3; ++k)
                            BM[3 * r + k] = B[3 * r] * Mi[k] + B[3 * r + 1] * Mi[3 + k] + B[3 * r + 2] * Mi[6 + k];
                    mv3(Mi, rp, Mr);
                    int e = 0;
#pragma unroll
                    for (int r = 0; r < 12; ++r) {
                        const int c = r / 6, ar = r % 6;
#pragma unroll
                        for (int s2 = r; s2 < 12; ++s2, ++e) {
                            double v = -(BM[3 * r] * B[3 * s2] + BM[3 * r + 1] * B[3 * s2 + 1] +
                                         BM[3 * r + 2] * B[3 * s2 + 2]);
                            if (s2 / 6 == c && L.ok[c]) {
                                const int as = s2 % 6;
                                v += L.Jx[c][ar] * L.Jx[c][as] + L.Jx[c][6 + ar] * L.Jx[c][6 + as];
                            }
                            acc[e * 64 + lane] += v;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 12; ++r) {
                        const int c = r / 6, ar = r % 6;
                        double v = -(B[3 * r] * Mr[0] + B[3 * r + 1] * Mr[1] + B[3 * r + 2] * Mr[2]);
                        if (L.ok[c]) v += L.Jx[c][ar] * L.b[c][0] + L.Jx[c][6 + ar] * L.b[c][1];
                        acc[(78 + r) * 64 + lane] += v;
                    }
                }
                double brr = 0.0;
                for (int k = 0; k < 6; ++k) brr += br[k] * br[k];
                const double oldLin = 0.5 * (wave_sum(oldLin_l) + 100.0 * (xi0[0] * xi0[0] + xi0[1] * xi0[1] +
                                                                         xi0[2] * xi0[2] + xi0[3] * xi0[3] +
                                                                         xi0[4] * xi0[4] + xi0[5] * xi0[5]) +
                                             brr);
                const bool any_bad = __ballot(bad) != 0ull;
                __syncthreads();
                for (int e = lane; e < kAcc; e += 64) {
                    double s = 0.0;
                    for (int l = 0; l < 64; ++l) s += acc[e * 64 + l];
                    // unpack into the full symmetric system (sys[0..143]) and the rhs (sys[144..155])
                    if (e < 78) {
                        int r = 0, rem = e;
                        while (rem >= 12 - r) { rem -= 12 - r; ++r; }
                        const int c2 = r + rem;
                        sys[12 * r + c2] = s;
                        sys[12 * c2 + r] = s;
                    } else {
                        sys[144 + (e - 78)] = s;
                    }
                }
                __syncthreads();
                if (lane == 0) {
                    double* S = sys;  // solved in place in LDS (lane 0; the system is 12 x 12)
                    double* s = sys + 144;
                    for (int k = 0; k < 12; ++k) S[13 * k] += lambda;
                    for (int k = 0; k < 6; ++k) {
                        S[13 * k] += 100.0;
                        s[k] += -xi0[k] * 100.0;
                    }
                    if (bf.on)  // between factor: A = J, b = -r
                        for (int a2 = 0; a2 < 12; ++a2) {
                            for (int b2 = 0; b2 < 12; ++b2) {
                                double v = 0;
                                for (int k = 0; k < 6; ++k) v += bJ[12 * k + a2] * bJ[12 * k + b2];
                                S[12 * a2 + b2] += v;
                            }
                            double v = 0;
                            for (int k = 0; k < 6; ++k) v += bJ[12 * k + a2] * br[k];
                            s[a2] -= v;
                        }
                    int ok = any_bad ? 0 : 1;
                    for (int j = 0; j < 12 && ok; ++j) {  // Cholesky
                        double v = S[13 * j];
                        for (int k = 0; k < j; ++k) v -= S[12 * j + k] * S[12 * j + k];
                        if (!(v > 0.0)) { ok = 0; break; }
                        const double d = sqrt(v);
                        S[13 * j] = d;
                        for (int i = j + 1; i < 12; ++i) {
                            double w = S[12 * i + j];
                            for (int k = 0; k < j; ++k) w -= S[12 * i + k] * S[12 * j + k];
                            S[12 * i + j] = w / d;
                        }
                    }
                    if (ok) {
                        for (int i = 0; i < 12; ++i) {
                            double v = s[i];
                            for (int k = 0; k < i; ++k) v -= S[12 * i + k] * s[k];
                            s[i] = v / S[13 * i];
                        }
                        for (int i = 11; i >= 0; --i) {
                            double v = s[i];
                            for (int k = i + 1; k < 12; ++k) v -= S[12 * k + i] * s[k];
                            s[i] = v / S[13 * i];
                        }
                        for (int k = 0; k < 12; ++k) sh_dc[k] = s[k];
                    }
                    sh_ok = ok;
                }
                __syncthreads();
                bool success = false, stop = false;
                double newErr = INFINITY;
                Pose Xn[2];
                if (sh_ok) {
                    double dc[12];
                    for (int k = 0; k < 12; ++k) dc[k] = sh_dc[k];
                    pose_retract(X[0], dc, Xn[0]);
                    pose_retract(X[1], dc + 6, Xn[1]);
                    // pass 2: back-substitution, linearized and nonlinear costs of the step
                    double nl = 0.0, ne = 0.0;
                    for (int j = lane; j < m; j += 64) {
                        TrackLin L;
                        linearize_track(X, K1, K2, P + 3 * j, UV + 4 * j, L);
                        double Mi[9], rp[3], B[36];
                        point_block(L, lambda, j == 0, P + 3 * j, prior, Mi, rp, B);
                        double q[3], dp[3];
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            q[k] = rp[k];
#pragma unroll
                            for (int r = 0; r < 12; ++r) q[k] -= B[3 * r + k] * dc[r];
                        }
                        mv3(Mi, q, dp);
                        double pn[3];
                        for (int k = 0; k < 3; ++k) pn[k] = P[3 * j + k] + dp[k];
                        for (int k = 0; k < 3; ++k) Pn[3 * j + k] = pn[k];
#pragma unroll
                        for (int c = 0; c < 2; ++c)
#pragma unroll
                            for (int r = 0; r < 2; ++r) {
                                double v = -L.b[c][r];
#pragma unroll
                                for (int k = 0; k < 6; ++k) v += L.Jx[c][6 * r + k] * dc[6 * c + k];
#pragma unroll
                                for (int k = 0; k < 3; ++k) v += L.Jp[c][3 * r + k] * dp[k];
                                nl += v * v;
                            }
                        ne += track_error(Xn, K1, K2, pn, UV + 4 * j);
                        if (j == 0)
                            for (int k = 0; k < 3; ++k) {
                                const double v = (dp[k] + (P[k] - prior[k])) * 10.0;
                                nl += v * v;
                                ne += 0.5 * (pn[k] - prior[k]) * (pn[k] - prior[k]) / 0.01;
                            }
                    }
                    double newLin = wave_sum(nl);
                    for (int k = 0; k < 6; ++k) {
                        const double v = (dc[k] + xi0[k]) * 10.0;
                        newLin += v * v;
                    }
                    if (bf.on)
                        for (int k = 0; k < 6; ++k) {
                            double v = br[k];
                            for (int c = 0; c < 12; ++c) v += bJ[12 * k + c] * dc[c];
                            newLin += v * v;
                        }
                    newLin *= 0.5;
                    const double linChange = oldLin - newLin;
                    if (linChange >= 0) {
                        newErr = wave_sum(ne) + pose_prior_error(Xn[0]) + between_error(bf, Xn);
                        const double costChange = err - newErr;
                        if (linChange > kDblEps * oldLin) success = costChange / linChange > kMinFidelity;
                        else success = true;
                        if (fabs(costChange) < 1e-5 * err) stop = true;
                    }
                }
                __syncthreads();
                if (success) {
                    X[0] = Xn[0];
                    X[1] = Xn[1];
                    for (int j = lane; j < m; j += 64)
                        for (int k = 0; k < 3; ++k) P[3 * j + k] = Pn[3 * j + k];
                    err = newErr;
                    lambda /= 10.0;
                    ++iters;
                    accepted = true;
                    __syncthreads();
                    break;
                }
                if (stop) break;
                lambda *= 10.0;
                if (lambda >= kLambdaUpper) break;
            }
            (void)accepted;
            const double dec = cur - err;
            if (iters >= a.max_iters || dec / cur <= 1e-5 || dec <= 1e-5 || !isfinite(cur)) break;
        }
    }
    __syncthreads();
    // filter_landmarks(reproj_thresh)
    int n_valid = 0;
    for (int j0 = 0; j0 < m; j0 += 64) {
        const int j = j0 + lane;
        bool good = false;
        if (j < m) {
            good = true;
            // reproj_error_thresh None (an infinite threshold): no filter at all, every track valid
            // (bundle_adjustment.py:346-355), without the cheirality test of filter_landmarks
            for (int c = 0; c < 2 && good && isfinite(a.reproj_thresh); ++c) {
                double pc[3], pr[2];
                if (!project(X[c], c ? K2 : K1, P + 3 * j, pc, pr)) { good = false; break; }
                const double dx = pr[0] - UV[4 * j + 2 * c], dy = pr[1] - UV[4 * j + 2 * c + 1];
                if (!(sqrt(dx * dx + dy * dy) < a.reproj_thresh)) good = false;
            }
            if (good) out_mask[list[j]] = 1;
        }
        n_valid += __popcll(__ballot(good));
    }
    if (lane == 0) {
        a.n_out[p] = n_valid;
        if (a.iters_out) a.iters_out[p] = iters;
        if (n_valid == 0) {  // no camera keeps a landmark: the verifier's pose (two_view_estimator.py:199-202)
            for (int k = 0; k < 9; ++k) a.R_out[9 * p + k] = a.R_in[9 * p + k];
            for (int k = 0; k < 3; ++k) a.t_out[3 * p + k] = a.t_in[3 * p + k];
            a.status_out[p] = 2;
        } else {
            double R[9], t[3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    R[3 * i + j] = X[1].R[i] * X[0].R[j] + X[1].R[3 + i] * X[0].R[3 + j] + X[1].R[6 + i] * X[0].R[6 + j];
            const double d[3] = {X[0].t[0] - X[1].t[0], X[0].t[1] - X[1].t[1], X[0].t[2] - X[1].t[2]};
            mtv3(X[1].R, d, t);
            const double nt = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
            for (int k = 0; k < 9; ++k) a.R_out[9 * p + k] = R[k];
            for (int k = 0; k < 3; ++k) a.t_out[3 * p + k] = t[k] / nt;
            a.status_out[p] = 0;
        }
    }
}

size_t ba2_layout(int n_pairs, int mcap, size_t* off) {
    const size_t n = (size_t)n_pairs * mcap;
    size_t o = 0;
    off[0] = o; o += gtsfm_align_up(n * 3 * sizeof(double), 256);
    off[1] = o; o += gtsfm_align_up(n * 3 * sizeof(double), 256);
    off[2] = o; o += gtsfm_align_up(n * 4 * sizeof(double), 256);
    off[3] = o; o += gtsfm_align_up(n * sizeof(int), 256);
    return o;
}

}  // namespace

extern "C" {

size_t gtsfm_ba2_workspace_bytes(int n_pairs, int mcap) {
    if (n_pairs <= 0 || mcap <= 0) return 0;
    size_t off[4];
    return ba2_layout(n_pairs, mcap, off);
}

int gtsfm_ba2_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax, const int* d_pairs,
                      int n_pairs, const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                      const uint8_t* d_in_mask, const double* d_R_in, const double* d_t_in, const int* d_status_in,
                      const double* d_prior_Rt, const double* d_prior_sigmas, int min_inliers, int max_iters,
                      double reproj_thresh, double tri_thresh, void* d_workspace,
                      size_t workspace_bytes, double* d_R_out, double* d_t_out, uint8_t* d_out_mask, int* d_n_out,
                      int* d_status_out, int* d_iters, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_kp_xy || !d_intrinsics || !d_pairs || !d_match_idx || !d_match_count || !d_in_mask || !d_R_in || !d_t_in ||
        !d_status_in || !d_workspace || !d_R_out || !d_t_out || !d_out_mask || !d_n_out || !d_status_out ||
        n_img <= 0 || kmax <= 0 || n_pairs < 0 || mcap <= 0 || max_iters < 0 || !(reproj_thresh > 0) ||
        !(tri_thresh > 0))
        return GTSFM_ERR_ARG;
    size_t off[4];
    if (workspace_bytes < ba2_layout(n_pairs, mcap, off)) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    Ba2Args a;
    a.kp_xy = d_kp_xy;
    a.intr = d_intrinsics;
    a.kmax = kmax;
    a.pairs = d_pairs;
    a.match_idx = (const uint2*)d_match_idx;
    a.match_count = d_match_count;
    a.mcap = mcap;
    a.in_mask = d_in_mask;
    a.R_in = d_R_in;
    a.t_in = d_t_in;
    a.status_in = d_status_in;
    a.prior_Rt = d_prior_Rt;
    a.prior_sig = d_prior_sigmas;
    a.min_inliers = min_inliers;
    a.max_iters = max_iters;
    a.reproj_thresh = reproj_thresh;
    a.tri_thresh = tri_thresh;
    a.P = (double*)(ws + off[0]);
    a.Pn = (double*)(ws + off[1]);
    a.UV = (double*)(ws + off[2]);
    a.list = (int*)(ws + off[3]);
    a.R_out = d_R_out;
    a.t_out = d_t_out;
    a.out_mask = d_out_mask;
    a.n_out = d_n_out;
    a.status_out = d_status_out;
    a.iters_out = d_iters;
    hipLaunchKernelGGL(ba2_kernel, dim3(n_pairs), dim3(64), 0, stream, a);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
