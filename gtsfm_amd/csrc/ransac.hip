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

#include <type_traits>

#include "common.hpp"

// Development instrumentation (off in the product build): -DGTSFM_RANSAC_PROF accumulates per-phase shader-clock
// cycles of every wave into g_rprof (vector global atomics from lane 0), read back with gtsfm_ransac_prof_read.
#ifdef GTSFM_RANSAC_PROF
__device__ unsigned long long g_rprof[32];
#define RPROF_DECL unsigned long long rprof_t = clock64();
#define RPROF(k)                                                              \
    do {                                                                      \
        const unsigned long long rprof_n = clock64();                         \
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_rprof[k], rprof_n - rprof_t); \
        rprof_t = rprof_n;                                                    \
    } while (0)
#define RPROF_COUNT(k, v) \
    do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_rprof[k], (unsigned long long)(v)); } while (0)
#else
#define RPROF_DECL
#define RPROF(k) do { } while (0)
#define RPROF_COUNT(k, v) do { } while (0)
#endif

// The essential-matrix path is compiled without FMA contraction: every fused multiply-add below is an explicit __builtin_fma()
// that oracle/ransac.c performs in the same place, so the solver, the refits and recoverPose reproduce the oracle's
// double arithmetic bit for bit (hypotheses, candidates, scores, the selected model, R and t).
#pragma clang fp contract(off)

namespace {

constexpr int kBatch = 64;      // hypotheses per chunk: the iteration bound is re-evaluated after each chunk
constexpr int kMaxGroups = 8;   // chunks one solve/score launch may cover
constexpr int kMaxHyp = kBatch * kMaxGroups;  // per-pair stride of the stage / nsol / cand buffers
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
        for (int j = 0; j < 4; ++j) q[kLL2Q[i][j]] = __builtin_fma(a[i], b[j], q[kLL2Q[i][j]]);
}

// c += s * q*l (oracle addmul_ql); s is 1, -1 or 2, so s * q[i] is exact and every term is one fused multiply-add
__device__ __forceinline__ void addmul_ql(const double* q, const double* l, double s, double* c) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const double sq = s * q[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) c[kQL2C[i][j]] = __builtin_fma(sq, l[j], c[kQL2C[i][j]]);
    }
}

// ------------------------------------------------------------------ lane-private arrays in LDS
// The solver's dynamically indexed arrays live in LDS, element i of lane l at base[i * 64 + l]: consecutive lanes hit
// consecutive words, so every access is bank-conflict free, and nothing spills to scratch. The solver runs in two
// kernels so each one's workgroup holds only its own phase's arrays:
//   stage 1 (sample, 5x9 null space in registers, 10x20 elimination), two lanes per hypothesis: rows 8..9 of this
//       lane's half of A (2 x 10; rows 0..7 in registers) = 10 KB per 64-lane workgroup;
//   stage 2 (det B(z), Sturm chain, isolation, bisection, E): the chain is built in registers (generic degrees;
//       a private-memory fallback for degree drops), the isolating intervals are selected into registers, and LDS
//       holds only the isolation stack as left ends (24 doubles + 24 count bytes) = 13.5 KB per workgroup, so
//       with <= 256 registers two waves share a SIMD.
constexpr int kLanes = 64;
// rows of the lane's half of A kept in registers (the rest in LDS): C2 solve1 per launch 364 / 330 / 330 / 323 us for
// 2 / 4 / 5 / 6 (profiles/r05an_*): each elimination step moves every LDS row through registers, and the register
// file has room (1 wave per SIMD either way: 314 VGPRs at 2, 406 at 6). With half-row construction and forward
// elimination + back-substitution: 298 / 285 / 266 / 263 / 256 us for 4 / 5 / 6 / 7 / 8 (profiles/r05aw_*); 9 and 10
// add more pivot-row selects (7292 / 7837 instructions against 6593 at 8)
constexpr int kRegRows = 8;
constexpr int kUnion = 10 * (10 - kRegRows);  // stage-1 doubles per lane: the LDS rows of the lane's half of A
constexpr int kStack = 24;    // == oracle/ransac.c ISO_STACK
constexpr int kRootDbl = kStack;  // stage-2 doubles per lane: the isolation stack's left ends
constexpr int kRootB = kStack;    // stage-2 bytes per lane: the stack's Sturm sign-variation counts
constexpr size_t kSolveLds = (size_t)kUnion * kLanes * sizeof(double);
constexpr size_t kRootLds = (size_t)kRootDbl * kLanes * sizeof(double) + (size_t)kRootB * kLanes;

template <typename T>
struct LaneArr {
    T* p;
    __device__ __forceinline__ T& operator[](int i) const { return p[i * kLanes]; }
    __device__ __forceinline__ LaneArr at(int off) const { return LaneArr{p + off * kLanes}; }
};

__device__ __forceinline__ double peval(LaneArr<double> p, int deg, double x) {
    double v = p[deg];
    for (int i = deg - 1; i >= 0; --i) v = __builtin_fma(v, x, p[i]);
    return v;
}

// r = a mod b (deg_a >= deg_b) using scratch t (11 entries); returns degree of r (-1 if zero)
__device__ int prem(LaneArr<double> a, int da, LaneArr<double> b, int db, LaneArr<double> r, LaneArr<double> t) {
    for (int i = 0; i <= da; ++i) t[i] = a[i];
    for (int k = da; k >= db; --k) {
        const double f = t[k] / b[db];
        for (int i = 0; i <= db; ++i) t[k - db + i] = __builtin_fma(-f, b[i], t[k - db + i]);
        t[k] = 0.0;
    }
    int dr = db - 1;
    double scale = 0.0;
    for (int i = 0; i <= da; ++i) scale = fmax(scale, fabs(a[i]));
    while (dr >= 0 && fabs(t[dr]) <= 1e-14 * scale) --dr;
    for (int i = 0; i <= dr; ++i) r[i] = t[i];
    return dr;
}

struct SolverMem {
    LaneArr<double> u;  // kUnion doubles
};

__device__ __forceinline__ SolverMem solver_mem(unsigned char* smem, int lane) {
    return SolverMem{LaneArr<double>{(double*)smem + lane}};
}

struct RootMem {
    LaneArr<double> u;     // kRootDbl doubles
    LaneArr<uint8_t> b;    // kRootB bytes
};

__device__ __forceinline__ RootMem root_mem(unsigned char* smem, int lane) {
    double* d = (double*)smem;
    uint8_t* b = smem + (size_t)kRootDbl * kLanes * sizeof(double);
    return RootMem{LaneArr<double>{d + lane}, LaneArr<uint8_t>{b + lane}};
}

// Register-resident Sturm chain: row k (degree <= 10 - k) at kRowOff[k], zero-padded to length 11 - k. Horner over
// the padded row equals Horner from the row's true degree bit for bit (leading zeros contribute exact zeros), and
// rows past the chain length evaluate to 0 and are skipped exactly like the oracle's loop bound.
constexpr int kChain = 66;
constexpr int kRootGroup = 4;  // root slots bisected / polished together (independent Horner chains)
__device__ __forceinline__ constexpr int row_off(int k) { return 11 * k - k * (k - 1) / 2; }

__device__ __forceinline__ int sign_changes_reg(const double (&R)[kChain], double x) {
    double v[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) {
        const int len = 11 - k, o = row_off(k);
        double a = R[o + len - 1];
#pragma unroll
        for (int i = len - 2; i >= 0; --i) a = __builtin_fma(a, x, R[o + i]);
        v[k] = a;
    }
    int c = 0;
    double prev = 0.0;
#pragma unroll
    for (int k = 0; k < 11; ++k) {
        if (v[k] != 0.0) {
            if (prev != 0.0 && ((v[k] < 0.0) != (prev < 0.0))) ++c;
            prev = v[k];
        }
    }
    return c;
}

__device__ __forceinline__ double peval1(const double (&R)[kChain], double x) {
    double a = R[row_off(1) + 9];
#pragma unroll
    for (int i = 8; i >= 0; --i) a = __builtin_fma(a, x, R[row_off(1) + i]);
    return a;
}

__device__ __forceinline__ double peval0(const double (&R)[kChain], double x) {
    double a = R[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) a = __builtin_fma(a, x, R[i]);
    return a;
}

// Sturm chain of p (degree <= 10), the rows of oracle/ransac.c real_roots, into the register chain R (row k
// zero-padded to 11 - k; rows past the chain's end 0). Generic case: p of degree 10 and every pseudo-remainder of
// degree exactly one less than its divisor, so every row's degree and every loop bound is a compile-time constant
// and the whole chain lives in registers. A lane whose polynomial leaves that pattern (a degree drop, a zero
// remainder) rebuilds the chain with run-time degrees in private memory, the oracle's loop verbatim. Both paths do
// the oracle's operations in the oracle's order.
__device__ __forceinline__ void sturm_chain_fallback(const double (&row0)[11], int deg, double (&R)[kChain]) {
    double S[11][11];
    int sd[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) S[0][i] = row0[i];
    sd[0] = deg;
    for (int i = 1; i <= deg; ++i) S[1][i - 1] = (double)i * row0[i];
    sd[1] = deg - 1;
    int n = 2;
    while (n < 11 && sd[n - 1] > 0) {
        const double* a = S[n - 2];
        const double* b = S[n - 1];
        const int da = sd[n - 2], db = sd[n - 1];
        double t[11];
        for (int i = 0; i <= da; ++i) t[i] = a[i];
        for (int k = da; k >= db; --k) {
            const double f = t[k] / b[db];
            for (int i = 0; i <= db; ++i) t[k - db + i] = __builtin_fma(-f, b[i], t[k - db + i]);
            t[k] = 0.0;
        }
        int dr = db - 1;
        double scale = 0.0;
        for (int i = 0; i <= da; ++i) scale = fmax(scale, fabs(a[i]));
        while (dr >= 0 && fabs(t[dr]) <= 1e-14 * scale) --dr;
        if (dr < 0) break;
        for (int i = 0; i <= dr; ++i) S[n][i] = -t[i];
        sd[n] = dr;
        n++;
    }
#pragma unroll
    for (int k = 0; k < 11; ++k)
#pragma unroll
        for (int i = 0; i < 11 - k; ++i) R[row_off(k) + i] = (k < n && i <= sd[k < n ? k : 0]) ? S[k][i] : 0.0;
}

// Real roots (ascending) of a degree <= 10 polynomial into xr[0..nr): Sturm isolation, then all isolating intervals
// bisected together to a relative width of 2^-20 and polished by 4 safeguarded Newton steps, the arithmetic of
// oracle/ransac.c real_roots. Isolation runs first and records the isolating intervals; all intervals are then
// bisected together (10 independent chains), so a wave never serialises one lane's bisection behind another's
// isolation step.
__device__ int real_roots(const double (&pin)[11], int deg, RootMem m, double (&xr)[kMaxSol]) {
    RPROF_DECL
    // the coefficients stay in registers: every index below is static (the degree only selects)
    double lead = pin[0];
#pragma unroll
    for (int i = 1; i < 11; ++i) lead = i == deg ? pin[i] : lead;
#pragma unroll
    for (int i = 10; i >= 1; --i) {
        if (i > deg) continue;
        if (i == deg && fabs(lead) <= 1e-300) {
            --deg;
            lead = pin[i - 1];
        }
    }
    if (deg <= 0) return 0;
    double R[kChain];
    double row0[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) row0[i] = i <= deg ? pin[i] / lead : 0.0;
    bool generic = deg == 10;
    {
#pragma unroll
        for (int i = 0; i < 11; ++i) R[i] = row0[i];
#pragma unroll
        for (int i = 1; i < 11; ++i) R[row_off(1) + i - 1] = (double)i * row0[i];
        // rows 2..10: row k = -(row k-2 mod row k-1), degrees 12-k / 11-k -> 10-k
#pragma unroll
        for (int k = 2; k < 11; ++k) {
            const int da = 12 - k, db = 11 - k;
            const int oa = row_off(k - 2), ob = row_off(k - 1);
            double t[13];
#pragma unroll
            for (int i = 0; i <= da; ++i) t[i] = R[oa + i];
#pragma unroll
            for (int kk = da; kk >= db; --kk) {
                const double f = t[kk] / R[ob + db];
#pragma unroll
                for (int i = 0; i <= db; ++i) t[kk - db + i] = __builtin_fma(-f, R[ob + i], t[kk - db + i]);
                t[kk] = 0.0;
            }
            double scale = 0.0;
#pragma unroll
            for (int i = 0; i <= da; ++i) scale = fmax(scale, fabs(R[oa + i]));
            generic = generic && fabs(t[db - 1]) > 1e-14 * scale;
#pragma unroll
            for (int i = 0; i <= db - 1; ++i) R[row_off(k) + i] = -t[i];
        }
    }
    if (!generic) sturm_chain_fallback(row0, deg, R);
    RPROF(7);
    // root bound (== oracle root_bound_pow2): exact exponent arithmetic, a power of two
    double bound;
    {
        int emax = -2000;
#pragma unroll
        for (int k = 1; k <= 10; ++k) {
            if (k > deg) continue;
            double mk = 0.0;
#pragma unroll
            for (int i = 0; i < 11; ++i) mk = i == deg - k ? fabs(R[i]) : mk;
            if (k == deg) mk *= 0.5;
            if (mk == 0.0) continue;
            int x;
            frexp(mk, &x);
            const int c = x >= 0 ? (x + k - 1) / k : -((-x) / k);
            emax = c > emax ? c : emax;
        }
        if (emax == -2000) emax = 0;
        bound = ldexp(1.0, emax + 1);
    }
    // isolation (depth-first, left interval first). The stack always partitions [left end of the top, bound] into
    // adjacent intervals, so an entry's right end (and its Sturm count) is the left end of the entry below it: only
    // left ends are stored. The isolating intervals are selected into registers.
    LaneArr<double> st_a = m.u;
    LaneArr<uint8_t> st_va = m.b;
    const int v_bound = sign_changes_reg(R, bound);
    double lo[kMaxSol], hi[kMaxSol];
#pragma unroll
    for (int k = 0; k < kMaxSol; ++k) lo[k] = hi[k] = 0.0;
    int ns = 1, nr = 0, guard = 0;
    st_a[0] = -bound;
    st_va[0] = (uint8_t)sign_changes_reg(R, -bound);
    while (ns > 0 && nr < kMaxSol && guard < 2000) {
        ++guard;
        --ns;
        const double a = st_a[ns];
        const int va = st_va[ns];
        const double b = ns > 0 ? st_a[ns > 0 ? ns - 1 : 0] : bound;
        const int vb = ns > 0 ? (int)st_va[ns > 0 ? ns - 1 : 0] : v_bound;
        const int cnt = va - vb;
        if (cnt <= 0) continue;
        if (cnt == 1 || b - a < 1e-10 * fmax(1.0, fabs(a))) {
#pragma unroll
            for (int k = 0; k < kMaxSol; ++k) {
                lo[k] = k == nr ? a : lo[k];
                hi[k] = k == nr ? b : hi[k];
            }
            ++nr;
            continue;
        }
        const double mid = 0.5 * (a + b);
        const int vm = sign_changes_reg(R, mid);
        if (ns + 2 <= kStack) {  // (mid, b) below (a, mid): left ends mid, a
            st_a[ns] = mid; st_va[ns] = (uint8_t)vm; ++ns;
            st_a[ns] = a; st_va[ns] = (uint8_t)va; ++ns;
        }
    }
    RPROF(8);
    RPROF_COUNT(20, guard);
    double flo[kMaxSol];
#pragma unroll
    for (int k = 0; k < kMaxSol; ++k) flo[k] = peval0(R, lo[k]);
    // all isolating intervals refined together (== oracle): bisection down to a relative width of 2^-20, then 4
    // safeguarded Newton steps with p' = Sturm row 1
    unsigned live = 0;
#pragma unroll
    for (int k = 0; k < kMaxSol; ++k) live |= (k < nr ? 1u : 0u) << k;
    const unsigned all_roots = live;
    // Slots are visited in groups of kRootGroup: a group is skipped only when no lane has a live root in it, and
    // inside a group every slot is evaluated unconditionally (results kept by `go`), so the group's Horner chains
    // are independent instructions the scheduler interleaves. Per slot the arithmetic is unchanged.
    for (int it = 0; it < 80; ++it) {
        if (!__any(live != 0)) break;
#pragma unroll
        for (int g = 0; g < kMaxSol; g += kRootGroup) {
            if (!__any((live >> g) & ((1u << kRootGroup) - 1u))) continue;
#pragma unroll
            for (int k = g; k < g + kRootGroup && k < kMaxSol; ++k) {
                const bool go =
                    ((live >> k) & 1u) && hi[k] - lo[k] > 0x1p-20 * fmax(1.0, fmax(fabs(lo[k]), fabs(hi[k])));
                if (!go) live &= ~(1u << k);
                const double mid = 0.5 * (lo[k] + hi[k]);
                const double fm = peval0(R, mid);
                const bool left = (fm < 0.0) == (flo[k] < 0.0) && fm != 0.0;
                lo[k] = go && left ? mid : lo[k];
                flo[k] = go && left ? fm : flo[k];
                hi[k] = go && !left ? mid : hi[k];
            }
        }
    }
    RPROF(9);
#pragma unroll
    for (int k = 0; k < kMaxSol; ++k) xr[k] = 0.5 * (lo[k] + hi[k]);
    live = all_roots;
    for (int it = 0; it < 4; ++it) {
#pragma unroll
        for (int g = 0; g < kMaxSol; g += kRootGroup) {
            if (!__any((live >> g) & ((1u << kRootGroup) - 1u))) continue;
#pragma unroll
            for (int k = g; k < g + kRootGroup && k < kMaxSol; ++k) {
                const double fx = peval0(R, xr[k]), dfx = peval1(R, xr[k]);
                const bool go = ((live >> k) & 1u) && fx != 0.0;
                if (!go) live &= ~(1u << k);
                const bool left = (fx < 0.0) == (flo[k] < 0.0);
                lo[k] = go && left ? xr[k] : lo[k];
                flo[k] = go && left ? fx : flo[k];
                hi[k] = go && !left ? xr[k] : hi[k];
                const double xn = xr[k] - fx / dfx;
                const double xs = (xn >= lo[k] && xn <= hi[k]) ? xn : 0.5 * (lo[k] + hi[k]);
                xr[k] = go ? xs : xr[k];
            }
        }
    }
    RPROF(10);
    RPROF_COUNT(21, nr);
    return nr;
}

// ------------------------------------------------------------------ Nister 5-point (one lane, arrays in LDS)
// Null space of the 5 x 9 epipolar system (oracle/ransac.c nullspace_5x9): Householder QR of its transpose,
// M^T = H_0 ... H_4 [R; 0], then columns 5..8 of H_0 ... H_4. Static indices only, so it stays in registers.
__device__ bool nullspace_5x9(const double* x1, const double* x2, double N[4][9]) {
    double a[5][9], v[5][9], beta[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
        a[i][0] = u2 * u1; a[i][1] = u2 * v1; a[i][2] = u2;
        a[i][3] = v2 * u1; a[i][4] = v2 * v1; a[i][5] = v2;
        a[i][6] = u1; a[i][7] = v1; a[i][8] = 1.0;
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        double sq = 0.0;
#pragma unroll
        for (int r = k; r < 9; ++r) sq = __builtin_fma(a[k][r], a[k][r], sq);
        const double nrm = sqrt(sq);
        ok = ok && !(nrm < 1e-12);
        const double alpha = a[k][k] >= 0.0 ? -nrm : nrm;
#pragma unroll
        for (int r = k; r < 9; ++r) v[k][r] = a[k][r];
        v[k][k] = v[k][k] - alpha;
        double vv = 0.0;
#pragma unroll
        for (int r = k; r < 9; ++r) vv = __builtin_fma(v[k][r], v[k][r], vv);
        beta[k] = 2.0 / vv;
#pragma unroll
        for (int c = k + 1; c < 5; ++c) {
            double d = 0.0;
#pragma unroll
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], a[c][r], d);
            d = d * beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) a[c][r] = __builtin_fma(-d, v[k][r], a[c][r]);
        }
    }
    if (!ok) return false;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        double y[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) y[j] = j == 5 + n ? 1.0 : 0.0;
#pragma unroll
        for (int k = 4; k >= 0; --k) {
            double d = 0.0;
#pragma unroll
            for (int r = k; r < 9; ++r) d = __builtin_fma(v[k][r], y[r], d);
            d = d * beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) y[r] = __builtin_fma(-d, v[k][r], y[r]);
        }
#pragma unroll
        for (int j = 0; j < 9; ++j) N[n][j] = y[j];
    }
    return true;
}

// Lanes 2k and 2k+1 solve one hypothesis together; the even lane holds columns 0..9 of the 10 x 20 matrix, the odd
// lane columns 10..19. Every pivot, pivot value and elimination factor comes from a column < 10, i.e. from the even
// lane, and reaches the odd one by a DPP quad permutation (no LDS, no waitcnt).
__device__ __forceinline__ int pair_lo(int v) { return __builtin_amdgcn_mov_dpp(v, 0xA0, 0xf, 0xf, false); }
__device__ __forceinline__ double pair_lo(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = pair_lo((int)(b & 0xffffffffll)), hi = pair_lo((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Nister 5-point, stage 1: 5 correspondences -> nullspace basis N (4 x 9) and rows 4..9, columns 10..19 of the
// Gauss-Jordan-reduced 10 x 20 constraint matrix (all that stage 2 reads; valid in the odd lane of the pair). The
// arithmetic per element is the single-lane elimination's, so the result is bit-identical to it. False for a
// degenerate sample (uniform over the pair).
//
// Each lane builds only its own ten columns, with the same code: read homogeneously in (x, y, z, w = 1), columns 0..9
// are the cubic monomials with at least two factors from {x, y} and 10..19 those with at least two from {z, w}, so
// the renaming (x, y, z, w) -> (z, w, x, y) maps the second set onto the first. The odd lane builds columns 0..9 of
// the constraint rows of the renamed E (each linear entry's coefficients [z w x y]) and so holds the original columns
// 10..19 in the order kHiCol below (oracle/ransac.c build_rows / oracle_five_point follow the same construction).
constexpr int kStageVals = 6 * 10 + 4 * 9;  // doubles handed from stage 1 to stage 2 per hypothesis
// original column (minus 10) of the odd lane's column k: xxx->zzz, yyy->1, xxy->zz, xyy->z, xxz->xzz, xx->yzz,
// yyz->x, yy->y, xyz->xz, xy->yz
constexpr int kHiCol[10] = {6, 9, 7, 8, 0, 3, 2, 5, 1, 4};

__device__ bool five_point_stage1(const double* x1, const double* x2, SolverMem m, int part, double N[4][9],
                                  double Rt[6][10]) {
    RPROF_DECL
    if (!nullspace_5x9(x1, x2, N)) return false;
    RPROF(1);
    double E[9][4];  // the odd lane's entries renamed: coefficients [z w x y]
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        E[e][0] = part ? N[2][e] : N[0][e];
        E[e][1] = part ? N[3][e] : N[1][e];
        E[e][2] = part ? N[0][e] : N[2][e];
        E[e][3] = part ? N[1][e] : N[3][e];
    }
    // This lane's half of A: rows 0..kRegRows-1 in registers (G), rows kRegRows..9 in LDS (A). Each row is
    // accumulated in registers (only columns 0..9 are live), then stored once.
    LaneArr<double> A = m.u.at(-10 * kRegRows);  // A[10 * r + j] for r >= kRegRows
    double G[kRegRows][10];
    auto store_row = [&](int r, const double(&row)[20]) {
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            if (r < kRegRows) G[r < kRegRows ? r : 0][k] = row[k];
            else A[10 * r + k] = row[k];
        }
    };
    double EEt[3][3][10], tr[10], tmp[10];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) {
#pragma unroll
            for (int mm = 0; mm < 10; ++mm) EEt[i][j][mm] = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mul_ll(E[3 * i + k], E[3 * j + k], tmp);
#pragma unroll
                for (int mm = 0; mm < 10; ++mm) EEt[i][j][mm] += tmp[mm];
            }
            if (j != i)
#pragma unroll
                for (int mm = 0; mm < 10; ++mm) EEt[j][i][mm] = EEt[i][j][mm];
        }
#pragma unroll
    for (int mm = 0; mm < 10; ++mm) tr[mm] = EEt[0][0][mm] + EEt[1][1][mm] + EEt[2][2][mm];
    // rows 9, 8, ..., 1, then the det row 0: the register rows are produced last (short live ranges)
#pragma unroll
    for (int ij = 8; ij >= 0; --ij) {
        const int i = ij / 3, j = ij % 3;
        double row[20];
#pragma unroll
        for (int k = 0; k < 20; ++k) row[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) addmul_ql(EEt[i][k], E[3 * k + j], 2.0, row);
        addmul_ql(tr, E[3 * i + j], -1.0, row);
        store_row(1 + ij, row);
    }
    {
        double row[20], q[10];
#pragma unroll
        for (int k = 0; k < 20; ++k) row[k] = 0.0;
        mul_ll(E[4], E[8], q); addmul_ql(q, E[0], 1.0, row);
        mul_ll(E[5], E[7], q); addmul_ql(q, E[0], -1.0, row);
        mul_ll(E[3], E[8], q); addmul_ql(q, E[1], -1.0, row);
        mul_ll(E[5], E[6], q); addmul_ql(q, E[1], 1.0, row);
        mul_ll(E[3], E[7], q); addmul_ql(q, E[2], 1.0, row);
        mul_ll(E[4], E[6], q); addmul_ql(q, E[2], -1.0, row);
        store_row(0, row);
    }
    RPROF(2);
    // Gaussian elimination with partial pivoting (Gauss-Jordan's pivots) on the lane's half rows, then back-substitution
    // of rows 4..9 (oracle/ransac.c oracle_five_point); every row is moved through registers whole. Row indices are
    // static except the pivot row pr, which is read / written through LDS or a register select.
    auto ld = [&](int r, int j) -> double { return r < kRegRows ? G[r < kRegRows ? r : 0][j] : A[10 * r + j]; };
    // one column step per call with a compile-time column (no dynamically indexed register rows)
    auto gj_step = [&](auto cc) -> bool {
        constexpr int c = decltype(cc)::value;
        int pr = c;
        double best = fabs(ld(c, c));  // meaningful in the even lane (column c)
#pragma unroll
        for (int r = c + 1; r < 10; ++r) {
            const double v = fabs(ld(r, c));
            if (v > best) { best = v; pr = r; }
        }
        pr = pair_lo(pr);
        best = pair_lo(best);
        if (best < 1e-14) return false;
        double prow[10];
        // pr >= c: only register rows c..kRegRows-1 can be the pivot (static bounds, fewer selects)
        if (c < kRegRows) {  // pr may be a register row
            const bool in_lds = pr >= kRegRows;
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                double v = in_lds ? A[10 * (in_lds ? pr : kRegRows) + j] : G[c < kRegRows ? c : 0][j];
#pragma unroll
                for (int q = c + 1; q < kRegRows; ++q) v = pr == q ? G[q][j] : v;
                prow[j] = v;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 10; ++j) prow[j] = A[10 * pr + j];
        }
        if (pr != c) {
            double crow[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) crow[j] = ld(c, j);
            if (pr >= kRegRows) {
#pragma unroll
                for (int j = 0; j < 10; ++j) A[10 * pr + j] = crow[j];
            } else {
#pragma unroll
                for (int q = c + 1; q < kRegRows; ++q)
#pragma unroll
                    for (int j = 0; j < 10; ++j) G[q][j] = pr == q ? crow[j] : G[q][j];
            }
        }
        const double inv = 1.0 / pair_lo(prow[c]);
#pragma unroll
        for (int j = 0; j < 10; ++j) prow[j] *= inv;
#pragma unroll
        for (int j = 0; j < 10; ++j) {
            if (c < kRegRows) G[c < kRegRows ? c : 0][j] = prow[j];
            else A[10 * c + j] = prow[j];
        }
#pragma unroll
        for (int r = c + 1; r < 10; ++r) {  // forward elimination only: rows 4..9 are back-substituted below
            double row[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) row[j] = ld(r, j);
            const double f = pair_lo(row[c]);
#pragma unroll
            for (int j = 0; j < 10; ++j) row[j] = __builtin_fma(-f, prow[j], row[j]);
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                if (r < kRegRows) G[r < kRegRows ? r : 0][j] = row[j];
                else A[10 * r + j] = row[j];
            }
        }
        return true;
    };
    using std::integral_constant;
    if (!gj_step(integral_constant<int, 0>{}) || !gj_step(integral_constant<int, 1>{}) ||
        !gj_step(integral_constant<int, 2>{}) || !gj_step(integral_constant<int, 3>{}) ||
        !gj_step(integral_constant<int, 4>{}) || !gj_step(integral_constant<int, 5>{}) ||
        !gj_step(integral_constant<int, 6>{}) || !gj_step(integral_constant<int, 7>{}) ||
        !gj_step(integral_constant<int, 8>{}) || !gj_step(integral_constant<int, 9>{}))
        return false;
    // back-substitution of rows 4..9 (all that stage 2 reads; rows 0..3 are dead after their forward step), each
    // pivot row fully reduced before it is used
#pragma unroll
    for (int c = 9; c >= 5; --c) {
        double prow[10];
#pragma unroll
        for (int j = 0; j < 10; ++j) prow[j] = ld(c, j);
#pragma unroll
        for (int r = 4; r < c; ++r) {
            double row[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) row[j] = ld(r, j);
            const double f = pair_lo(row[c]);
#pragma unroll
            for (int j = 0; j < 10; ++j) row[j] = __builtin_fma(-f, prow[j], row[j]);
#pragma unroll
            for (int j = 0; j < 10; ++j) {
                if (r < kRegRows) G[r < kRegRows ? r : 0][j] = row[j];
                else A[10 * r + j] = row[j];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int j = 0; j < 10; ++j) Rt[r][kHiCol[j]] = ld(4 + r, j);  // the odd lane's columns in original order
    RPROF(3);
    return true;
}

// Stage 2: the 3 x 3 polynomial matrix B(z) from the reduced rows, its degree-10 determinant, real roots, and up to
// 10 unit-norm E; on_sol(s, E) is called for each solution in root order.
// B(z) (3 x 3 polynomial matrix) from stage 1's reduced rows (`in`: this hypothesis' first stage value, stride
// kMaxHyp). Reads through a pointer the compiler cannot see through, so a second call reloads (from L2) instead of
// keeping B live across the root finder.
__device__ __forceinline__ void load_B(const double* in, double (&B)[3][3][5]) {
    uint64_t a = (uint64_t)in;
    asm volatile("" : "+v"(a));
    const double* q = (const double*)a;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double e[10], f[10];  // e[k] == A[4 + 2r][10 + k], f[k] == A[5 + 2r][10 + k]
#pragma unroll
        for (int j = 0; j < 10; ++j) {
            e[j] = q[(size_t)(10 * (2 * r) + j) * kMaxHyp];
            f[j] = q[(size_t)(10 * (2 * r + 1) + j) * kMaxHyp];
        }
        B[r][0][0] = e[2]; B[r][0][1] = e[1] - f[2]; B[r][0][2] = e[0] - f[1];
        B[r][0][3] = -f[0]; B[r][0][4] = 0.0;
        B[r][1][0] = e[5]; B[r][1][1] = e[4] - f[5]; B[r][1][2] = e[3] - f[4];
        B[r][1][3] = -f[3]; B[r][1][4] = 0.0;
        B[r][2][0] = e[9]; B[r][2][1] = e[8] - f[9]; B[r][2][2] = e[7] - f[8];
        B[r][2][3] = e[6] - f[7]; B[r][2][4] = -f[6];
    }
}

// Stage 2: the 3 x 3 polynomial matrix B(z) from the reduced rows, its degree-10 determinant, real roots, and up to
// 10 unit-norm E; on_sol(s, E) is called for each solution in root order. B and the null-space basis N are read
// from stage 1's output (`in`) before and after the root finder, so neither holds registers during it.
template <typename SolFn>
__device__ int five_point_stage2(const double* in, RootMem m, SolFn&& on_sol) {
    RPROF_DECL
    double n[11];
    {
        double B[3][3][5];
        load_B(in, B);
#pragma unroll
        for (int i = 0; i < 11; ++i) n[i] = 0.0;
        const int deg[3] = {3, 3, 4};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int c1 = (c + 1) % 3, c2 = (c + 2) % 3;
            double mm[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) mm[i] = 0.0;
#pragma unroll
            for (int i = 0; i <= deg[c1]; ++i)
#pragma unroll
                for (int j = 0; j <= deg[c2]; ++j) mm[i + j] = __builtin_fma(B[1][c1][i], B[2][c2][j], mm[i + j]);
#pragma unroll
            for (int i = 0; i <= deg[c2]; ++i)
#pragma unroll
                for (int j = 0; j <= deg[c1]; ++j) mm[i + j] = __builtin_fma(-B[1][c2][i], B[2][c1][j], mm[i + j]);
            const int dm = deg[c1] + deg[c2];
#pragma unroll
            for (int i = 0; i <= deg[c]; ++i)
#pragma unroll
                for (int j = 0; j <= dm; ++j) n[i + j] = __builtin_fma(B[0][c][i], mm[j], n[i + j]);
        }
    }
    RPROF(6);
    double xr[kMaxSol];
    const int nr = real_roots(n, 10, m, xr);
    double B[3][3][5], N[4][9];
    load_B(in, B);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 9; ++j) N[k][j] = in[(size_t)(60 + 9 * k + j) * kMaxHyp];
    int nsol = 0;
#pragma unroll
    for (int k = 0; k < kMaxSol; ++k) {
        if (!__any(k < nr)) break;
        if (k >= nr) continue;
        const double z = xr[k];
        double Bz[3][3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int dg = c == 2 ? 4 : 3;
                double v = B[r][c][dg];
#pragma unroll
                for (int i = dg - 1; i >= 0; --i) v = __builtin_fma(v, z, B[r][c][i]);
                Bz[r][c] = v;
            }
        double bx = 0, by = 0, bzz = 0, bn = -1.0;
#pragma unroll
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
        double Eo[9], nrm = 0.0;
#pragma unroll
        for (int e = 0; e < 9; ++e) {
            Eo[e] = x * N[0][e] + y * N[1][e] + z * N[2][e] + N[3][e];
            nrm += Eo[e] * Eo[e];
        }
        nrm = sqrt(nrm);
        if (!(nrm > 0.0)) continue;
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[e] /= nrm;
        on_sol(nsol, Eo);
        ++nsol;
    }
    RPROF(11);
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

// MSAC term of one correspondence (oracle/ransac.c msac_cost): the inlier test of sampson_inlier, then the squared
// Sampson error quantised to floor(e * 2^16 / thr^2) (<= 65535) for an inlier, 65536 for an outlier. Every operation
// is a single correctly rounded fp32 operation, so the integer matches the oracle's bit for bit.
__device__ __forceinline__ uint32_t msac_cost(const float* E, float4 p, float thr2, float scale, bool& in) {
    const float a0 = fmaf(E[1], p.y, fmaf(E[0], p.x, E[2]));
    const float a1 = fmaf(E[4], p.y, fmaf(E[3], p.x, E[5]));
    const float a2 = fmaf(E[7], p.y, fmaf(E[6], p.x, E[8]));
    const float b0 = fmaf(E[3], p.w, fmaf(E[0], p.z, E[6]));
    const float b1 = fmaf(E[4], p.w, fmaf(E[1], p.z, E[7]));
    const float num = fmaf(p.w, a1, fmaf(p.z, a0, a2));
    const float den = fmaf(b1, b1, fmaf(b0, b0, fmaf(a1, a1, __fmul_rn(a0, a0))));
    const float nn = __fmul_rn(num, num);
    in = nn <= __fmul_rn(thr2, den);
    if (!in) return 65536u;
    const float r = den > 0.0f ? __fdiv_rn(nn, den) : 0.0f;
    const float q = __fmul_rn(r, scale);
    return q < 65535.0f ? (uint32_t)q : 65535u;
}

// Two putatives per lane in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: one instruction for both): the same fused
// and rounded operations as msac_cost / sampson_inlier, component-wise, so each component is bit-identical to the
// scalar path. Only the division stays scalar.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <bool kMsac>
__device__ __forceinline__ void score2(const float (&E)[9], f2 x1, f2 y1, f2 x2, f2 y2, float thr2, float scale,
                                       uint32_t& bad, int& cnt) {
    const f2 a0 = pfma((f2)E[1], y1, pfma((f2)E[0], x1, (f2)E[2]));
    const f2 a1 = pfma((f2)E[4], y1, pfma((f2)E[3], x1, (f2)E[5]));
    const f2 a2 = pfma((f2)E[7], y1, pfma((f2)E[6], x1, (f2)E[8]));
    const f2 b0 = pfma((f2)E[3], y2, pfma((f2)E[0], x2, (f2)E[6]));
    const f2 b1 = pfma((f2)E[4], y2, pfma((f2)E[1], x2, (f2)E[7]));
    const f2 num = pfma(y2, a1, pfma(x2, a0, a2));
    const f2 den = pfma(b1, b1, pfma(b0, b0, pfma(a1, a1, a0 * a0)));
    const f2 nn = num * num;
    const f2 rhs = (f2)thr2 * den;
    const bool in0 = nn.x <= rhs.x, in1 = nn.y <= rhs.y;
    cnt += (in0 ? 1 : 0) + (in1 ? 1 : 0);
    if constexpr (kMsac) {
        f2 r;
        if (__all(fminf(den.x, den.y) >= 0x1p-60f)) {
            // nn / den correctly rounded: the compiler's division sequence (reciprocal, one Newton step on it, two
            // residual corrections) without its operand scaling and special-case fixup, which only act when an
            // operand or an intermediate leaves the normal range. Here den is in [2^-60, 16] and nn in [0, 16], so
            // for every quotient >= 2^-100 the result is the IEEE quotient bit for bit; a smaller one (nn near
            // underflow) may differ in its last bits, but both quantise to the same cost 0 (q scale < 2^-44).
            const f2 rc = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
            const f2 e = pfma(-den, rc, (f2)1.0f);
            const f2 rr = pfma(e, rc, rc);
            f2 q = nn * rr;
            const f2 e2 = pfma(-den, q, nn);
            q = pfma(e2, rr, q);
            const f2 e3 = pfma(-den, q, nn);
            r = pfma(e3, rr, q);
        } else {
            r = {den.x > 0.0f ? __fdiv_rn(nn.x, den.x) : 0.0f, den.y > 0.0f ? __fdiv_rn(nn.y, den.y) : 0.0f};
        }
        const f2 qq = r * (f2)scale;
        const uint32_t c0 = qq.x < 65535.0f ? (uint32_t)qq.x : 65535u;
        const uint32_t c1 = qq.y < 65535.0f ? (uint32_t)qq.y : 65535u;
        bad += (in0 ? c0 : 65536u) + (in1 ? c1 : 65536u);
    } else {
        bad += (in0 ? 0u : 1u) + (in1 ? 0u : 1u);
    }
}

// Wave-wide sum, uniform result: DPP prefix sum within each row of 16 (row_shr 1, 2, 4, 8), then row_bcast 15 / 31
// carry the row totals forward; lane 63 holds the total. Six VALU ops, no LDS crossbar traffic.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}

// Wave-wide MSAC score of E over M points (its inlier count in `count`).
__device__ uint32_t wave_msac(const float* E, const float4* pts, int M, float thr2, float scale, int& count,
                              int lane) {
    uint32_t sc = 0;
    int c = 0;
    for (int base = 0; base < M; base += 64) {
        const int i = base + lane;
        bool in = false;
        const uint32_t q = i < M ? msac_cost(E, pts[i], thr2, scale, in) : 0u;
        c += __popcll(__ballot(in));
        sc += wave_sum_u32(q);
    }
    count = c;
    return sc;
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

// ------------------------------------------------------------------ small dense linear algebra
// Cyclic Jacobi eigen-decomposition, the same rotation sequence as oracle/ransac.c jacobi_eig. N = 3: fully
// unrolled, register resident (redundant per lane).
template <int N>
__device__ __forceinline__ void jacobi_eig_reg(double (&a)[N * N], double (&w)[N], double (&V)[N * N]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) V[i * N + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = i + 1; j < N; ++j) off += a[i * N + j] * a[i * N + j];
        if (off < 1e-30) break;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p * N + q];
                if (fabs(apq) < 1e-300) continue;
                const double app = a[p * N + p], aqq = a[q * N + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double akp = a[k * N + p], akq = a[k * N + q];
                    a[k * N + p] = c * akp - s * akq;
                    a[k * N + q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double apk = a[p * N + k], aqk = a[q * N + k];
                    a[p * N + k] = c * apk - s * aqk;
                    a[q * N + k] = s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = c * vkp - s * vkq;
                    V[k * N + q] = s * vkp + c * vkq;
                }
            }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) w[i] = a[i * N + i];
}

// 9x9 Jacobi on a wave: a and V live in LDS, the rotation angles are computed redundantly by every lane (uniform
// control flow), the k-loops of one rotation run one k per lane. Element-wise identical to the oracle.
__device__ void jacobi9_lds(double* a, double* V, int lane) {
    constexpr int N = 9;
    for (int i = lane; i < N * N; i += 64) V[i] = (i / N == i % N) ? 1.0 : 0.0;
    __syncthreads();
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
        for (int i = 0; i < N; ++i)
            for (int j = i + 1; j < N; ++j) off += a[i * N + j] * a[i * N + j];
        if (off < 1e-30) break;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p * N + q];
                if (fabs(apq) < 1e-300) continue;
                const double app = a[p * N + p], aqq = a[q * N + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                __syncthreads();
                if (lane < N) {
                    const int k = lane;
                    const double akp = a[k * N + p], akq = a[k * N + q];
                    a[k * N + p] = c * akp - s * akq;
                    a[k * N + q] = s * akp + c * akq;
                }
                __syncthreads();
                if (lane < N) {
                    const int k = lane;
                    const double apk = a[p * N + k], aqk = a[q * N + k];
                    a[p * N + k] = c * apk - s * aqk;
                    a[q * N + k] = s * apk + c * aqk;
                } else if (lane < 2 * N) {
                    const int k = lane - N;
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = c * vkp - s * vkq;
                    V[k * N + q] = s * vkp + c * vkq;
                }
                __syncthreads();
            }
    }
}

__device__ void svd3(const double* E, double* U, double* s, double* V) {
    double ata[9], w[3], Vt[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += E[k * 3 + i] * E[k * 3 + j];
            ata[i * 3 + j] = acc;
        }
    jacobi_eig_reg<3>(ata, w, Vt);
    // descending order of w (selection by comparisons, same result as the oracle's index sort)
    int o0 = 0, o1 = 1, o2 = 2;
    if (w[o1] > w[o0]) { const int t = o0; o0 = o1; o1 = t; }
    if (w[o2] > w[o0]) { const int t = o0; o0 = o2; o2 = t; }
    if (w[o2] > w[o1]) { const int t = o1; o1 = o2; o2 = t; }
    const int order[3] = {o0, o1, o2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int oc = order[c];
        const double wc = oc == 0 ? w[0] : oc == 1 ? w[1] : w[2];
        s[c] = sqrt(fmax(wc, 0.0));
#pragma unroll
        for (int r = 0; r < 3; ++r) V[r * 3 + c] = oc == 0 ? Vt[r * 3] : oc == 1 ? Vt[r * 3 + 1] : Vt[r * 3 + 2];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        double u[3], nrm = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            u[r] = E[r * 3 + 0] * V[0 * 3 + c] + E[r * 3 + 1] * V[1 * 3 + c] + E[r * 3 + 2] * V[2 * 3 + c];
            nrm += u[r] * u[r];
        }
        nrm = sqrt(nrm);
#pragma unroll
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
    const double a0 = __builtin_fma(E[1], p1.y, __builtin_fma(E[0], p1.x, E[2]));
    const double a1 = __builtin_fma(E[4], p1.y, __builtin_fma(E[3], p1.x, E[5]));
    const double a2 = __builtin_fma(E[7], p1.y, __builtin_fma(E[6], p1.x, E[8]));
    const double b0 = __builtin_fma(E[3], p2.y, __builtin_fma(E[0], p2.x, E[6]));
    const double b1 = __builtin_fma(E[4], p2.y, __builtin_fma(E[1], p2.x, E[7]));
    const double num = __builtin_fma(p2.y, a1, __builtin_fma(p2.x, a0, a2));
    const double den = __builtin_fma(b1, b1, __builtin_fma(b0, b0, __builtin_fma(a1, a1, a0 * a0)));
    *den_out = den;
    return den > 0.0 ? num * num / den : 1e300;
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __shfl_xor((int)(u & 0xFFFFFFFFull), m), hi = __shfl_xor((int)(u >> 32), m);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Wave-wide fp64 sum, uniform result (read from lane 63): the DPP scan of wave_sum_u32 on the two halves of each
// double (row_shr 1, 2, 4, 8 inside rows of 16, then row_bcast 15 / 31), all VALU, no LDS permutes. A fixed order,
// so the result is deterministic.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
    const long long b = __double_as_longlong(v);
    int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    switch (ctrl_sel) {
        case 0: lo = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, false); break;
        case 1: lo = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xf, 0xf, false); break;
        case 2: lo = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xf, 0xf, false); break;
        case 3: lo = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xf, 0xf, false); break;
        case 4: lo = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xa, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xa, 0xf, false); break;
        default: lo = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xc, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xc, 0xf, false); break;
    }
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int c = 0; c < 6; ++c) v += dpp_f64(v, c);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Wave-cooperative Sampson-weighted 8-point refit (oracle/ransac.c refit_essential). The 45 unique normal-matrix
// entries are summed per lane (point i in lane i mod 64), then reduced across the wave by wave_sum_f64; the oracle
// forms the same partial sums and restates the reduction order (wave_sum_order), so the sums agree bit for bit.
__device__ bool wave_refit(const double2* x1, const double2* x2, int M, const double* Esel, double th2,
                           const uint8_t* sel, const double* Ew, double* Eout, int lane, double* jac_a,
                           double* jac_v) {
    double acc[45];
#pragma unroll
    for (int k = 0; k < 45; ++k) acc[k] = 0.0;
    int n = 0;
    for (int i = lane; i < M; i += 64) {
        double den;
        if (sel ? !sel[i] : sampson_sq(Esel, x1[i], x2[i], &den) > th2) continue;  // a label, or the threshold
        double dw;
        sampson_sq(Ew, x1[i], x2[i], &dw);
        const double w2 = dw > 1e-300 ? 1.0 / dw : 0.0;
        const double u1 = x1[i].x, v1 = x1[i].y, u2 = x2[i].x, v2 = x2[i].y;
        const double r[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
        int k = 0;
#pragma unroll
        for (int a = 0; a < 9; ++a) {
            const double wa = w2 * r[a];
#pragma unroll
            for (int b = a; b < 9; ++b, ++k) acc[k] = __builtin_fma(wa, r[b], acc[k]);
        }
        ++n;
    }
    for (int m = 32; m >= 1; m >>= 1) n += __shfl_xor(n, m);
    if (n < 8) return false;
#pragma unroll
    for (int k = 0; k < 45; ++k) acc[k] = wave_sum_f64(acc[k]);
    // Smallest eigenvector of the normal matrix: shifted inverse iteration on its Cholesky factor, register-resident
    // and computed redundantly by every lane (no LDS, no barriers). The shift (1e-12 of the trace) keeps the factor
    // positive definite; 8 iterations contract the other eigen-directions by ((l1 + s) / (l2 + s))^8. The oracle
    // runs the same iteration; the LDS Jacobi (oracle jacobi_eig) is the fallback of both when the factor breaks
    // down (uniform across the wave: every lane holds identical values).
    double E[9];
    {
        auto A = [&](int i, int j) -> double {  // full symmetric entry from the packed upper triangle (static)
            const int a = i < j ? i : j, b = i < j ? j : i;
            return acc[a * 9 - a * (a - 1) / 2 + (b - a)];
        };
        double tr = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) tr += A(i, i);
        const double shift = 1e-12 * tr;
        // The factor's diagonal is kept as reciprocals (nine divisions instead of 36 in the factorisation and 144 in
        // the eight inverse-iteration solves): fp64 division is a ~10-instruction sequence.
        double L[45];  // packed lower triangle, row i at i (i + 1) / 2; the diagonal entries hold 1 / L_ii
        bool ok = tr > 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                double v = A(i, j) + (i == j ? shift : 0.0);
#pragma unroll
                for (int k = 0; k < j; ++k) v = __builtin_fma(-L[i * (i + 1) / 2 + k], L[j * (j + 1) / 2 + k], v);
                if (i == j) {
                    ok = ok && v > 0.0;
                    L[i * (i + 1) / 2 + i] = 1.0 / sqrt(fmax(v, 1e-300));
                } else {
                    L[i * (i + 1) / 2 + j] = v * L[j * (j + 1) / 2 + j];
                }
            }
        if (ok) {
            double x[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) x[i] = 1.0;
            for (int it = 0; it < 8; ++it) {
#pragma unroll
                for (int i = 0; i < 9; ++i) {  // L y = x
                    double v = x[i];
#pragma unroll
                    for (int k = 0; k < i; ++k) v = __builtin_fma(-L[i * (i + 1) / 2 + k], x[k], v);
                    x[i] = v * L[i * (i + 1) / 2 + i];
                }
#pragma unroll
                for (int i = 8; i >= 0; --i) {  // L^T z = y
                    double v = x[i];
#pragma unroll
                    for (int k = i + 1; k < 9; ++k) v = __builtin_fma(-L[k * (k + 1) / 2 + i], x[k], v);
                    x[i] = v * L[i * (i + 1) / 2 + i];
                }
                double nrm = 0.0;
#pragma unroll
                for (int i = 0; i < 9; ++i) nrm = __builtin_fma(x[i], x[i], nrm);
                nrm = 1.0 / sqrt(nrm);
#pragma unroll
                for (int i = 0; i < 9; ++i) x[i] *= nrm;
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) E[k] = x[k];
        } else {
            if (lane < 45) {
                int a = 0, k = lane;
                while (k >= 9 - a) { k -= 9 - a; ++a; }
                const int b = a + k;
                double v = acc[0];
#pragma unroll
                for (int q = 1; q < 45; ++q) v = q == lane ? acc[q] : v;
                jac_a[a * 9 + b] = v;
                jac_a[b * 9 + a] = v;
            }
            __syncthreads();
            jacobi9_lds(jac_a, jac_v, lane);
            int imin = 0;
            double wmin = jac_a[0];
            for (int i = 1; i < 9; ++i)
                if (jac_a[i * 9 + i] < wmin) { wmin = jac_a[i * 9 + i]; imin = i; }
            for (int k = 0; k < 9; ++k) E[k] = jac_v[k * 9 + imin];
            __syncthreads();  // every lane has read the result before the LDS is reused
        }
    }
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

__device__ __attribute__((noinline)) int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmax(p, 0.0); p = fmin(p, 1.0);
    ep = fmax(ep, 0.0); ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - pow(1.0 - ep, (double)model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)llround(num / denom);
}

// The bound update_num_iters(p, (M - b) / M, 5, n) for every best count b, without the clamp to n: the caller's
// min(n, T[b]) equals `upd = update_num_iters(..., n); if (upd < n) n = upd` (the clamp test -num >= n * (-denom) and
// num / denom >= n differ only within rounding of a quotient <= 1000, never across a llround boundary).
__device__ int num_iters_bound(double p, double ep, int model_points) {
    p = fmax(p, 0.0); p = fmin(p, 1.0);
    ep = fmax(ep, 0.0); ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, 2.2250738585072014e-308);
    double denom = 1.0 - pow(1.0 - ep, (double)model_points);
    if (denom < 2.2250738585072014e-308) return 0;
    num = log(num);
    denom = log(denom);
    if (denom >= 0) return 0x7FFFFFFF;
    const double q = num / denom;
    return q >= 1073741824.0 ? 0x7FFFFFFF : (int)llround(q);
}

// ------------------------------------------------------------------ kernels
// Per pair, the iteration bound for every best count 0..M (table[p][b]), so the scoring loop needs no logarithms.
__global__ void ransac_bound_table_kernel(const int* __restrict__ match_count, int mcap, double prob,
                                          int* __restrict__ table) {
    const int p = blockIdx.y, b = blockIdx.x * blockDim.x + threadIdx.x;
    const int M = match_count[p];
    if (b > M || M < 6) return;
    table[(size_t)p * (mcap + 1) + b] = b > 0 ? num_iters_bound(prob, (double)(M - b) / M, 5) : 0x7FFFFFFF;
}

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

struct RansacOutputs {
    double* E;       // [P][9]
    double* R;       // [P][9]
    double* t;       // [P][3]
    int* n_inliers;  // [P]
    int* status;     // [P]: 0 ok, 1 too few putatives (M < 6), 2 no model
    int* n_hyp;      // [P] (may be null)
    uint8_t* mask;   // [P][mcap]
    int* n_models;   // [P] (may be null): candidate models scored (real 5-point solutions of the scored samples)
};

struct PairState {
    int best, best_h, best_s, done;  // best: inlier count of the selected model
    int niters, n_models;
    uint32_t best_score, pad2;       // MSAC score of the selected model (0xFFFFFFFF: none yet)
    double bestE[9];
    double pad3;
};

__global__ void ransac_init_kernel(PairState* __restrict__ st, int n_pairs, int max_iters) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pairs) return;
    PairState s{};
    s.best = -1;
    s.best_h = -1;
    s.best_s = -1;
    s.done = 0;
    s.niters = max_iters;
    s.best_score = 0xFFFFFFFFu;
    st[p] = s;
}

// Stage 1, two 64-lane workgroups per chunk of an active pair (blockIdx.y = half of a chunk): lanes 2k, 2k+1 sample
// hypothesis h = done + 32 blockIdx.y + k, both run the nullspace, and split the 10 x 20 elimination by column halves;
// N (even lane) + the reduced rows (odd lane) go to stage 2 through `stage` ([P][kStageVals][kMaxHyp],
// hypothesis-minor). nsol = 1 marks a non-degenerate sample for stage 2, 0 a finished one. A launch covers
// gridDim.y / 2 chunks; a chunk that starts at or past the pair's current iteration bound is skipped (the bound only
// falls, so the score kernel never reaches it).
__global__ __launch_bounds__(64, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void ransac_solve1_kernel(const int* __restrict__ match_count, int mcap,
                                                              const double2* __restrict__ x1n_all,
                                                              const double2* __restrict__ x2n_all, uint64_t seed,
                                                              int pair_id_base, const int* __restrict__ pair_ids,
                                                              const PairState* __restrict__ st,
                                                              double* __restrict__ stage, int* __restrict__ nsol) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int p = blockIdx.x, lane = threadIdx.x;
    const int part = lane & 1, hyp = blockIdx.y * (kLanes / 2) + (lane >> 1);
    const int M = match_count[p];
    if (M < 6) return;
    const int done = st[p].done;
    if (done + (hyp & ~(kBatch - 1)) >= st[p].niters) return;
    const double2* x1 = x1n_all + (size_t)p * mcap;
    const double2* x2 = x2n_all + (size_t)p * mcap;
    const SolverMem mem = solver_mem(smem, lane);
    RPROF_DECL
    RPROF_COUNT(16, 1);
    int ok = 0;
    int idx[5];
    if (sample5(seed, pair_ids ? pair_ids[p] : pair_id_base + p, done + hyp, M, idx)) {
        double s1[10], s2[10];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const double2 a = x1[idx[k]], b = x2[idx[k]];
            s1[2 * k] = a.x; s1[2 * k + 1] = a.y;
            s2[2 * k] = b.x; s2[2 * k + 1] = b.y;
        }
        double N[4][9], Rt[6][10];
        RPROF(0);
        if (five_point_stage1(s1, s2, mem, part, N, Rt)) {
            ok = 1;
            double* out = stage + (size_t)p * kStageVals * kMaxHyp + hyp;
            if (part) {
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int j = 0; j < 10; ++j) out[(10 * r + j) * kMaxHyp] = Rt[r][j];
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < 9; ++j) out[(60 + 9 * k + j) * kMaxHyp] = N[k][j];
            }
        }
    }
    if (!part) nsol[(size_t)p * kMaxHyp + hyp] = ok;
    RPROF(4);
}

// Stage 2, one 64-lane workgroup per chunk of an active pair (blockIdx.y = chunk): lane l turns stage 1's output into
// the candidate essential matrices of hypothesis done + 64 blockIdx.y + l (fp64) -> cand, nsol.
__global__ __launch_bounds__(64, 2) void ransac_solve2_kernel(const int* __restrict__ match_count,
                                                              const PairState* __restrict__ st,
                                                              const double* __restrict__ stage,
                                                              double* __restrict__ cand, int* __restrict__ nsol) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int p = blockIdx.x, lane = threadIdx.x;
    const int M = match_count[p];
    if (M < 6) return;
    const int hyp = blockIdx.y * kBatch + lane;
    if (st[p].done + (int)blockIdx.y * kBatch >= st[p].niters) return;
    int* ns_out = nsol + (size_t)p * kMaxHyp + hyp;
    if (*ns_out == 0) return;  // degenerate sample: stays 0
    const RootMem mem = root_mem(smem, lane);
    RPROF_DECL
    RPROF_COUNT(17, 1);
    const double* in = stage + (size_t)p * kStageVals * kMaxHyp + hyp;
    // candidates hypothesis-minor, [P][kMaxSol][9][kMaxHyp]: the lanes' stores of one element are contiguous
    double* cout = cand + (size_t)p * kMaxSol * 9 * kMaxHyp + hyp;
    RPROF(5);
    const int ns = five_point_stage2(in, mem, [&](int s, const double* E) {
#pragma unroll
        for (int e = 0; e < 9; ++e) cout[(size_t)(9 * s + e) * kMaxHyp] = E[e];
    });
    *ns_out = ns;
    RPROF(12);
}

// Pair order for the one-workgroup-per-pair launches (score, refine): pairs by putative count, largest first
// (counting sort on 1024 count bins; order within a bin unspecified), so the longest workgroups start first and the
// launch does not end on a large pair dispatched last. Outputs do not depend on the order.
constexpr int kOrderBins = 1024;
__global__ __launch_bounds__(kOrderBins) void pair_order_kernel(const int* __restrict__ match_count, int n_pairs,
                                                                 int mcap, int* __restrict__ order) {
    __shared__ int cnt[kOrderBins];
    int shift = 0;
    while ((mcap >> shift) >= kOrderBins) ++shift;
    const int tid = threadIdx.x;
    cnt[tid] = 0;
    __syncthreads();
    for (int p = tid; p < n_pairs; p += kOrderBins)
        atomicAdd(&cnt[kOrderBins - 1 - (min(max(match_count[p], 0), mcap) >> shift)], 1);  // descending
    __syncthreads();
    // inclusive scan (Hillis-Steele), then exclusive starts
    for (int d = 1; d < kOrderBins; d <<= 1) {
        const int v = tid >= d ? cnt[tid - d] : 0;
        __syncthreads();
        cnt[tid] += v;
        __syncthreads();
    }
    const int start = tid ? cnt[tid - 1] : 0;
    __syncthreads();
    cnt[tid] = start;
    __syncthreads();
    for (int p = tid; p < n_pairs; p += kOrderBins)
        order[atomicAdd(&cnt[kOrderBins - 1 - (min(max(match_count[p], 0), mcap) >> shift)], 1)] = p;
}

// Scoring, one workgroup of kScoreThreads lanes per active pair and launch, LANE PER CANDIDATE: the candidates of the
// launch's chunks (flattened in (hypothesis, solution) order, the oracle's scan order) are dealt to the lanes, and
// every lane walks all putatives of its own candidate in index order, reading each putative as one broadcast LDS
// load. No cross-lane reduction sits on the per-point path. The per-point terms are the oracle's (msac_cost /
// sampson_inlier), integer sums, so the order of evaluation cannot change a score.
// Selection is exactly the oracle's sequential scan (oracle/ransac.c:716-740: a candidate replaces the best only with
// a strictly lower MSAC score / strictly more inliers, so the first in order wins a tie): every candidate carries the
// 64-bit key (badness << 32 | flat index + 1 << 19 | inlier count) with badness = MSAC score or outlier count, and the
// winner is the smallest key. A lane drops its candidate as soon as its partial badness (which only grows) shows that
// it cannot beat the best key among the pre-launch best and the finished candidates of chunks <= its own (`pref`):
// such a candidate can be neither its chunk's prefix minimum nor the chunk minimum that the walk below needs. After
// all lanes finish, thread 0 walks the chunks in order exactly like the oracle's batch loop
// (oracle/ransac.c:679-706): best = min(best, chunk minimum), the iteration bound from the best count, done += 64,
// stop once done >= niters (chunks past that point were solved speculatively and are discarded).
// measured 64 / 128 / 256 / 512: 11.9 / 9.1 / 7.8 / 7.4 ms C2 verify; with largest-first pairs 256 / 512 / 1024:
// 360 / 284 / 318 us per C2 launch (profiles/r05_late_ablations/r05cc_*)
constexpr int kScoreThreads = 512;
constexpr int kMaxCand = kMaxHyp * kMaxSol;  // candidates one launch may hold per pair (13 bits of the key)
static_assert(kMaxCand < (1 << 13), "flat candidate index must fit the key's 13 bits");
constexpr int kKeyCountBits = 19;

template <bool kLds, bool kMsac, int kS>
__global__ __launch_bounds__(kScoreThreads) void ransac_score_kernel(const int* __restrict__ pairs,
                                                                    const double* __restrict__ intr,
                                                                    const int* __restrict__ match_count, int mcap,
                                                                    const float4* __restrict__ pts_all,
                                                                    double thr_px, double prob,
                                                                    const double* __restrict__ cand,
                                                                    const int* __restrict__ nsol, int n_chunks,
                                                                    const int* __restrict__ bound_tab,
                                                                    PairState* __restrict__ st,
                                                                    const int* __restrict__ order) {
    extern __shared__ float4 spts[];  // [M]
    __shared__ int flat_off[kMaxHyp + 1];       // candidates of the launch's hypotheses < h
    __shared__ uint16_t hyp_of[kMaxCand];       // flat candidate -> hypothesis slot of the launch
    __shared__ int chunk_tot[kMaxGroups];
    __shared__ unsigned long long chunk_min[kMaxGroups], pref[kMaxGroups];
    const int p = order[blockIdx.x], tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int M = match_count[p];
    if (M < 6) return;
    int best = st[p].best, best_h = st[p].best_h, best_s = st[p].best_s, done = st[p].done, niters = st[p].niters;
    int n_models = st[p].n_models;
    uint32_t best_score = st[p].best_score;
    if (done >= niters) return;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const double fx = fmax(intr[3 * i1], intr[3 * i2]);  // opencv_verifier_base.py:86
    const double thr = thr_px / fx;
    const float thr2 = (float)(thr * thr);
    const float scale = __fdiv_rn(65536.0f, thr2);
    const float4* pts = pts_all + (size_t)p * mcap;
    // kLds: the putatives are staged in LDS in pair blocks, block j = {x1, y1, x2, y2} of points 2j and 2j + 1 as
    // (a, b) pairs ({x1a, x1b, y1a, y1b}, {x2a, x2b, y2a, y2b}), so the packed evaluation reads its operand pairs
    // straight into register pairs
    float* spf = (float*)spts;
    if (kLds)
        for (int i = tid; i < M; i += kScoreThreads) {
            const float4 v = pts[i];
            float* b = spf + 8 * (i >> 1) + (i & 1);
            b[0] = v.x; b[2] = v.y; b[4] = v.z; b[6] = v.w;
        }
    auto point = [&](int i) -> float4 {
        if (!kLds) return pts[i];
        const float* b = spf + 8 * (i >> 1) + (i & 1);
        return make_float4(b[0], b[2], b[4], b[6]);
    };
    RPROF_DECL
    RPROF_COUNT(18, 1);
    // flattened candidate offsets over the chunks the solver kernels processed (those starting below niters)
    const size_t hbase = (size_t)p * kMaxHyp;
    for (int c = wave; c < n_chunks; c += kScoreThreads / 64) {
        int v = done + c * kBatch < niters ? nsol[hbase + c * kBatch + lane] : 0;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const int o = __shfl_up(v, m);
            if (lane >= m) v += o;
        }
        flat_off[c * kBatch + lane + 1] = v;
        if (lane == 63) chunk_tot[c] = v;
    }
    // the pre-launch best as a key (flat index 0: before every candidate of this launch)
    const uint32_t prev_bad = kMsac ? best_score : (best < 0 ? 0xFFFFFFFFu : (uint32_t)(M - best));
    const unsigned long long prev_key = ((unsigned long long)prev_bad << 32) | (uint32_t)(best < 0 ? 0 : best);
    if (tid < kMaxGroups) {
        chunk_min[tid] = ~0ull;
        pref[tid] = prev_key;
    }
    if (tid == 0) flat_off[0] = 0;
    __syncthreads();
    for (int h = tid; h < n_chunks * kBatch; h += kScoreThreads) {
        int off = 0;
        for (int j = 0; j < (h >> 6); ++j) off += chunk_tot[j];
        flat_off[h + 1] += off;
    }
    __syncthreads();
    for (int h = tid; h < n_chunks * kBatch; h += kScoreThreads) {
        const int o = h == 0 ? 0 : flat_off[h], e = flat_off[h + 1];
        for (int k = o; k < e; ++k) hyp_of[k] = (uint16_t)h;
    }
    __syncthreads();
    const int total = flat_off[n_chunks * kBatch];
    RPROF(14);
    auto finish = [&](int c, uint32_t myid, uint32_t bad, int cnt) {
        const unsigned long long key = ((unsigned long long)bad << 32) |
                                       ((unsigned long long)myid << kKeyCountBits) | (unsigned long long)cnt;
        atomicMin(&chunk_min[c], key);
        for (int j = c; j < n_chunks; ++j) atomicMin(&pref[j], key);
    };
    // one block of up to four putatives (block b = points 4b .. 4b + 3), packed pairs when the block is full
    auto block = [&](const float (&E)[9], int b, uint32_t& bad, int& cnt) {
        const int base = 4 * b;
        if (base + 4 <= M) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f2 x1, y1, x2, y2;
                if (kLds) {
                    const float4 lo = ((const float4*)spf)[(base >> 1) * 2 + 2 * h];
                    const float4 hi = ((const float4*)spf)[(base >> 1) * 2 + 2 * h + 1];
                    x1 = {lo.x, lo.y}; y1 = {lo.z, lo.w}; x2 = {hi.x, hi.y}; y2 = {hi.z, hi.w};
                } else {
                    const float4 a = pts[base + 2 * h], q = pts[base + 2 * h + 1];
                    x1 = {a.x, q.x}; y1 = {a.y, q.y}; x2 = {a.z, q.z}; y2 = {a.w, q.w};
                }
                score2<kMsac>(E, x1, y1, x2, y2, thr2, scale, bad, cnt);
            }
            return;
        }
        for (int u = base; u < M; ++u) {
            const float4 q = point(u);
            if constexpr (kMsac) {
                bool in;
                bad += msac_cost(E, q, thr2, scale, in);
                cnt += in ? 1 : 0;
            } else {
                const bool in = sampson_inlier(E, q, thr2);
                cnt += in ? 1 : 0;
                bad += in ? 0u : 1u;
            }
        }
    };
    auto load_E = [&](int ci, float (&E)[9], int& c) {
        const int h = hyp_of[ci];
        c = h >> 6;
        const double* ch = cand + (hbase * kMaxSol * 9 + (size_t)9 * (ci - flat_off[h]) * kMaxHyp) + h;
#pragma unroll
        for (int k = 0; k < 9; ++k) E[k] = (float)ch[(size_t)k * kMaxHyp];
    };
    // kS lanes per candidate (a power of two <= 64, aligned groups inside a wave): lane `sub` of the group takes the
    // point blocks sub, sub + kS, ...; the group's partial badness (a butterfly sum over its lanes) drives the exact
    // pruning test and the final key. kS = 1 for launches with many pairs; the host picks kS = 16 when a launch's
    // candidates alone would not fill the GPU (few pairs with many putatives, e.g. C1's 66 pairs of ~2000).
    const int sub = tid & (kS - 1), grp = tid / kS;
    auto gsum = [&](uint32_t v) {
#pragma unroll
        for (int m = 1; m < kS; m <<= 1) v += (uint32_t)__shfl_xor((int)v, m);
        return v;
    };
    const int nb = (M + 3) >> 2, n_it = (nb + kS - 1) / kS;
#pragma unroll 1
    for (int ci = grp; ci < total; ci += kScoreThreads / kS) {
        float E[9];
        int c;
        load_E(ci, E, c);
        const uint32_t myid = (uint32_t)ci + 1u;
        uint32_t bad = 0;  // MSAC: partial score; RANSAC: outliers so far (this lane's blocks)
        int cnt = 0;
        bool alive = true;
#pragma unroll 1
        for (int it = 0; it < n_it; ++it) {
            unsigned long long pk = __atomic_load_n(&pref[c], __ATOMIC_RELAXED);
            if constexpr (kS > 1) {  // one lane's read for the whole group: the prune decision is provably uniform
                const int src = (tid & 63) & ~(kS - 1);
                const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)pk, src), hi = (uint32_t)__shfl((int)(pk >> 32), src);
                pk = ((unsigned long long)hi << 32) | lo;
            }
            const uint32_t pb = (uint32_t)(pk >> 32), pid = (uint32_t)(pk >> kKeyCountBits) & 0x1FFFu;
            const uint32_t gb = gsum(bad);  // uniform over the group
            if (gb > pb || (gb == pb && myid > pid)) {
                alive = false;
                break;
            }
            const int b = it * kS + sub;
            if (b < nb) block(E, b, bad, cnt);
        }
        bad = gsum(bad);
        cnt = (int)gsum((uint32_t)cnt);
        if (alive && sub == 0) finish(c, myid, bad, cnt);
    }
    RPROF(13);
    __syncthreads();
    if (tid == 0) {
        long best_off = -1;  // cand offset of a winner found by this launch
        unsigned long long cur = prev_key;
        for (int c = 0; c < n_chunks && done < niters; ++c) {
            const unsigned long long k = chunk_min[c];
            if (k < cur) {  // a candidate of this chunk beat the best so far
                cur = k;
                const int ci = (int)((k >> kKeyCountBits) & 0x1FFFu) - 1;
                const int h = hyp_of[ci], sI = ci - flat_off[h];
                best = (int)(k & ((1u << kKeyCountBits) - 1u));
                if (kMsac) best_score = (uint32_t)(k >> 32);
                best_h = done + (h & (kBatch - 1));
                best_s = sI;
                best_off = (long)(hbase * kMaxSol * 9 + (size_t)9 * sI * kMaxHyp + h);
            }
            if (best > 0) niters = min(niters, bound_tab[(size_t)p * (mcap + 1) + best]);
            n_models += flat_off[(c + 1) * kBatch] - flat_off[c * kBatch];
            done += kBatch;
        }
        PairState& o = st[p];
        o.best = best;
        o.best_h = best_h;
        o.best_s = best_s;
        o.done = done;
        o.niters = niters;
        o.n_models = n_models;
        o.best_score = best_score;
        if (best_off >= 0)
            for (int e = 0; e < 9; ++e) o.bestE[e] = cand[best_off + (size_t)e * kMaxHyp];
    }
}

// ------------------------------------------------------------------ graph-cut LO (GC-RANSAC, oracle/ransac.c gc_label)
// The MSAC path's local optimisation: label every putative inlier / outlier by the minimum s-t cut of the truncated
// quadratic energy with spatial coherence over a 4-D grid of (x1, y1, x2, y2), refit on the labelled points, keep the
// refit while its MSAC score drops. Same-cell neighbours make the graph a union of cliques whose minimum cut has a
// closed form (the oracle's header proves it): sort by (cell, MSAC term, index), then per run of one cell the m lowest
// terms are the inliers for the m minimising the integer energy 2 E(m). Pairs above kGcMaxM keep the iterative LO.
constexpr int kGcIters = 10;
constexpr double kGcCellThr = 12.5;  // grid cell side in inlier thresholds (50 px at 4 px)
constexpr long long kGcLamNum = 39, kGcLamDen = 40;
constexpr int kGcMaxM = 32768;       // the sort key's 15-bit index
constexpr int kGcLdsKeys = 2048;     // pairs with up to this many putatives sort in LDS (18 KB), larger ones in HBM

__device__ __forceinline__ uint32_t gc_cell_key(float4 p, double inv_cell) {
    const float c[4] = {p.x, p.y, p.z, p.w};
    uint32_t k = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) k = (k << 8) | ((uint32_t)((int)floor((double)c[d] * inv_cell) + 128) & 0xFFu);
    return k;
}

// Labels (lab[i] = 1: inlier) of the M putatives under E; returns their number (uniform). keys: 2^ceil(log2 M) u64
// of scratch. Sort key = cell << 32 | MSAC term << 15 | index, bitonic-sorted by the wave in place.
__device__ __forceinline__ int wave_gc_label(const float* Ef, const float4* pts, int M, float thr2, float scale,
                                             double inv_cell, unsigned long long* keys, uint8_t* lab, int lane) {
    int n2 = 1;
    while (n2 < M) n2 <<= 1;
    for (int i = lane; i < n2; i += 64) {
        unsigned long long k = ~0ull;
        if (i < M) {
            bool in;
            const uint32_t q = msac_cost(Ef, pts[i], thr2, scale, in);
            k = ((unsigned long long)gc_cell_key(pts[i], inv_cell) << 32) | ((unsigned long long)q << 15) |
                (unsigned long long)i;
            lab[i] = 0;
        }
        keys[i] = k;
    }
    __syncthreads();
#ifdef GTSFM_RANSAC_PROF
    const unsigned long long gc_t0 = clock64();
#endif
    for (int kk = 2; kk <= n2; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < n2; i += 64) {
                const int l = i ^ j;
                if (l > i) {
                    const unsigned long long a = keys[i], b = keys[l];
                    if ((a > b) == ((i & kk) == 0)) {
                        keys[i] = b;
                        keys[l] = a;
                    }
                }
            }
            __syncthreads();
        }
#ifdef GTSFM_RANSAC_PROF
    if (lane == 0) atomicAdd(&g_rprof[29], clock64() - gc_t0);
#endif
    // every run head (first element of a cell) scans its run: prefix sums of the MSAC terms and 2 E(m) for all m
    int n_in = 0;
    const long long Q = 65536;
    for (int i = lane; i < M; i += 64) {
        const unsigned long long ki = keys[i];
        if (i > 0 && (keys[i - 1] >> 32) == (ki >> 32)) continue;
        long long sum = 0;
        int b = i;
        while (b < M && (keys[b] >> 32) == (ki >> 32)) sum += (long long)((keys[b++] >> 15) & 0x1FFFFu);
        const long long k = b - i;
        long long best = LLONG_MAX, pre = 0;
        int best_m = 0;
        for (long long m = 0; m <= k; ++m) {
            if (m > 0) pre += (long long)((keys[i + m - 1] >> 15) & 0x1FFFFu);
            const long long t = k - m, post = sum - pre;
            const long long U = 2 * pre + 2 * (t * Q - post);
            const long long P = (m > 0 ? (m - 1) * pre : 0) + t * (t - 1) * Q - (t > 0 ? (t - 1) * post : 0) +
                                2 * m * t * Q;
            const long long e = (kGcLamDen - kGcLamNum) * U + kGcLamNum * P;
            if (e < best) {
                best = e;
                best_m = (int)m;
            }
        }
        for (int m = 0; m < best_m; ++m) lab[keys[i + m] & 0x7FFFu] = 1;
        n_in += best_m;
    }
    __syncthreads();
    for (int m = 32; m >= 1; m >>= 1) n_in += __shfl_xor(n_in, m);
    return n_in;
}

// Per pair: status, LO from the best hypothesis (graph-cut for MSAC, iterative for RANSAC), final mask, recoverPose.
// two waves per SIMD (256 VGPRs, 22 spilled): 0.92 -> 0.73 ms per C2 step against one
__global__ __launch_bounds__(64, 2) void ransac_refine_kernel(const int* __restrict__ pairs,
                                                           const double* __restrict__ intr,
                                                           const int* __restrict__ match_count, int mcap,
                                                           const double2* __restrict__ x1n_all,
                                                           const double2* __restrict__ x2n_all,
                                                           const float4* __restrict__ pts_all, double thr_px,
                                                           int msac, RansacOutputs out,
                                                           const PairState* __restrict__ st,
                                                           unsigned char* __restrict__ gc_scratch,
                                                           size_t gc_stride, const int* __restrict__ order) {
    __shared__ double jac_a[81], jac_v[81];
    __shared__ unsigned long long gc_keys_lds[kGcLdsKeys];
    __shared__ uint8_t gc_lab_lds[kGcLdsKeys];
    const int p = order[blockIdx.x];
    const int lane = threadIdx.x;
    const int M = match_count[p];
    uint8_t* mask = out.mask + (size_t)p * mcap;
    if (M < 6) {  // opencv_verifier_base.py:69-78
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 1;
            if (out.n_hyp) out.n_hyp[p] = 0;
            if (out.n_models) out.n_models[p] = 0;
        }
        for (int i = lane; i < M; i += 64) mask[i] = 0;
        return;
    }
    RPROF_DECL
    const PairState ps = st[p];
    if (ps.best <= 0) {
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 2;
            if (out.n_hyp) out.n_hyp[p] = ps.done;
            if (out.n_models) out.n_models[p] = ps.n_models;
        }
        for (int i = lane; i < M; i += 64) mask[i] = 0;
        return;
    }
    const int done = ps.done;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const double fx = fmax(intr[3 * i1], intr[3 * i2]);
    const double thr = thr_px / fx;
    const float thr2 = (float)(thr * thr);
    const double2* x1 = x1n_all + (size_t)p * mcap;
    const double2* x2 = x2n_all + (size_t)p * mcap;
    const float4* pts = pts_all + (size_t)p * mcap;
    double bestE[9];
    for (int e = 0; e < 9; ++e) bestE[e] = ps.bestE[e];
    // iterative LO (oracle/ransac.c): thresholds kLoMult*thr -> thr, Sampson-weighted refits
    const float scale = __fdiv_rn(65536.0f, thr2);
    auto count_d = [&](const double* Ed) {
        float Ef[9];
        for (int e = 0; e < 9; ++e) Ef[e] = (float)Ed[e];
        return wave_count(Ef, pts, M, thr2, -1, lane);
    };
    auto msac_d = [&](const double* Ed, int& cnt) {
        float Ef[9];
        for (int e = 0; e < 9; ++e) Ef[e] = (float)Ed[e];
        return wave_msac(Ef, pts, M, thr2, scale, cnt, lane);
    };
    // a refit replaces the model when it has at least as many inliers (RANSAC) / a score no higher (MSAC)
    int cur = 0;
    uint32_t cur_sc = 0;
    if (msac)
        cur_sc = msac_d(bestE, cur);
    else
        cur = count_d(bestE);
    RPROF(22);
    const bool gc = msac && M <= kGcMaxM;
    if (gc) {  // graph-cut LO (oracle_ransac_E: the MSAC path)
        int n2 = 1;
        while (n2 < M) n2 <<= 1;
        const bool in_lds = n2 <= kGcLdsKeys;
        unsigned long long* keys = in_lds ? gc_keys_lds : (unsigned long long*)(gc_scratch + (size_t)p * gc_stride);
        uint8_t* lab = in_lds ? gc_lab_lds : (uint8_t*)(keys + n2);
        const double inv_cell = 1.0 / (kGcCellThr * thr);
        for (int g = 0; g < kGcIters; ++g) {
            float Ef[9];
            for (int e = 0; e < 9; ++e) Ef[e] = (float)bestE[e];
            const int n_lab = in_lds ? wave_gc_label(Ef, pts, M, thr2, scale, inv_cell, gc_keys_lds, gc_lab_lds, lane)
                                     : wave_gc_label(Ef, pts, M, thr2, scale, inv_cell, keys, lab, lane);
            RPROF(23);
            RPROF_COUNT(28, 1);
            if (n_lab < 8) break;
            double En[9];
            if (!wave_refit(x1, x2, M, nullptr, 0.0, lab, bestE, En, lane, jac_a, jac_v)) break;
            bool ok = true;
            for (int r = 1; r < kLoIrls && ok; ++r) {
                double Et[9];
                ok = wave_refit(x1, x2, M, nullptr, 0.0, lab, En, Et, lane, jac_a, jac_v);
                if (ok)
                    for (int e = 0; e < 9; ++e) En[e] = Et[e];
            }
            RPROF(24);
            int c;
            const uint32_t sc = msac_d(En, c);
            RPROF(25);
            if (sc >= cur_sc) break;
            cur_sc = sc;
            cur = c;
            for (int e = 0; e < 9; ++e) bestE[e] = En[e];
        }
    } else {
        double E[9];
        for (int e = 0; e < 9; ++e) E[e] = bestE[e];
        for (int k = 0; k < kLoSteps; ++k) {
            const double th = thr * (kLoMult - (kLoMult - 1.0) * k / (kLoSteps - 1));
            double Esel[9], En[9];
            for (int e = 0; e < 9; ++e) Esel[e] = E[e];
            if (!wave_refit(x1, x2, M, Esel, th * th, nullptr, Esel, En, lane, jac_a, jac_v)) break;
            bool ok = true;
            for (int r = 1; r < kLoIrls && ok; ++r) {
                double Et[9];
                ok = wave_refit(x1, x2, M, Esel, th * th, nullptr, En, Et, lane, jac_a, jac_v);
                if (ok)
                    for (int e = 0; e < 9; ++e) En[e] = Et[e];
            }
            int c;
            bool better;
            if (msac) {
                const uint32_t sc = msac_d(En, c);
                better = sc <= cur_sc;
                if (better) cur_sc = sc;
            } else {
                c = count_d(En);
                better = c >= cur;
            }
            for (int e = 0; e < 9; ++e) E[e] = En[e];
            if (better) {
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
    RPROF(26);
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
        if (out.n_models) out.n_models[p] = ps.n_models;
    }
    RPROF(27);
}

}  // namespace

extern "C" {

static size_t ransac_layout(int n_pairs, int mcap, size_t* off_x2, size_t* off_pts, size_t* off_st, size_t* off_cand,
                            size_t* off_nsol, size_t* off_stage) {
    const size_t n = (size_t)n_pairs * mcap;
    size_t o = 0;
    o += gtsfm_align_up(n * sizeof(double2), 256);
    *off_x2 = o;
    o += gtsfm_align_up(n * sizeof(double2), 256);
    *off_pts = o;
    o += gtsfm_align_up(n * sizeof(float4), 256);
    *off_st = o;
    o += gtsfm_align_up((size_t)n_pairs * sizeof(PairState), 256);
    *off_cand = o;
    o += gtsfm_align_up((size_t)n_pairs * kMaxHyp * kMaxSol * 9 * sizeof(double), 256);
    *off_nsol = o;
    o += gtsfm_align_up((size_t)n_pairs * kMaxHyp * sizeof(int), 256);
    *off_stage = o;
    o += gtsfm_align_up((size_t)n_pairs * kStageVals * kMaxHyp * sizeof(double), 256);
    o += gtsfm_align_up((size_t)n_pairs * (mcap + 1) * sizeof(int), 256);  // bound table
    o += gtsfm_align_up((size_t)n_pairs * sizeof(int), 256);               // pair order (last)
    return o;
}

#ifdef GTSFM_RANSAC_PROF
int gtsfm_ransac_prof_read(unsigned long long* out, int reset) {
    GTSFM_CHECK_HIP(hipDeviceSynchronize());
    GTSFM_CHECK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rprof), sizeof(unsigned long long) * 32));
    if (reset) {
        static const unsigned long long zeros[32] = {};
        GTSFM_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rprof), zeros, sizeof(zeros)));
    }
    return GTSFM_OK;
}
#endif

size_t gtsfm_ransac_workspace_bytes(int n_pairs, int mcap) {
    if (n_pairs <= 0 || mcap <= 0) return 0;
    size_t a, b, c, d, e, f;
    return ransac_layout(n_pairs, mcap, &a, &b, &c, &d, &e, &f);
}

int gtsfm_ransac_E_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax, const int* d_pairs,
                           int n_pairs, const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                           double thr_px, double prob, int max_iters, int scoring, uint64_t seed, int pair_id_base,
                           const int* d_pair_ids, void* d_workspace, size_t workspace_bytes, double* d_E, double* d_R, double* d_t,
                           int* d_n_inliers, int* d_status, int* d_n_hyp, int* d_n_models, uint8_t* d_inlier_mask,
                           void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_kp_xy || !d_intrinsics || !d_pairs || !d_match_idx || !d_match_count || !d_E || !d_R || !d_t ||
        !d_n_inliers || !d_status || !d_inlier_mask || n_img <= 0 || kmax <= 0 || n_pairs < 0 || mcap <= 0 ||
        max_iters <= 0 || !(thr_px > 0.0) ||
        (scoring != GTSFM_RANSAC_SCORING_RANSAC && scoring != GTSFM_RANSAC_SCORING_MSAC))
        return GTSFM_ERR_ARG;
    const bool msac = scoring == GTSFM_RANSAC_SCORING_MSAC;
    // selection key widths (ransac_score_kernel): the inlier count holds kKeyCountBits bits, and an MSAC score (at
    // most 65536 per putative) must not wrap its 32 bits
    if (mcap >= (1 << kKeyCountBits) || (msac && mcap > 65535)) return GTSFM_ERR_ARG;
    size_t o_x2, o_pts, o_st, o_cand, o_nsol, o_stage;
    const size_t need = ransac_layout(n_pairs, mcap, &o_x2, &o_pts, &o_st, &o_cand, &o_nsol, &o_stage);
    if (workspace_bytes < need) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    double2* x1n = (double2*)ws;
    double2* x2n = (double2*)(ws + o_x2);
    float4* pts = (float4*)(ws + o_pts);
    PairState* st = (PairState*)(ws + o_st);
    double* cand = (double*)(ws + o_cand);
    int* nsol = (int*)(ws + o_nsol);
    double* stage = (double*)(ws + o_stage);
    int* bound_tab = (int*)(ws + o_stage + gtsfm_align_up((size_t)n_pairs * kStageVals * kMaxHyp * sizeof(double), 256));
    int* order = bound_tab + gtsfm_align_up((size_t)n_pairs * (mcap + 1) * sizeof(int), 256) / sizeof(int);
    hipLaunchKernelGGL(ransac_bound_table_kernel, dim3((mcap + 1 + 255) / 256, n_pairs), dim3(256), 0, stream,
                       d_match_count, mcap, prob, bound_tab);
    hipLaunchKernelGGL(normalize_putatives_kernel, dim3((mcap + 255) / 256, n_pairs), dim3(256), 0, stream, d_kp_xy,
                       d_intrinsics, kmax, d_pairs, d_match_idx, d_match_count, mcap, x1n, x2n, pts);
    hipLaunchKernelGGL(ransac_init_kernel, dim3((n_pairs + 255) / 256), dim3(256), 0, stream, st, n_pairs, max_iters);
    hipLaunchKernelGGL(pair_order_kernel, dim3(1), dim3(kOrderBins), 0, stream, d_match_count, n_pairs, mcap, order);
    GTSFM_CHECK_HIP(hipGetLastError());
    GTSFM_CHECK_HIP(gtsfm_set_dynamic_lds((const void*)ransac_solve1_kernel, (int)kSolveLds));
    // the score kernel stages a pair's putatives in LDS when they fit (16 B each, up to 136 KiB beside its tables)
    const size_t score_pts = (size_t)((mcap + 1) & ~1) * sizeof(float4);  // pair blocks of 32 B
    const bool score_in_lds = score_pts <= 136 * 1024;
    const size_t score_lds = score_in_lds ? score_pts : 0;
    // lanes per candidate: 1, unless the launch's candidates (~272 per pair and chunk) would leave most of the GPU's
    // lanes idle while each walks many putatives
    const bool wide = (size_t)n_pairs * 272 < (size_t)64 * 1024 * 2 && mcap >= 256;
    using ScoreFn = void (*)(const int*, const double*, const int*, int, const float4*, double, double, const double*,
                             const int*, int, const int*, PairState*, const int*);
    ScoreFn score_fn;
    if (wide)
        score_fn = score_in_lds ? (msac ? ransac_score_kernel<true, true, 16> : ransac_score_kernel<true, false, 16>)
                                : (msac ? ransac_score_kernel<false, true, 16> : ransac_score_kernel<false, false, 16>);
    else
        score_fn = score_in_lds ? (msac ? ransac_score_kernel<true, true, 1> : ransac_score_kernel<true, false, 1>)
                                : (msac ? ransac_score_kernel<false, true, 1> : ransac_score_kernel<false, false, 1>);
    if (score_lds > 65536) GTSFM_CHECK_HIP(gtsfm_set_dynamic_lds((const void*)score_fn, (int)score_lds));
    // Chunks of 64 hypotheses, as the oracle; launches cover 1, 1, 2, 4, 8, 8, ... chunks. Most pairs stop within the
    // first two chunks; the pairs that run on are few, so their later chunks are solved together (speculatively: a
    // chunk the score kernel does not reach is discarded) to give the solver kernels enough waves.
    // A small batch (e.g. one rank's share of C2 at 8 GPUs: 619 pairs) leaves most of the GPU idle in those first
    // one-chunk launches and pays each launch's latency: launches then cover 2, 4, 8, 8, ... chunks (the extra
    // chunks are speculative, exactly as later launches' are: n_hyp and the selected model do not change).
    const int n_batches = (max_iters + kBatch - 1) / kBatch;
    const bool small = (size_t)n_pairs * (kBatch / (kLanes / 2)) < 2048;  // solve1 workgroups of a one-chunk launch
    for (int b = 0, g = 1, launch = 0; b < n_batches; b += g, ++launch) {
        g = small ? std::min(kMaxGroups, 2 << launch) : launch < 2 ? 1 : std::min(kMaxGroups, 1 << (launch - 1));
        g = std::min(g, n_batches - b);
        hipLaunchKernelGGL(ransac_solve1_kernel, dim3(n_pairs, g * kBatch / (kLanes / 2)), dim3(64), kSolveLds, stream,
                           d_match_count, mcap, x1n, x2n, seed, pair_id_base, d_pair_ids, st, stage, nsol);
        hipLaunchKernelGGL(ransac_solve2_kernel, dim3(n_pairs, g), dim3(64), kRootLds, stream, d_match_count, st,
                           stage, cand, nsol);
        hipLaunchKernelGGL(score_fn, dim3(n_pairs), dim3(kScoreThreads), score_lds, stream, d_pairs, d_intrinsics,
                           d_match_count, mcap, pts, thr_px, prob, cand, nsol, g, bound_tab, st, order);
    }
    GTSFM_CHECK_HIP(hipGetLastError());
    const RansacOutputs o{d_E, d_R, d_t, d_n_inliers, d_status, d_n_hyp, d_inlier_mask, d_n_models};
    // the graph-cut LO sorts in the stage buffer (free once the solver loop is done): 2^ceil(log2 M) keys + M labels
    static_assert((size_t)kStageVals * kMaxHyp * sizeof(double) >= (size_t)kGcMaxM * 9, "GC scratch fits the stage");
    hipLaunchKernelGGL(ransac_refine_kernel, dim3(n_pairs), dim3(64), 0, stream, d_pairs, d_intrinsics, d_match_count,
                       mcap, x1n, x2n, pts, thr_px, msac ? 1 : 0, o, st, (unsigned char*)stage,
                       (size_t)kStageVals * kMaxHyp * sizeof(double), order);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"

// ====================================================================================================================
// Fundamental-matrix verifier (use_intrinsics_in_verification=False): the restatement in oracle/fundamental.c of
// cv2.findFundamentalMat(FM_RANSAC, px, 0.999999, 1e6) (frontend/verifier/ransac.py:84-111) + E = K2^T F K1
// (utils/verification.py:97-110) + recoverPose (utils/verification.py:52-94). Everything below is compiled without
// FMA contraction and performs the oracle's double operations in the oracle's order, so the GPU reproduces the
// oracle's samples, minimal models, errors, counts and the final F bit for bit.
// ====================================================================================================================
#pragma clang fp contract(off)
namespace {

constexpr int kFBatch = 64;
constexpr int kFAttempts = 4;
constexpr int kFDraws = 16;
constexpr int kFMaxSol = 3;
constexpr float kFltEps = 1.19209290e-07f;
constexpr double kDblEps = 2.220446049250313e-16;

__device__ __forceinline__ bool fm_collinear3(float ax, float ay, float bx, float by, float cx, float cy) {
    const float dx1 = bx - ax, dy1 = by - ay, dx2 = cx - ax, dy2 = cy - ay;
    return fabsf(dx2 * dy1 - dy2 * dx1) <= kFltEps * (fabsf(dx1) + fabsf(dy1) + fabsf(dx2) + fabsf(dy2));
}

// 7 distinct indices without a collinear triple in either image (oracle_sample7)
__device__ bool sample7(uint64_t seed, int pair, int h, int M, const float4* __restrict__ pts, int* idx) {
    const uint64_t key = sm_mix(seed ^ sm_mix((uint64_t)(uint32_t)pair));
    for (int a = 0; a < kFAttempts; ++a) {
        int n = 0;
        for (int d = 0; d < kFDraws && n < 7; ++d) {
            const uint64_t r = sm_mix(key + ((uint64_t)h * kFAttempts + (uint64_t)a) * kFDraws + (uint64_t)d);
            const int v = (int)(((r >> 32) * (uint64_t)(uint32_t)M) >> 32);
            bool dup = false;
            for (int k = 0; k < n; ++k) dup |= (idx[k] == v);
            if (!dup) idx[n++] = v;
        }
        if (n < 7) continue;
        float4 q[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) q[k] = pts[idx[k]];
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 7; ++i)
#pragma unroll
            for (int j = i + 1; j < 7; ++j)
#pragma unroll
                for (int k = j + 1; k < 7; ++k)
                    bad |= fm_collinear3(q[i].x, q[i].y, q[j].x, q[j].y, q[k].x, q[k].y) ||
                           fm_collinear3(q[i].z, q[i].w, q[j].z, q[j].w, q[k].z, q[k].w);
        if (!bad) return true;
    }
    return false;
}

__device__ __forceinline__ double fm_cubic_eval(const double* a, double x) { return ((x + a[0]) * x + a[1]) * x + a[2]; }

__device__ int fm_bisect(const double* a, double lo, double hi, double* root) {
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

__device__ int fm_solve_cubic(const double* c, double* r) {
    const double m = fmax(fmax(fabs(c[0]), fabs(c[1])), fmax(fabs(c[2]), fabs(c[3])));
    if (!(m > 0.0)) return 0;
    if (fabs(c[0]) <= 1e-12 * m) {
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
    const double a[3] = {c[1] / c[0], c[2] / c[0], c[3] / c[0]};
    const double B = 1.0 + fmax(fabs(a[0]), fmax(fabs(a[1]), fabs(a[2])));
    const double disc = a[0] * a[0] - 3.0 * a[1];
    int n = 0;
    if (disc <= 0.0) return fm_bisect(a, -B, B, r);
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

// F = T2^T Fn T1 (Hartley de-normalisation), scaled so F33 = 1 when |F33| > DBL_EPSILON
__device__ __forceinline__ void fm_denormalize(const double* Fn, double s1, double c1x, double c1y, double s2,
                                               double c2x, double c2y, double* F) {
    const double T1[9] = {s1, 0.0, -s1 * c1x, 0.0, s1, -s1 * c1y, 0.0, 0.0, 1.0};
    const double T2[9] = {s2, 0.0, -s2 * c2x, 0.0, s2, -s2 * c2y, 0.0, 0.0, 1.0};
    double G[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
            G[3 * r + cc] = Fn[3 * r + 0] * T1[0 * 3 + cc] + Fn[3 * r + 1] * T1[1 * 3 + cc] + Fn[3 * r + 2] * T1[2 * 3 + cc];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
            F[3 * r + cc] = T2[0 * 3 + r] * G[0 * 3 + cc] + T2[1 * 3 + r] * G[1 * 3 + cc] + T2[2 * 3 + r] * G[2 * 3 + cc];
    if (fabs(F[8]) > kDblEps) {
        const double inv = 1.0 / F[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) F[i] = F[i] * inv;
        F[8] = 1.0;
    }
}

// 7-point solver (oracle_seven_point); the 7x9 system stays in registers (row swaps by selects)
__device__ int seven_point(const float4* __restrict__ pts, const int* idx, double* Fs) {
    float4 q[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) q[k] = pts[idx[k]];
    double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        c1x += q[k].x; c1y += q[k].y; c2x += q[k].z; c2y += q[k].w;
    }
    c1x /= 7.0; c1y /= 7.0; c2x /= 7.0; c2y /= 7.0;
    double d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double ax = q[k].x - c1x, ay = q[k].y - c1y, bx = q[k].z - c2x, by = q[k].w - c2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return 0;
    const double s1 = 1.4142135623730951 * 7.0 / d1, s2 = 1.4142135623730951 * 7.0 / d2;
    double A[7][9];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double u1 = (q[k].x - c1x) * s1, v1 = (q[k].y - c1y) * s1;
        const double u2 = (q[k].z - c2x) * s2, v2 = (q[k].w - c2y) * s2;
        A[k][0] = u2 * u1; A[k][1] = u2 * v1; A[k][2] = u2;
        A[k][3] = v2 * u1; A[k][4] = v2 * v1; A[k][5] = v2;
        A[k][6] = u1; A[k][7] = v1; A[k][8] = 1.0;
    }
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        int pr = c;
        double best = fabs(A[c][c]);
#pragma unroll
        for (int r = c + 1; r < 7; ++r)
            if (fabs(A[r][c]) > best) { best = fabs(A[r][c]); pr = r; }
        if (!(best > 1e-10)) return 0;
#pragma unroll
        for (int r = c + 1; r < 7; ++r) {
            const bool sw = (r == pr);
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const double a = A[c][j], b = A[r][j];
                A[c][j] = sw ? b : a;
                A[r][j] = sw ? a : b;
            }
        }
        const double inv = 1.0 / A[c][c];
#pragma unroll
        for (int j = 0; j < 9; ++j) A[c][j] = A[c][j] * inv;
#pragma unroll
        for (int r = 0; r < 7; ++r) {
            if (r == c) continue;
            const double f = A[r][c];
#pragma unroll
            for (int j = 0; j < 9; ++j) A[r][j] = A[r][j] - f * A[c][j];
        }
    }
    double f1[9], f2[9];
#pragma unroll
    for (int r = 0; r < 7; ++r) { f1[r] = -A[r][7]; f2[r] = -A[r][8]; }
    f1[7] = 1.0; f1[8] = 0.0;
    f2[7] = 0.0; f2[8] = 1.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) f1[i] = f1[i] - f2[i];
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
    for (int k = 0; k < nr; ++k) {
        double Fn[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) Fn[i] = roots[k] * f1[i] + f2[i];
        fm_denormalize(Fn, s1, c1x, c1y, s2, c2x, c2y, Fs + 9 * k);
    }
    return nr;
}

// FMEstimatorCallback::computeError (oracle_f_error)
__device__ __forceinline__ float fm_error(const double* F, float4 p) {
    const double x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
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

// inlier count of F at thr2, -1 once it provably cannot exceed floor_count
__device__ int fm_wave_count(const double* F, const float4* __restrict__ pts, int M, float thr2, int floor_count,
                             int lane) {
    int c = 0;
    for (int base = 0; base < M; base += 64) {
        const int i = base + lane;
        bool in = false;
        if (i < M) in = fm_error(F, pts[i]) <= thr2;
        c += __popcll(__ballot(in));
        const int remaining = M - (base + 64);
        if (remaining > 0 && c + remaining <= floor_count) return -1;
    }
    return c;
}

// serial cyclic Jacobi (oracle fm_jacobi), one lane
template <int N>
__device__ void fm_jacobi(double* a, double* w, double* V) {
    for (int i = 0; i < N * N; ++i) V[i] = 0.0;
    for (int i = 0; i < N; ++i) V[i * N + i] = 1.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) off += a[p * N + q] * a[p * N + q];
        if (!(off > 1e-300)) break;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p * N + q];
                if (fabs(apq) < 1e-300) continue;
                const double theta = (a[q * N + q] - a[p * N + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < N; ++k) {
                    const double akp = a[k * N + p], akq = a[k * N + q];
                    a[k * N + p] = c * akp - sn * akq;
                    a[k * N + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < N; ++k) {
                    const double apk = a[p * N + k], aqk = a[q * N + k];
                    a[p * N + k] = c * apk - sn * aqk;
                    a[q * N + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = c * vkp - sn * vkq;
                    V[k * N + q] = sn * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < N; ++i) w[i] = a[i * N + i];
}

// normalised 8-point on the masked correspondences (oracle_eight_point), one lane, arrays in LDS scratch
__device__ bool eight_point_serial(const float4* __restrict__ pts, const uint8_t* __restrict__ mask, int M,
                                   double* AtA /*81*/, double* V /*81*/, double* F) {
    int n = 0;
    double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float4 p = pts[i];
        c1x += p.x; c1y += p.y; c2x += p.z; c2y += p.w;
        ++n;
    }
    if (n < 8) return false;
    c1x /= n; c1y /= n; c2x /= n; c2y /= n;
    double d1 = 0.0, d2 = 0.0;
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float4 p = pts[i];
        const double ax = p.x - c1x, ay = p.y - c1y, bx = p.z - c2x, by = p.w - c2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return false;
    const double s1 = 1.4142135623730951 * n / d1, s2 = 1.4142135623730951 * n / d2;
    for (int k = 0; k < 81; ++k) AtA[k] = 0.0;
    for (int i = 0; i < M; ++i) {
        if (!mask[i]) continue;
        const float4 p = pts[i];
        const double u1 = (p.x - c1x) * s1, v1 = (p.y - c1y) * s1;
        const double u2 = (p.z - c2x) * s2, v2 = (p.w - c2y) * s2;
        const double r[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
            for (int b = a; b < 9; ++b) AtA[a * 9 + b] = AtA[a * 9 + b] + r[a] * r[b];
    }
    for (int a = 0; a < 9; ++a)
        for (int b = 0; b < a; ++b) AtA[a * 9 + b] = AtA[b * 9 + a];
    double w[9];
    fm_jacobi<9>(AtA, w, V);
    int kmin = 0;
    for (int k = 1; k < 9; ++k)
        if (w[k] < w[kmin]) kmin = k;
    double Fn[9];
    for (int e = 0; e < 9; ++e) Fn[e] = V[e * 9 + kmin];
    double FtF[9], w3[3], V3[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            FtF[a * 3 + b] = Fn[0 * 3 + a] * Fn[0 * 3 + b] + Fn[1 * 3 + a] * Fn[1 * 3 + b] + Fn[2 * 3 + a] * Fn[2 * 3 + b];
    fm_jacobi<3>(FtF, w3, V3);
    int k3 = 0;
    for (int k = 1; k < 3; ++k)
        if (w3[k] < w3[k3]) k3 = k;
    const double v[3] = {V3[0 * 3 + k3], V3[1 * 3 + k3], V3[2 * 3 + k3]};
    for (int r = 0; r < 3; ++r) {
        const double fv = Fn[3 * r] * v[0] + Fn[3 * r + 1] * v[1] + Fn[3 * r + 2] * v[2];
        for (int c = 0; c < 3; ++c) Fn[3 * r + c] = Fn[3 * r + c] - fv * v[c];
    }
    fm_denormalize(Fn, s1, c1x, c1y, s2, c2x, c2y, F);
    return true;
}

// Gather the putatives of every pair: pixel float4 (x1, y1, x2, y2) for estimation and K-normalised double2 for
// recoverPose (utils/verification.py:78-79).
__global__ void fmat_gather_kernel(const float* __restrict__ kp_xy, const double* __restrict__ intr, int kmax,
                                   const int* __restrict__ pairs, const uint32_t* __restrict__ match_idx,
                                   const int* __restrict__ match_count, int mcap, float4* __restrict__ pts,
                                   double2* __restrict__ x1n, double2* __restrict__ x2n) {
    const int p = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int M = match_count[p];
    if (i >= M) return;
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const uint32_t a = match_idx[((size_t)p * mcap + i) * 2], b = match_idx[((size_t)p * mcap + i) * 2 + 1];
    const float* k1 = kp_xy + ((size_t)i1 * kmax + a) * 2;
    const float* k2 = kp_xy + ((size_t)i2 * kmax + b) * 2;
    const size_t o = (size_t)p * mcap + i;
    pts[o] = make_float4(k1[0], k1[1], k2[0], k2[1]);
    x1n[o] = make_double2(((double)k1[0] - intr[3 * i1 + 1]) / intr[3 * i1], ((double)k1[1] - intr[3 * i1 + 2]) / intr[3 * i1]);
    x2n[o] = make_double2(((double)k2[0] - intr[3 * i2 + 1]) / intr[3 * i2], ((double)k2[1] - intr[3 * i2 + 2]) / intr[3 * i2]);
}

struct FOutputs {
    double* F;
    double* E;
    double* R;
    double* t;
    int* n_inliers;
    int* status;
    int* n_hyp;
    uint8_t* mask;
};

// One wave per pair: 7-point RANSAC (M >= 15) or LMedS (8 <= M < 15) in batches of 64 hypotheses (lane = hypothesis),
// candidates scored in (hypothesis, root) order, then the 8-point refit, E = K2^T F K1 and recoverPose. Every lane
// runs the same number of batches (niters is wave-uniform), so the loop always drains.
__global__ __launch_bounds__(64) void fmat_ransac_kernel(const int* __restrict__ pairs, const double* __restrict__ intr,
                                                         const int* __restrict__ match_count, int mcap,
                                                         const float4* __restrict__ pts_all,
                                                         const double2* __restrict__ x1n_all,
                                                         const double2* __restrict__ x2n_all, double thr_px,
                                                         double prob, int max_iters, uint64_t seed, int pair_id_base,
                                                         const int* __restrict__ pair_ids, FOutputs out) {
    __shared__ double candF[kFBatch * kFMaxSol * 9];
    __shared__ int cand_n[kFBatch];
    __shared__ double scratch[81 * 2 + 9];
    __shared__ int refit_ok;
    const int p = blockIdx.x, lane = threadIdx.x;
    const int M = match_count[p];
    uint8_t* mask = out.mask + (size_t)p * mcap;
    if (M < 8) {  // verifier_base.py:39-44 (NUM_MATCHES_REQ_F_MATRIX)
        for (int i = lane; i < M; i += 64) mask[i] = 0;
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 1;
            if (out.n_hyp) out.n_hyp[p] = 0;
        }
        return;
    }
    const float4* pts = pts_all + (size_t)p * mcap;
    const int pid = pair_ids ? pair_ids[p] : pair_id_base + p;
    const bool lmeds = M < 15;
    int niters = lmeds ? update_num_iters(prob, 0.45, 7, max_iters) : max_iters;
    if (niters < 1) niters = 1;
    const float thr2 = (float)(thr_px * thr_px);
    int done = 0, best = -1;
    bool have = false;
    float min_median = 3.402823466e+38f;
    double bestF[9];
    for (int e = 0; e < 9; ++e) bestF[e] = 0.0;
    while (done < niters) {
        int idx[7];
        int ns = 0;
        if (sample7(seed, pid, done + lane, M, pts, idx)) ns = seven_point(pts, idx, candF + lane * kFMaxSol * 9);
        cand_n[lane] = ns;
        __syncthreads();
        for (int hl = 0; hl < kFBatch; ++hl) {
            const int nsh = cand_n[hl];
            for (int s = 0; s < nsh; ++s) {
                const double* F = candF + (hl * kFMaxSol + s) * 9;
                double Fr[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) Fr[e] = F[e];
                if (lmeds) {
                    const float err = lane < M ? fm_error(Fr, pts[lane]) : 0.0f;
                    int rank = 0;
                    for (int j = 0; j < M; ++j) {
                        const float ej = __shfl(err, j);
                        rank += (ej < err || (ej == err && j < lane)) ? 1 : 0;
                    }
                    const uint64_t who = __ballot(lane < M && rank == M / 2);
                    const float med = __shfl(err, (int)__ffsll((unsigned long long)who) - 1);
                    if (med < min_median) {
                        min_median = med;
#pragma unroll
                        for (int e = 0; e < 9; ++e) bestF[e] = Fr[e];
                        have = true;
                    }
                } else {
                    const int floor_c = best > 6 ? best : 6;
                    const int c = fm_wave_count(Fr, pts, M, thr2, floor_c, lane);
                    if (c > floor_c) {
                        best = c;
#pragma unroll
                        for (int e = 0; e < 9; ++e) bestF[e] = Fr[e];
                        have = true;
                    }
                }
            }
        }
        __syncthreads();  // candF / cand_n are rewritten by the next batch
        done += kFBatch;
        if (!lmeds && best > 0) {
            const int upd = update_num_iters(prob, (double)(M - best) / M, 7, niters);
            if (upd < niters) niters = upd;
        }
    }
    int cnt = -1;
    if (have) {
        double th = thr_px;
        if (lmeds) {
            th = 2.5 * 1.4826 * (1.0 + 5.0 / (M - 7)) * sqrt((double)min_median);
            if (th < 0.001) th = 0.001;
        }
        const float th2 = (float)(th * th);
        auto write_mask = [&](const double* F) {
            int c = 0;
            for (int i = lane; i < M; i += 64) {
                const bool in = fm_error(F, pts[i]) <= th2;
                mask[i] = in ? 1 : 0;
                c += in ? 1 : 0;
            }
            for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
            return c;
        };
        cnt = write_mask(bestF);
        if (cnt >= 8) {
            __syncthreads();  // mask visible to lane 0
            if (lane == 0) refit_ok = eight_point_serial(pts, mask, M, scratch, scratch + 81, scratch + 162) ? 1 : 0;
            __syncthreads();
            if (refit_ok) {
                double Fr[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) Fr[e] = scratch[162 + e];
                const int cr = fm_wave_count(Fr, pts, M, th2, -1, lane);
                if (cr >= cnt) {
#pragma unroll
                    for (int e = 0; e < 9; ++e) bestF[e] = Fr[e];
                    cnt = write_mask(bestF);
                }
            }
        }
        if (lmeds && cnt < 7) cnt = -1;
    }
    if (cnt < 0) {
        for (int i = lane; i < M; i += 64) mask[i] = 0;
        if (lane == 0) {
            out.n_inliers[p] = 0;
            out.status[p] = 2;
            if (out.n_hyp) out.n_hyp[p] = done;
        }
        return;
    }
    __syncthreads();  // final mask visible to every lane
    // E = K2^T F K1 (utils/verification.py:97-110)
    const int i1 = pairs[2 * p], i2 = pairs[2 * p + 1];
    const double K1[9] = {intr[3 * i1], 0.0, intr[3 * i1 + 1], 0.0, intr[3 * i1], intr[3 * i1 + 2], 0.0, 0.0, 1.0};
    const double K2[9] = {intr[3 * i2], 0.0, intr[3 * i2 + 1], 0.0, intr[3 * i2], intr[3 * i2 + 2], 0.0, 0.0, 1.0};
    double FK[9], E[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            FK[3 * r + c] = bestF[3 * r + 0] * K1[0 * 3 + c] + bestF[3 * r + 1] * K1[1 * 3 + c] + bestF[3 * r + 2] * K1[2 * 3 + c];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            E[3 * r + c] = K2[0 * 3 + r] * FK[0 * 3 + c] + K2[1 * 3 + r] * FK[1 * 3 + c] + K2[2 * 3 + r] * FK[2 * 3 + c];
    // recoverPose on the K-normalised inliers (same decomposition + cheirality vote as the E path)
    const double2* x1 = x1n_all + (size_t)p * mcap;
    const double2* x2 = x2n_all + (size_t)p * mcap;
    double U[9], sv[3], V[9];
    svd3(E, U, sv, V);
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
            out.F[9 * p + k] = bestF[k];
            out.E[9 * p + k] = E[k];
            out.R[9 * p + k] = Rs[k];
        }
        for (int k = 0; k < 3; ++k) out.t[3 * p + k] = ts[k];
        out.n_inliers[p] = cnt;
        out.status[p] = 0;
        if (out.n_hyp) out.n_hyp[p] = done;
    }
}

}  // namespace

extern "C" {

static size_t fmat_layout(int n_pairs, int mcap, size_t* off_x1n, size_t* off_x2n) {
    const size_t n = (size_t)n_pairs * mcap;
    size_t o = gtsfm_align_up(n * sizeof(float4), 256);
    *off_x1n = o;
    o += gtsfm_align_up(n * sizeof(double2), 256);
    *off_x2n = o;
    o += gtsfm_align_up(n * sizeof(double2), 256);
    return o;
}

size_t gtsfm_ransac_F_workspace_bytes(int n_pairs, int mcap) {
    if (n_pairs <= 0 || mcap <= 0) return 0;
    size_t a, b;
    return fmat_layout(n_pairs, mcap, &a, &b);
}

int gtsfm_ransac_F_batched(const float* d_kp_xy, const double* d_intrinsics, int n_img, int kmax, const int* d_pairs,
                           int n_pairs, const uint32_t* d_match_idx, const int* d_match_count, int mcap,
                           double thr_px, double prob, int max_iters, uint64_t seed, int pair_id_base,
                           const int* d_pair_ids, void* d_workspace, size_t workspace_bytes, double* d_F, double* d_E,
                           double* d_R, double* d_t, int* d_n_inliers, int* d_status, int* d_n_hyp,
                           uint8_t* d_inlier_mask, void* stream_v) {
    hipStream_t stream = (hipStream_t)stream_v;
    if (n_pairs == 0) return GTSFM_OK;
    if (!d_kp_xy || !d_intrinsics || !d_pairs || !d_match_idx || !d_match_count || !d_F || !d_E || !d_R || !d_t ||
        !d_n_inliers || !d_status || !d_inlier_mask || n_img <= 0 || kmax <= 0 || n_pairs < 0 || mcap <= 0 ||
        max_iters <= 0 || !(thr_px > 0.0))
        return GTSFM_ERR_ARG;
    size_t o_x1n, o_x2n;
    const size_t need = fmat_layout(n_pairs, mcap, &o_x1n, &o_x2n);
    if (workspace_bytes < need) return GTSFM_ERR_CAPACITY;
    unsigned char* ws = (unsigned char*)d_workspace;
    float4* pts = (float4*)ws;
    double2* x1n = (double2*)(ws + o_x1n);
    double2* x2n = (double2*)(ws + o_x2n);
    hipLaunchKernelGGL(fmat_gather_kernel, dim3((mcap + 255) / 256, n_pairs), dim3(256), 0, stream, d_kp_xy,
                       d_intrinsics, kmax, d_pairs, d_match_idx, d_match_count, mcap, pts, x1n, x2n);
    const FOutputs o{d_F, d_E, d_R, d_t, d_n_inliers, d_status, d_n_hyp, d_inlier_mask};
    hipLaunchKernelGGL(fmat_ransac_kernel, dim3(n_pairs), dim3(64), 0, stream, d_pairs, d_intrinsics, d_match_count,
                       mcap, pts, x1n, x2n, thr_px, prob, max_iters, seed, pair_id_base, d_pair_ids, o);
    GTSFM_CHECK_HIP(hipGetLastError());
    return GTSFM_OK;
}

}  // extern "C"
