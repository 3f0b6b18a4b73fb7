/*
 * ORACLE — test infrastructure only. CPU restatement of the reference's TwoWayMatcher.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
 * and only as the checker / CPU baseline; the product path never calls it.
 *
 * Restates (reference file:line, /root/reference):
 *   gtsfm/frontend/matcher/twoway_matcher.py:104-121  __perform_matching (1->2, 2->1, mutual filter
 *                                                      iterated in 1->2 dict order)
 *   gtsfm/frontend/matcher/twoway_matcher.py:123-144  __perform_oneway_matching:
 *       cv.BFMatcher(NORM_L2, crossCheck=False).knnMatch(k=2)  (:102, :136)  or .match (k=1, :139)
 *       keep m1 iff m1.distance <= ratio * m2.distance     (:137; Python double compare of f32 distances)
 *       sorted(matches, key=distance) (stable)           (:141)
 *       dict {queryIdx: trainIdx}                          (:142)
 * Third-party semantics restated (OpenCV BFMatcher, opencv-python>=4.5.4.58, environment_linux.yml:50):
 *   distance = sqrt(sum_k (q_k - t_k)^2) in float32; the k nearest are kept by a strict '<' insertion scan
 *   over train indices in increasing order, so equal distances keep the lowest train index first.
 *   Summation order here is sequential over k (OpenCV's SIMD order differs only in float rounding; for
 *   integer-valued descriptors such as SIFT's the sums are exact integers and every order agrees).
 *
 * Build: compiled with -ffp-contract=off so (a-b)*(a-b)+acc is never fused (the HIP exact path matches).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float d1, d2; /* distances of best and second best (d2 = +inf when absent) */
    int j1;       /* index of best (-1 if none) */
} top2_t;

/* One-way kNN (k=2) of every query row against all train rows. */
static void oneway_top2(const float* q, int nq, const float* t, int nt, int D, top2_t* out) {
    for (int i = 0; i < nq; ++i) {
        float b1 = INFINITY, b2 = INFINITY;
        int j1 = -1;
        const float* qi = q + (size_t)i * D;
        for (int j = 0; j < nt; ++j) {
            const float* tj = t + (size_t)j * D;
            float acc = 0.f;
            for (int k = 0; k < D; ++k) {
                float df = qi[k] - tj[k];
                acc = acc + df * df;
            }
            float d = sqrtf(acc);
            if (d < b2) {
                if (d < b1) {
                    b2 = b1;
                    b1 = d;
                    j1 = j;
                } else {
                    b2 = d;
                }
            }
        }
        out[i].d1 = b1;
        out[i].d2 = b2;
        out[i].j1 = j1;
    }
}

static int passes_ratio(const top2_t* m, double ratio) {
    if (ratio < 0.0) return 1; /* no ratio test: BFMatcher.match path */
    return (double)m->d1 <= ratio * (double)m->d2;
}

typedef struct {
    float d;
    int i;
} sortrec_t;

static int cmp_sortrec(const void* a, const void* b) {
    const sortrec_t* x = (const sortrec_t*)a;
    const sortrec_t* y = (const sortrec_t*)b;
    if (x->d < y->d) return -1;
    if (x->d > y->d) return 1;
    return (x->i > y->i) - (x->i < y->i); /* Python's stable sort keeps query order on ties */
}

/*
 * Mutual-NN (+ optional ratio test) matching of d1 (n1 x D) against d2 (n2 x D).
 * ratio < 0 disables the ratio test. out must hold 2*min(n1,n2) uint32. Returns the match count,
 * rows ordered by ascending 1->2 distance (ties by index in image 1), as the reference does.
 */
int oracle_twoway_match(const float* d1, int n1, const float* d2, int n2, int D, double ratio, uint32_t* out) {
    if (n1 <= 0 || n2 <= 0 || D <= 0) return 0;
    top2_t* r12 = (top2_t*)malloc(sizeof(top2_t) * (size_t)n1);
    top2_t* r21 = (top2_t*)malloc(sizeof(top2_t) * (size_t)n2);
    sortrec_t* recs = (sortrec_t*)malloc(sizeof(sortrec_t) * (size_t)n1);
    oneway_top2(d1, n1, d2, n2, D, r12);
    oneway_top2(d2, n2, d1, n1, D, r21);
    int m = 0;
    for (int i = 0; i < n1; ++i) {
        if (r12[i].j1 < 0 || !passes_ratio(&r12[i], ratio)) continue;
        recs[m].d = r12[i].d1;
        recs[m].i = i;
        ++m;
    }
    qsort(recs, (size_t)m, sizeof(sortrec_t), cmp_sortrec);
    int nout = 0;
    for (int k = 0; k < m; ++k) {
        int i = recs[k].i;
        int j = r12[i].j1;
        if (r21[j].j1 == i && passes_ratio(&r21[j], ratio)) {
            out[2 * nout] = (uint32_t)i;
            out[2 * nout + 1] = (uint32_t)j;
            ++nout;
        }
    }
    free(r12);
    free(r21);
    free(recs);
    return nout;
}

/* Per-row top-2 (exposed for intermediate-level parity checks). */
void oracle_oneway_top2(const float* q, int nq, const float* t, int nt, int D, float* d1, float* d2, int* j1) {
    top2_t* r = (top2_t*)malloc(sizeof(top2_t) * (size_t)(nq > 0 ? nq : 1));
    oneway_top2(q, nq, t, nt, D, r);
    for (int i = 0; i < nq; ++i) {
        d1[i] = r[i].d1;
        d2[i] = r[i].d2;
        j1[i] = r[i].j1;
    }
    free(r);
}
