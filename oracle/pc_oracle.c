/*
 * pc_oracle.c — C restatement of stable PC-fisherz skeleton discovery.
 * TEST INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py (as the checker / CPU baseline), never by rcaeval_amd.
 *
 * Restates:
 *   - lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:70-144 (vendored; stable branch)
 *       level loop `while max_degree()-1 > depth` (:72), node skip `len(Neigh_x) < depth-1`
 *       (:83), `combinations(Neigh_x \ {y}, depth)` (:106), `p > alpha` -> deferred removal +
 *       sepset union (:124-130, :135-136), removal at the level barrier (:141-144).
 *   - lib/causallearn/graph/GraphClass.py:78-106: cache key (min, max, S) — here realised by
 *       computing each unique test once on its canonical owner side, `neighbors`, `max_degree`.
 *   - causal-learn 0.1.3.3 FisherZ.__call__ [U]: inv of the (d+2)x(d+2) sub-correlation by
 *       LU with partial pivoting (LAPACK dgetf2/dgetrs order, as numpy.linalg.inv -> dgesv),
 *       r = -inv01/sqrt(inv00*inv11), Z = 0.5*log((1+r)/(1-r)), X = sqrt(N-d-3)|Z|,
 *       p = 2*(1 - ndtr(|X|)) with cephes ndtr's branch structure.
 *
 * Dedup rule (= the reference's memo): the test (min(x,y), max(x,y), S) is computed on
 * node x's side unless y < x and S is a subset of adj(y) (then node y computes it). An
 * independent result is OR-ed into x's side union, and into y's side union whenever
 * S is a subset of adj(y) (the reference reaches the same cached p from both sides).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_MAXD 32

typedef struct {
    int64_t tests[32];   /* unique tests per depth            */
    int64_t calls[32];   /* ci_test invocations per depth     */
    int64_t indep[32];   /* unique tests with p > alpha       */
    int32_t levels;      /* number of depths run              */
    int32_t error;       /* 0 ok, 1 singular, 2 math domain   */
    double secs[32];     /* wall seconds per depth            */
} orc_stats;

typedef struct {         /* one unique test (record mode) */
    int32_t a, b;        /* a < b */
    int32_t d;
    int32_t s[12];       /* sorted conditioning set, -1 padded */
    double p;
} orc_record;

/* cephes ndtr branch structure: p = 2*(1 - ndtr(|X|)). */
static double pvalue_from_X(double X) {
    double a = fabs(X);
    double x = a * M_SQRT1_2;
    double z = fabs(x), y;
    if (z < M_SQRT1_2) {
        y = 0.5 + 0.5 * erf(x);
    } else {
        y = 0.5 * erfc(z);
        if (x > 0) y = 1.0 - y;
    }
    return 2.0 * (1.0 - y);
}

/* numpy.linalg.inv (dgesv with B = I) restricted to columns 0 and 1 of the inverse.
 * Returns 0 ok, 1 exactly singular (LAPACK INFO > 0). */
static int lu_inv01(double *A, int m, double *i00, double *i01, double *i11) {
    int piv[ORC_MAXD + 2];
    int info = 0;
    for (int j = 0; j < m; ++j) {
        int p = j;
        double best = fabs(A[j * m + j]);
        for (int i = j + 1; i < m; ++i) {
            double v = fabs(A[i * m + j]);
            if (v > best) { best = v; p = i; }
        }
        piv[j] = p;
        if (A[p * m + j] != 0.0) {
            if (p != j)
                for (int k = 0; k < m; ++k) { double t = A[j * m + k]; A[j * m + k] = A[p * m + k]; A[p * m + k] = t; }
            double rcp = 1.0 / A[j * m + j];
            for (int i = j + 1; i < m; ++i) A[i * m + j] *= rcp;
        } else if (!info) {
            info = j + 1;
        }
        for (int i = j + 1; i < m; ++i) {
            double l = A[i * m + j];
            for (int k = j + 1; k < m; ++k) A[i * m + k] -= l * A[j * m + k];
        }
    }
    if (info) return 1;
    double B[2][ORC_MAXD + 2];
    for (int c = 0; c < 2; ++c) {
        for (int i = 0; i < m; ++i) B[c][i] = (i == c) ? 1.0 : 0.0;
        for (int i = 0; i < m; ++i) { int p = piv[i]; if (p != i) { double t = B[c][i]; B[c][i] = B[c][p]; B[c][p] = t; } }
        for (int i = 0; i < m; ++i) for (int k = 0; k < i; ++k) B[c][i] -= A[i * m + k] * B[c][k];
        for (int i = m - 1; i >= 0; --i) {
            for (int k = i + 1; k < m; ++k) B[c][i] -= A[i * m + k] * B[c][k];
            B[c][i] /= A[i * m + i];
        }
    }
    *i00 = B[0][0];
    *i01 = B[1][0];   /* inv[0,1] = column 1, row 0 */
    *i11 = B[1][1];
    return 0;
}

/* One Fisher-z test on canonical (a<b, S sorted). err: 0 ok, 1 singular, 2 domain. */
double orc_fisherz(const double *C, int n, int N, int a, int b, const int *S, int d, int *err) {
    int var[ORC_MAXD + 2];
    double A[(ORC_MAXD + 2) * (ORC_MAXD + 2)];
    int m = d + 2;
    var[0] = a; var[1] = b;
    for (int k = 0; k < d; ++k) var[2 + k] = S[k];
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) A[i * m + j] = C[(int64_t)var[i] * n + var[j]];
    double i00, i01, i11;
    *err = 0;
    if (lu_inv01(A, m, &i00, &i01, &i11)) { *err = 1; return NAN; }
    double prod = i00 * i11;
    if (prod < 0) { *err = 2; return NAN; }            /* math.sqrt(negative) */
    double r = -i01 / sqrt(prod);
    double ratio = (1.0 + r) / (1.0 - r);               /* numpy scalar: x/0 -> inf */
    if (ratio <= 0) { *err = 2; return NAN; }           /* math.log(<=0) */
    double Z = 0.5 * log(ratio);
    double dof = (double)N - d - 3;
    if (dof < 0) { *err = 2; return NAN; }
    double X = sqrt(dof) * fabs(Z);
    return pvalue_from_X(X);
}

static inline int has_bit(const uint64_t *row, int j) { return (row[j >> 6] >> (j & 63)) & 1; }

typedef struct {            /* one depth of the x-side loop (SkeletonDiscovery.py:77-136) */
    const double *C;
    int n, N, W, d;
    double alpha;
    const uint64_t *adj;    /* n x W adjacency at the start of the depth */
    const int32_t *deg, *nbr;
    uint8_t *rm;            /* n x n removal flags (NULL: count only) */
    uint64_t *side_union;
    orc_record *rec, *nearl;
    int64_t rec_cap, near_cap, *rec_count, *near_count;
    int x0, xstep;          /* nodes x = x0, x0 + xstep, ... (a node sample when xstep > 1) */
} orc_level;

/* Runs the visits of the selected nodes; returns the error code (0 ok). */
static int level_pass(const orc_level *L, int64_t *tests_out, int64_t *calls_out, int64_t *indep_out) {
    const int n = L->n, W = L->W, d = L->d;
    int64_t tests = 0, calls = 0, indep = 0;
    volatile int error = 0;
    /* work items = (x, y) visits, so that one high-degree node (work ~ D^(d+1)) is spread over
       the threads instead of forming a tail */
    int64_t nitem = 0;
    for (int x = L->x0; x < n; x += L->xstep)
        if (L->deg[x] >= d - 1) nitem += L->deg[x];
    int32_t *item = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)(nitem > 0 ? nitem : 1));
    if (!item) return -1;
    {
        int64_t k = 0;
        for (int x = L->x0; x < n; x += L->xstep)
            if (L->deg[x] >= d - 1)
                for (int yi = 0; yi < L->deg[x]; ++yi) { item[2 * k] = x; item[2 * k + 1] = yi; ++k; }
    }
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tests, calls, indep)
    for (int64_t it = 0; it < nitem; ++it) {
        const int x = item[2 * it];
        const int D = L->deg[x];
        const int32_t *nx = L->nbr + (size_t)x * n;
        int idx[ORC_MAXD + 1], S[ORC_MAXD + 1];
        {
            const int yi = item[2 * it + 1];
            const int y = nx[yi];
            const uint64_t *ady = L->adj + (size_t)y * W;
            /* combinations of nx \ {y} of size d, lexicographic */
            const int M = D - 1;
            if (M < d) continue;
            for (int k = 0; k < d; ++k) idx[k] = k;
            for (;;) {
                int in_y = 1;
                for (int k = 0; k < d; ++k) {
                    int li = idx[k] < yi ? idx[k] : idx[k] + 1;
                    S[k] = nx[li];
                    if (!has_bit(ady, S[k])) in_y = 0;
                }
                calls++;
                if (!(y < x && in_y)) {
                    int a = x < y ? x : y, b = x < y ? y : x, err;
                    double p = orc_fisherz(L->C, n, L->N, a, b, S, d, &err);
                    if (err) error = err;
                    tests++;
                    if (L->rec) {
                        int64_t slot = __atomic_fetch_add(L->rec_count, 1, __ATOMIC_RELAXED);
                        if (slot < L->rec_cap) {
                            orc_record *r = L->rec + slot;
                            r->a = a; r->b = b; r->d = d;
                            for (int k = 0; k < 12; ++k) r->s[k] = k < d ? S[k] : -1;
                            r->p = p;
                        }
                    }
                    if (L->nearl && fabs(p - L->alpha) < 1e-9) {
                        int64_t slot = __atomic_fetch_add(L->near_count, 1, __ATOMIC_RELAXED);
                        if (slot < L->near_cap) {
                            orc_record *r = L->nearl + slot;
                            r->a = a; r->b = b; r->d = d;
                            for (int k = 0; k < 12; ++k) r->s[k] = k < d ? S[k] : -1;
                            r->p = p;
                        }
                    }
                    if (p > L->alpha) {
                        indep++;
                        if (L->rm) {
                            __atomic_store_n(&L->rm[(size_t)x * n + y], 1, __ATOMIC_RELAXED);
                            __atomic_store_n(&L->rm[(size_t)y * n + x], 1, __ATOMIC_RELAXED);
                        }
                        if (L->side_union) {
                            uint64_t *ux = L->side_union + ((size_t)x * n + y) * W;
                            uint64_t *uy = L->side_union + ((size_t)y * n + x) * W;
                            for (int k = 0; k < d; ++k) {
                                __atomic_fetch_or(&ux[S[k] >> 6], 1ull << (S[k] & 63), __ATOMIC_RELAXED);
                                if (in_y) __atomic_fetch_or(&uy[S[k] >> 6], 1ull << (S[k] & 63), __ATOMIC_RELAXED);
                            }
                        }
                    }
                }
                /* next combination */
                int k = d - 1;
                while (k >= 0 && idx[k] == M - d + k) --k;
                if (k < 0) break;
                idx[k]++;
                for (int j = k + 1; j < d; ++j) idx[j] = idx[j - 1] + 1;
            }
        }
    }
    free(item);
    *tests_out = tests;
    *calls_out = calls;
    *indep_out = indep;
    return error;
}

static double now_s(void) {
#ifdef _OPENMP
    return omp_get_wtime();
#else
    return (double)clock() / CLOCKS_PER_SEC;
#endif
}

/* degrees + ascending neighbour lists of the adjacency bitmask; returns the max degree */
static int build_lists(const uint64_t *adj, int n, int W, int32_t *deg, int32_t *nbr) {
    int maxdeg = 0;
    for (int x = 0; x < n; ++x) {
        int c = 0;
        for (int w = 0; w < W; ++w) c += __builtin_popcountll(adj[(size_t)x * W + w]);
        deg[x] = c;
        if (c > maxdeg) maxdeg = c;
        int k = 0;
        for (int y = 0; y < n; ++y) if (has_bit(adj + (size_t)x * W, y)) nbr[(size_t)x * n + k++] = y;
    }
    return maxdeg;
}

/*
 * Stable skeleton. C: n x n row-major correlation. Outputs:
 *   removed_level[n*n]   int8, -1 = survives, else depth at which the edge was removed
 *   deg_at_level[32*n]   optional (NULL ok): degree of each node at the start of each depth
 *   side_union[n*n*W]    optional (NULL ok), W = ceil(n/64): for a removed pair (x,y) the
 *                        union of independent S on x's side at the removal depth
 *   rec/rec_cap/rec_count optional: every unique test (record mode)
 *   nearl/near_cap/near_count optional: every unique test with |p - alpha| < 1e-9 (the tests
 *                        whose decision north_star allows to differ; enumerated like the engine)
 * max_depth < 0: unlimited. nthreads <= 0: all. st->secs: wall time per depth.
 */
/* banned (NULL ok): n x n pairs forbidden in both directions by background knowledge; queued
 * for removal at the end of depth 0 beside the tests' own decisions (SkeletonDiscovery.py:86-106,
 * stable branch: every visit at every depth queues them, so they are gone after depth 0). */
int orc_skeleton_bk(const double *C, int n, int N, double alpha, int max_depth,
                    int8_t *removed_level, int32_t *deg_at_level, uint64_t *side_union,
                    orc_record *rec, int64_t rec_cap, int64_t *rec_count,
                    orc_record *nearl, int64_t near_cap, int64_t *near_count,
                    orc_stats *st, int nthreads, const uint8_t *banned) {
    const int W = (n + 63) / 64;
    uint64_t *adj = (uint64_t *)calloc((size_t)n * W, sizeof(uint64_t));
    int32_t *deg = (int32_t *)malloc(sizeof(int32_t) * n);
    int32_t *nbr = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * n);
    uint8_t *rm = (uint8_t *)calloc((size_t)n * n, 1);
    if (!adj || !deg || !nbr || !rm) return -1;
    memset(st, 0, sizeof(*st));
    for (int64_t i = 0; i < (int64_t)n * n; ++i) removed_level[i] = -1;
    for (int x = 0; x < n; ++x)
        for (int y = 0; y < n; ++y)
            if (x != y) adj[(size_t)x * W + (y >> 6)] |= 1ull << (y & 63);
    if (side_union) memset(side_union, 0, sizeof(uint64_t) * (size_t)n * n * W);
    if (rec_count) *rec_count = 0;
    if (near_count) *near_count = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int depth = -1, error = 0;
    for (;;) {
        const int maxdeg = build_lists(adj, n, W, deg, nbr);
        if (!(maxdeg - 1 > depth)) break;
        if (max_depth >= 0 && depth >= max_depth) break;
        ++depth;
        if (depth >= 32 || depth > ORC_MAXD) break;
        if (deg_at_level) memcpy(deg_at_level + (size_t)depth * n, deg, sizeof(int32_t) * n);
        memset(rm, 0, (size_t)n * n);
        orc_level L = {C, n, N, W, depth, alpha, adj, deg, nbr, rm, side_union, rec, nearl,
                       rec_cap, near_cap, rec_count, near_count, 0, 1};
        const double t0 = now_s();
        int64_t tests, calls, indep;
        error = level_pass(&L, &tests, &calls, &indep);
        st->secs[depth] = now_s() - t0;
        st->tests[depth] = tests;
        st->calls[depth] = calls;
        st->indep[depth] = indep;
        st->levels = depth + 1;
        if (banned && depth == 0)
            for (int x = 0; x < n; ++x)
                for (int y = 0; y < n; ++y)
                    if (x != y && banned[(size_t)x * n + y]) rm[(size_t)x * n + y] = 1;
        for (int x = 0; x < n; ++x)
            for (int y = 0; y < n; ++y)
                if (rm[(size_t)x * n + y]) {
                    adj[(size_t)x * W + (y >> 6)] &= ~(1ull << (y & 63));
                    removed_level[(size_t)x * n + y] = (int8_t)depth;
                }
        if (error) break;
    }
    st->error = error;
    free(adj); free(deg); free(nbr); free(rm);
    return error ? 1 : 0;
}

int orc_skeleton(const double *C, int n, int N, double alpha, int max_depth,
                 int8_t *removed_level, int32_t *deg_at_level, uint64_t *side_union,
                 orc_record *rec, int64_t rec_cap, int64_t *rec_count,
                 orc_record *nearl, int64_t near_cap, int64_t *near_count,
                 orc_stats *st, int nthreads) {
    return orc_skeleton_bk(C, n, N, alpha, max_depth, removed_level, deg_at_level, side_union, rec, rec_cap,
                           rec_count, nearl, near_cap, near_count, st, nthreads, NULL);
}

/* CPU-baseline sample of one depth: the visits of nodes x0, x0+xstep, ... at depth d on the
 * adjacency {(x, y): removed_level[x,y] == -1 or >= d} (the graph at the start of depth d).
 * Counts only (no removal, no sepsets). Returns the error code; tests/seconds out. */
int orc_level_sample(const double *C, int n, int N, double alpha, const int8_t *removed_level, int d,
                     int x0, int xstep, int nthreads, int64_t *tests_out, double *seconds_out) {
    const int W = (n + 63) / 64;
    uint64_t *adj = (uint64_t *)calloc((size_t)n * W, sizeof(uint64_t));
    int32_t *deg = (int32_t *)malloc(sizeof(int32_t) * n);
    int32_t *nbr = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * n);
    if (!adj || !deg || !nbr) return -1;
    for (int x = 0; x < n; ++x)
        for (int y = 0; y < n; ++y) {
            const int8_t r = removed_level[(size_t)x * n + y];
            if (x != y && (r < 0 || r >= d)) adj[(size_t)x * W + (y >> 6)] |= 1ull << (y & 63);
        }
    build_lists(adj, n, W, deg, nbr);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    orc_level L = {C, n, N, W, d, alpha, adj, deg, nbr, NULL, NULL, NULL, NULL, 0, 0, NULL, NULL,
                   x0, xstep > 0 ? xstep : 1};
    const double t0 = now_s();
    int64_t tests, calls, indep;
    const int err = level_pass(&L, &tests, &calls, &indep);
    *seconds_out = now_s() - t0;
    *tests_out = tests;
    free(adj); free(deg); free(nbr);
    return err;
}

/* Fisher-z p-values for an explicit list of tests (used to cross-check the numpy oracle). */
void orc_fisherz_batch(const double *C, int n, int N, const int32_t *ab, const int32_t *S, int d,
                       int64_t count, double *p_out, int32_t *err_out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < count; ++i) {
        int err;
        p_out[i] = orc_fisherz(C, n, N, ab[2 * i], ab[2 * i + 1], S + i * (d > 0 ? d : 1), d, &err);
        err_out[i] = err;
    }
}

/* Threaded np.corrcoef(data.T)-equivalent (numpy order: centre, dot, *1/(N-1), /s_i, /s_j, clip). */
void orc_corrcoef(const double *X, int64_t N, int n, double *C) {
    double *mean = (double *)calloc(n, sizeof(double));
    for (int64_t t = 0; t < N; ++t) for (int j = 0; j < n; ++j) mean[j] += X[t * n + j];
    for (int j = 0; j < n; ++j) mean[j] /= (double)N;
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = 0; i < n; ++i)
        for (int j = i; j < n; ++j) {
            double s = 0;
            for (int64_t t = 0; t < N; ++t) s += (X[t * n + i] - mean[i]) * (X[t * n + j] - mean[j]);
            C[(int64_t)i * n + j] = C[(int64_t)j * n + i] = s * (1.0 / (double)(N - 1));
        }
    double *sd = (double *)malloc(sizeof(double) * n);
    for (int i = 0; i < n; ++i) sd[i] = sqrt(C[(int64_t)i * n + i]);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = C[(int64_t)i * n + j] / sd[i];
            v = v / sd[j];
            C[(int64_t)i * n + j] = v > 1 ? 1 : (v < -1 ? -1 : v);
        }
    free(mean); free(sd);
}
