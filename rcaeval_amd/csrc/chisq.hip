// chisq.hip — batched discrete CI tests (chi-square / G-square) for RCD's skeletons.
//
// Replaces causal-learn's `chisq` / `gsq` (utils/cit.py `chisq_or_gsq_test` [U], causal-learn
// 0.1.2.3 in RCAEval's RCD environment, requirements_rcd.lock:20) as called by
// lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:152-210 (local_skeleton_discovery) and
// :70-144 (stable=False) from RCAEval/e2e/rcd.py:72-102 (run_pc, CI_TEST = chisq, :21).
//
// Per test (x < y, S): the contingency table T[s, x, y] of the integer-coded samples with the
// reference's mixed-radix stratum index (S[0] fastest, cardCumProd of [S..., X, Y]); strata
// with no samples are dropped (`SMarginalCounts != 0`); expected E = Sx * Sy / Sm (int64
// products, float64 division); statistic = sum over the kept (k, x, y) cells in C order of
// (T - E)^2 / (E == 0 ? 1 : E) (chi-square) or 2 * T * log(T / E) (G-square, ratio 0 -> 1),
// summed like numpy's sum (pairwise: 8 accumulators, 128-element leaves, inside blocks of 8192
// elements accumulated in order), so the chi-square statistic is bitwise numpy's (G-square up to
// the last bit of the device log); df = sum_k (cX - 1 - zero rows_k) * (cY - 1 - zero cols_k).
// The tail probability chi2.sf(stat, df) is left to the caller (scipy's chdtrc on the host:
// one vectorised call per batch), p = 1 when df <= 0.
//
// Layout: data is variable-major n x N int32 (one variable's samples contiguous, so a test
// streams 2 + |S| coalesced columns); one 256-thread block per test, the table in LDS when it
// has <= LDS_CELLS cells, else in the block's slice of a handle-owned global scratch.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "handle.h"

namespace {

constexpr int CHI_BLOCK = 256;
constexpr int LDS_CELLS = 8192;          // int32 counts: 32 KB

struct ChiPlan {
    int a, b, d, bad;
    int64_t cS, cX, cY, cells;
    int s[PCG_MAX_LEVEL_DEPTH];
    int64_t cum[PCG_MAX_LEVEL_DEPTH];
};

// numpy pairwise_sum over a[0..n): leaves of <= 128 (8 accumulators), halves rounded down to a
// multiple of 8 — post-order over an explicit stack (thread-local)
__device__ double np_pairwise_leaf(const double *a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

__device__ double np_pairwise_sum(const double *a, int64_t n) {
    struct Frame { int64_t s, n; int state; double left; };
    Frame st[64];
    int sp = 1;
    st[0] = {0, n, 0, 0.0};
    double result = 0.0;      // value of the frame that finished last
    while (sp) {
        Frame &f = st[sp - 1];
        if (f.n <= 128) {
            result = np_pairwise_leaf(a + f.s, f.n);
            --sp;
            continue;
        }
        int64_t n2 = f.n / 2;
        n2 -= n2 % 8;
        if (f.state == 0) {
            f.state = 1;
            st[sp++] = {f.s, n2, 0, 0.0};
        } else if (f.state == 1) {
            f.left = result;
            f.state = 2;
            st[sp++] = {f.s + n2, f.n - n2, 0, 0.0};
        } else {
            result = f.left + result;
            --sp;
        }
    }
    return result;
}

__global__ __launch_bounds__(CHI_BLOCK) void k_chisq(const int32_t *data, int64_t N, int n, const int32_t *card,
                                                     const int32_t *tests, int stride, int64_t count, int g_sq,
                                                     int64_t max_cells, char *scratch, int64_t per_block,
                                                     double *stat, int64_t *dfout, int32_t *status) {
    __shared__ ChiPlan P;
    __shared__ int lds_hist[LDS_CELLS];
    __shared__ int bad_sample;
    __shared__ int64_t part_cnt[CHI_BLOCK];
    char *mine = scratch + (int64_t)blockIdx.x * per_block;
    for (int64_t t = blockIdx.x; t < count; t += gridDim.x) {
        const int tid = threadIdx.x;
        if (tid == 0) {
            const int32_t *row = tests + t * (int64_t)stride;
            P.a = row[0]; P.b = row[1]; P.d = row[2];
            int bad = (P.d < 0 || P.d > PCG_MAX_LEVEL_DEPTH || P.d + 3 > stride || P.a < 0 || P.b < 0 || P.a >= n ||
                       P.b >= n || P.a == P.b);
            int64_t cS = 1;
            for (int q = 0; !bad && q < P.d; ++q) {
                const int s = row[3 + q];
                bad |= (s < 0 || s >= n || s == P.a || s == P.b);
                if (bad) break;
                P.s[q] = s;
                P.cum[q] = cS;
                const int c = card[s];
                bad |= c < 1;
                cS *= c;
                bad |= cS > max_cells;
            }
            if (!bad) {
                P.cS = cS;
                P.cX = card[P.a];
                P.cY = card[P.b];
                bad |= P.cX < 1 || P.cY < 1;
                P.cells = P.cS * P.cX * P.cY;
                if (!bad && P.cells > max_cells) bad = 2;
            }
            P.bad = bad;
            bad_sample = 0;
        }
        __syncthreads();
        if (P.bad) {
            if (tid == 0) {
                status[t] = P.bad == 2 ? 4 : 3;
                stat[t] = __builtin_nan("");
                dfout[t] = 0;
            }
            __syncthreads();
            continue;
        }
        const int64_t cS = P.cS, cX = P.cX, cY = P.cY, cells = P.cells;
        // scratch slice: [counts int32 (global table only)] [terms f64] [Sm i64] [Sx i64] [Sy i64] [rank i64]
        int *ghist = reinterpret_cast<int *>(mine);
        double *terms = reinterpret_cast<double *>(mine + ((sizeof(int) * max_cells + 15) & ~(size_t)15));
        int64_t *Sm = reinterpret_cast<int64_t *>(terms + max_cells);
        int64_t *Sx = Sm + max_cells;
        int64_t *Sy = Sx + max_cells;
        int64_t *rank = Sy + max_cells;
        int *hist = cells <= LDS_CELLS ? lds_hist : ghist;
        for (int64_t e = tid; e < cells; e += CHI_BLOCK) hist[e] = 0;
        __syncthreads();
        for (int64_t i = tid; i < N; i += CHI_BLOCK) {
            int64_t idx = 0;
            int ok = 1;
            for (int q = 0; q < P.d; ++q) {
                const int v = data[(int64_t)P.s[q] * N + i];
                ok &= (unsigned)v < (unsigned)card[P.s[q]];
                idx += (int64_t)v * P.cum[q];
            }
            const int vx = data[(int64_t)P.a * N + i], vy = data[(int64_t)P.b * N + i];
            ok &= (unsigned)vx < (unsigned)cX && (unsigned)vy < (unsigned)cY;
            if (ok) atomicAdd(&hist[idx + cS * (vx + cX * vy)], 1);
            else bad_sample = 1;
        }
        __syncthreads();
        if (bad_sample) {
            if (tid == 0) {
                status[t] = 3;      // a sample outside [0, card): refused
                stat[t] = __builtin_nan("");
                dfout[t] = 0;
            }
            __syncthreads();
            continue;
        }
        // per-stratum marginals
        for (int64_t s = tid; s < cS; s += CHI_BLOCK) {
            int64_t m = 0;
            for (int64_t x = 0; x < cX; ++x) {
                int64_t r = 0;
                for (int64_t y = 0; y < cY; ++y) r += hist[s + cS * (x + cX * y)];
                Sx[s * cX + x] = r;
                m += r;
            }
            for (int64_t y = 0; y < cY; ++y) {
                int64_t c = 0;
                for (int64_t x = 0; x < cX; ++x) c += hist[s + cS * (x + cX * y)];
                Sy[s * cY + y] = c;
            }
            Sm[s] = m;
        }
        __syncthreads();
        // rank of each non-empty stratum (strata ascending, like the reference's filtered table)
        const int64_t per = (cS + CHI_BLOCK - 1) / CHI_BLOCK;
        const int64_t lo = std::min<int64_t>(cS, per * tid), hi = std::min<int64_t>(cS, lo + per);
        int64_t c = 0;
        for (int64_t s = lo; s < hi; ++s) c += Sm[s] != 0;
        part_cnt[tid] = c;
        __syncthreads();
        if (tid == 0) {
            int64_t acc = 0;
            for (int k = 0; k < CHI_BLOCK; ++k) { const int64_t v = part_cnt[k]; part_cnt[k] = acc; acc += v; }
        }
        __syncthreads();
        {
            int64_t r = part_cnt[tid];
            for (int64_t s = lo; s < hi; ++s) rank[s] = Sm[s] != 0 ? r++ : -1;
        }
        __syncthreads();
        // cell terms in C order of (kept stratum, x, y); df per stratum into part_cnt
        int64_t dfl = 0;
        for (int64_t s = tid; s < cS; s += CHI_BLOCK) {
            const int64_t k = rank[s];
            if (k < 0) continue;
            const double sm = (double)Sm[s];
            int64_t zr = 0, zc = 0;
            for (int64_t x = 0; x < cX; ++x) zr += Sx[s * cX + x] == 0;
            for (int64_t y = 0; y < cY; ++y) zc += Sy[s * cY + y] == 0;
            dfl += (cX - 1 - zr) * (cY - 1 - zc);
            for (int64_t x = 0; x < cX; ++x)
                for (int64_t y = 0; y < cY; ++y) {
                    const double e = (double)(Sx[s * cX + x] * Sy[s * cY + y]) / sm;
                    const double cnt = (double)hist[s + cS * (x + cX * y)];
                    const double e1 = e == 0.0 ? 1.0 : e;
                    double term;
                    if (!g_sq) {
                        const double dlt = cnt - e;
                        term = (dlt * dlt) / e1;
                    } else {
                        double div = cnt / e1;
                        if (div == 0.0) div = 1.0;
                        term = cnt * log(div);
                    }
                    terms[(k * cX + x) * cY + y] = term;
                }
        }
        __syncthreads();
        part_cnt[tid] = dfl;
        __syncthreads();
        if (tid == 0) {
            int64_t df = 0, kept = 0;
            for (int k = 0; k < CHI_BLOCK; ++k) df += part_cnt[k];
            for (int64_t s = 0; s < cS; ++s) kept += Sm[s] != 0;
            // numpy reduces a contiguous array in buffer-sized blocks of 8192 elements: pairwise
            // inside a block, blocks accumulated in order onto 0.0
            const int64_t total = kept * cX * cY;
            double v = 0.0;
            for (int64_t b0 = 0; b0 < total; b0 += 8192) v += np_pairwise_sum(terms + b0, min((int64_t)8192, total - b0));
            if (g_sq) v = 2.0 * v;
            stat[t] = v;
            dfout[t] = df;
            status[t] = 0;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" int pcg_chisq_batch(pcg_handle *h, const int32_t *data, int64_t N, int64_t n, const int32_t *card,
                               const int32_t *tests, int32_t stride, int64_t count, int g_sq, int64_t max_cells,
                               double *stat, int64_t *df, int32_t *status) {
    if (!h) return PCG_ERR_INVALID;
    if (count < 0 || n < 2 || N < 1 || stride < 3 || stride > PCG_MAX_LEVEL_DEPTH + 3 || max_cells < 1 ||
        max_cells > ((int64_t)1 << 26))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_chisq_batch: bad shape (n=%lld N=%lld stride=%d max_cells=%lld)",
                        (long long)n, (long long)N, stride, (long long)max_cells);
    if (count == 0) return PCG_OK;
    if (!data || !card || !tests || !stat || !df || !status)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_chisq_batch: null pointer");
    PCG_HIP(h, hipSetDevice(h->device));
    const int64_t per_block = (int64_t)((sizeof(int) * max_cells + 15) & ~(size_t)15) +
                              (int64_t)(sizeof(double) + 4 * sizeof(int64_t)) * max_cells;
    // blocks in flight: enough to fill the chip, bounded by a 1 GiB scratch
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>({count, 4096, ((int64_t)1 << 30) / per_block}));
    if (!pcg_ensure(h, h->chisq_scratch, (size_t)(per_block * grid)))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_chisq_batch: scratch (%lld B)", (long long)(per_block * grid));
    hipLaunchKernelGGL(k_chisq, dim3((unsigned)grid), dim3(CHI_BLOCK), 0, h->stream, data, N, (int)n, card, tests,
                       (int)stride, count, g_sq ? 1 : 0, max_cells, (char *)h->chisq_scratch.p, per_block, stat, df,
                       status);
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}
