// pagerank.hip — K4: ranking heads on the GPU.
//
// (1) scikit-network 0.31.0 PageRank(damping_factor=0.85, solver='piteration', n_iter=10,
//     tol=1e-6).fit_transform(A) [U], as called at RCAEval/e2e/pc_pagerank.py:31-32 and
//     RCAEval/graph_heads/page_rank.py:85-89. Restated semantics:
//       out_deg = A @ 1 (bool);  a = (d * normalize(A, p=1)).T  (CSR, rows sorted by column)
//       b = (1 - d * out_deg) * seeds,  seeds = 1/m
//       scores = b; repeat n_iter: s_ = a @ scores + b * sum(scores); s_ /= sum(s_)
//                    if ||scores - s_||_1 < tol: break  else scores = s_
//       return scores / sum(scores)
//     Sums use numpy's pairwise summation (8 accumulators, 128-element leaves), the SpMV
//     scipy's sequential row order without FMA contraction, so ties rank identically.
// (2) RandomWalkScorer._walk (RCAEval/graph_heads/random_walk.py:179-186): numpy
//     Generator(PCG64).choice(index, p=column) draws — cdf = cumsum(p); cdf /= cdf[-1];
//     idx = searchsorted(cdf, random(), 'right'), random() = (next64 >> 11) * 2^-53.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "handle.h"

#pragma clang fp contract(off)

namespace {

constexpr int PR_THREADS = 1024;
constexpr int MAX_LEAVES = 1024;
constexpr int PR_LDS_M = 768;    // 5 * 768 doubles + colptr = 33 KiB of dynamic LDS beside the ~25 KiB static (< 64 KiB)

// numpy pairwise_sum leaf (n <= 128)
__device__ double pw_leaf(const double *a, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

struct Leaves {
    int count;
    int start[MAX_LEAVES];
    int len[MAX_LEAVES];
    // post-order program: op >= 0 push leaf op; op == -1 pop two, push sum
    int nprog;
    int prog[2 * MAX_LEAVES];
};
// k_pagerank's LDS: static (Leaves, leaf sums, total_nnz, block_pw_sum's result) + the dynamic
// per-node vectors and column pointers for m <= PR_LDS_M must fit one workgroup's 64 KiB
static_assert(sizeof(Leaves) + MAX_LEAVES * sizeof(double) + 32 + 5 * PR_LDS_M * sizeof(double) +
                      (PR_LDS_M + 1) * sizeof(int32_t) <= 65536,
              "k_pagerank LDS budget");

__device__ void pw_plan(Leaves &L, int n) {  // thread 0 only
    int st_s[64], st_n[64], st_state[64], sp = 0;
    L.count = 0;
    L.nprog = 0;
    st_s[0] = 0; st_n[0] = n; st_state[0] = 0; sp = 1;
    while (sp) {
        const int s = st_s[sp - 1], len = st_n[sp - 1];
        if (len <= 128) {
            L.start[L.count] = s;
            L.len[L.count] = len;
            L.prog[L.nprog++] = L.count++;
            --sp;
            continue;
        }
        int n2 = len / 2;
        n2 -= n2 % 8;
        if (st_state[sp - 1] == 0) {
            st_state[sp - 1] = 1;
            st_s[sp] = s; st_n[sp] = n2; st_state[sp] = 0; ++sp;
        } else if (st_state[sp - 1] == 1) {
            st_state[sp - 1] = 2;
            st_s[sp] = s + n2; st_n[sp] = len - n2; st_state[sp] = 0; ++sp;
        } else {
            L.prog[L.nprog++] = -1;
            --sp;
        }
    }
}

// block-wide pairwise sum of v[0..n) (optionally of |v|) — identical to numpy add.reduce
__device__ double block_pw_sum(const double *v, const Leaves &L, double *leafsum, bool absval,
                               double *tmp) {
    const double *src = v;
    if (absval) {
        for (int i = threadIdx.x; i < L.start[L.count - 1] + L.len[L.count - 1]; i += blockDim.x)
            tmp[i] = fabs(v[i]);
        __syncthreads();
        src = tmp;
    }
    for (int l = threadIdx.x; l < L.count; l += blockDim.x) leafsum[l] = pw_leaf(src + L.start[l], L.len[l]);
    __syncthreads();
    __shared__ double result;
    if (threadIdx.x == 0) {
        double st[64];
        int sp = 0;
        for (int k = 0; k < L.nprog; ++k) {
            const int op = L.prog[k];
            if (op >= 0) st[sp++] = leafsum[op];
            else { const double b = st[--sp]; const double a = st[--sp]; st[sp++] = a + b; }
        }
        result = st[0];
    }
    __syncthreads();
    const double r = result;
    __syncthreads();
    return r;
}

// scratch layout (global): colptr[m+1] int | rowidx[nnz] int | val[nnz] | b[m] | s[m] | s_[m] | tmp[m]
__global__ __launch_bounds__(PR_THREADS) void k_pagerank(const double *A, int m, int64_t lda,
                                                         const int32_t *indptr, const int32_t *indices,
                                                         const double *data, double damping, int n_iter,
                                                         double tol, int32_t *colptr, int32_t *rowidx,
                                                         double *val, double *work, double *scores,
                                                         int64_t nnz_cap, int *status) {
    __shared__ Leaves L;
    __shared__ double leafsum[MAX_LEAVES];
    __shared__ int total_nnz;
    __shared__ int bad_csr;
    // the five per-node vectors live in LDS for m <= PR_LDS_M (every iteration's sums and
    // sweeps then avoid global round trips between barriers), else in the global scratch
    extern __shared__ double pr_lds[];
    if (m <= PR_LDS_M) {
        work = pr_lds;
        colptr = reinterpret_cast<int32_t *>(pr_lds + 5 * m);   // thread 0's prefix scan stays in LDS
    }
    double *b = work, *s = work + m, *s2 = work + 2 * m, *tmp = work + 3 * m, *inv = work + 4 * m;
    const int tid = threadIdx.x;
    if (tid == 0) pw_plan(L, m);
    // out-degree sums (row sums in column order) and their pseudo-inverse
    for (int j = tid; j < m; j += blockDim.x) {
        double rs = 0.0;
        if (A) {
            for (int k = 0; k < m; ++k) rs += fabs(A[(int64_t)j * lda + k]);
        } else {
            for (int q = indptr[j]; q < indptr[j + 1]; ++q) rs += fabs(data[q]);
        }
        inv[j] = rs != 0.0 ? 1.0 / rs : 0.0;
        b[j] = (1.0 - damping * (rs != 0.0 ? 1.0 : 0.0)) * (1.0 / (double)m);
    }
    __syncthreads();
    // transposed CSR of (d * D^-1 A): row i of a lists j ascending with A[j, i] != 0
    if (A) {
        for (int i = tid; i < m; i += blockDim.x) {
            int c = 0;
            for (int j = 0; j < m; ++j) c += A[(int64_t)j * lda + i] != 0.0;
            colptr[i + 1] = c;
        }
    } else {
        for (int i = tid; i <= m; i += blockDim.x) colptr[i] = 0;
        if (tid == 0) bad_csr = 0;
        __syncthreads();
        for (int j = tid; j < m; j += blockDim.x) {
            if (indptr[j + 1] < indptr[j] || indptr[j] < 0) { bad_csr = 1; continue; }
            for (int q = indptr[j]; q < indptr[j + 1]; ++q)
                if (data[q] != 0.0) {
                    const int c = indices[q];
                    if ((unsigned)c < (unsigned)m) atomicAdd(&colptr[c + 1], 1);
                    else bad_csr = 1;
                }
        }
    }
    __syncthreads();
    if (!A && bad_csr) {   // malformed CSR (decreasing indptr, column out of range): refuse
        if (tid == 0) *status = 3;
        return;
    }
    if (tid == 0) {
        colptr[0] = 0;
        for (int i = 0; i < m; ++i) colptr[i + 1] += colptr[i];
        total_nnz = colptr[m];
    }
    __syncthreads();
    if (total_nnz == 0) {  // sknetwork check_format: "The input matrix is empty."
        if (tid == 0) *status = 1;
        return;
    }
    if ((int64_t)total_nnz > nnz_cap) {   // CSR caller understated nnz: refuse before the fill
        if (tid == 0) *status = 2;
        return;
    }
    if (A) {
        for (int i = tid; i < m; i += blockDim.x) {
            int p = colptr[i];
            for (int j = 0; j < m; ++j) {
                const double aij = A[(int64_t)j * lda + i];
                if (aij != 0.0) { rowidx[p] = j; val[p] = damping * (inv[j] * aij); ++p; }
            }
        }
    } else {
        for (int i = tid; i < m; i += blockDim.x) {
            int p = colptr[i];
            for (int j = 0; j < m; ++j)   // j ascending: scan rows for column i
                for (int q = indptr[j]; q < indptr[j + 1]; ++q)
                    if (indices[q] == i && data[q] != 0.0) { rowidx[p] = j; val[p] = damping * (inv[j] * data[q]); ++p; }
        }
    }
    for (int i = tid; i < m; i += blockDim.x) s[i] = b[i];
    __syncthreads();
    for (int it = 0; it < n_iter; ++it) {
        const double ssum = block_pw_sum(s, L, leafsum, false, tmp);
        for (int i = tid; i < m; i += blockDim.x) {
            double acc = 0.0;
            for (int p = colptr[i]; p < colptr[i + 1]; ++p) acc += val[p] * s[rowidx[p]];
            s2[i] = acc + b[i] * ssum;
        }
        __syncthreads();
        const double tot = block_pw_sum(s2, L, leafsum, false, tmp);
        for (int i = tid; i < m; i += blockDim.x) {
            s2[i] = s2[i] / tot;
            tmp[i] = s[i] - s2[i];
        }
        __syncthreads();
        const double diff = block_pw_sum(tmp, L, leafsum, true, tmp);
        if (diff < tol) break;  // block-uniform
        for (int i = tid; i < m; i += blockDim.x) s[i] = s2[i];
        __syncthreads();
    }
    const double fin = block_pw_sum(s, L, leafsum, false, tmp);
    for (int i = tid; i < m; i += blockDim.x) scores[i] = s[i] / fin;
    if (tid == 0) *status = 0;
}

// ---------------- random walk ----------------
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 pcg_mult() {
    return ((u128)0x2360ED051FC65DA4ull << 64) | (u128)0x4385DF649FCCF645ull;
}

__device__ u128 pcg_advance(u128 state, u128 inc, unsigned long long delta) {
    u128 cur_mult = pcg_mult(), cur_plus = inc, acc_mult = 1, acc_plus = 0;
    while (delta > 0) {
        if (delta & 1) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta >>= 1;
    }
    return acc_mult * state + acc_plus;
}

__device__ __forceinline__ double pcg_double(u128 state) {
    const unsigned rot = (unsigned)(state >> 122);
    const unsigned long long xs = (unsigned long long)(state >> 64) ^ (unsigned long long)state;
    const unsigned long long out = (xs >> rot) | (xs << ((64 - rot) & 63));
    return (double)(out >> 11) * (1.0 / 9007199254740992.0);
}

// cdf[c][r] = cumsum(P[:, c]) / cdf[-1]  (one thread per column; numpy cumsum is sequential)
__global__ void k_rw_cdf(const double *P, int m, int64_t ldp, double *cdf, int *uniform) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    double acc = 0.0;
    double *col = cdf + (int64_t)c * m;
    for (int r = 0; r < m; ++r) { acc += P[(int64_t)r * ldp + c]; col[r] = acc; }
    const double last = col[m - 1];
    for (int r = 0; r < m; ++r) col[r] = col[r] / last;
    // columns identical to column 0 -> the walk does not depend on the current node
    if (c > 0)
        for (int r = 0; r < m; ++r)
            if (P[(int64_t)r * ldp + c] != P[(int64_t)r * ldp]) { atomicAnd(uniform, 0); break; }
}

__device__ __forceinline__ int search_right(const double *cdf, int m, double u) {
    int lo = 0, hi = m;  // first index with cdf[idx] > u
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void k_rw_parallel(const double *cdf, int m, unsigned long long s_hi, unsigned long long s_lo,
                              unsigned long long i_hi, unsigned long long i_lo, int64_t num_loop,
                              unsigned long long *counts) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= num_loop) return;
    const u128 st = ((u128)s_hi << 64) | s_lo, inc = ((u128)i_hi << 64) | i_lo;
    const u128 sk = pcg_advance(st, inc, (unsigned long long)k + 1);
    const int idx = search_right(cdf, m, pcg_double(sk));
    atomicAdd(&counts[min(idx, m - 1)], 1ull);
}

__global__ void k_rw_serial(const double *cdf, int m, int64_t start, unsigned long long s_hi,
                            unsigned long long s_lo, unsigned long long i_hi, unsigned long long i_lo,
                            int64_t num_loop, unsigned long long *counts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    u128 st = ((u128)s_hi << 64) | s_lo;
    const u128 inc = ((u128)i_hi << 64) | i_lo;
    int64_t node = start;
    for (int64_t k = 0; k < num_loop; ++k) {
        st = st * pcg_mult() + inc;
        node = search_right(cdf + node * m, m, pcg_double(st));
        if (node >= m) node = m - 1;
        counts[node] += 1;
    }
}

}  // namespace

static int pagerank_common(pcg_handle *h, const double *A, const int32_t *indptr, const int32_t *indices,
                           const double *data, int64_t m, int64_t lda, int64_t nnz_hint, double damping,
                           int n_iter, double tol, double *scores) {
    PCG_HIP(h, hipSetDevice(h->device));
    const int64_t nnz_cap = A ? m * m : std::max<int64_t>(nnz_hint, 1);
    const size_t bytes = sizeof(int32_t) * (m + 1 + nnz_cap) + sizeof(double) * (nnz_cap + 5 * m) + 64;
    if (!pcg_ensure(h, h->pr_scratch, bytes)) return pcg_fail(h, PCG_ERR_OOM, "pagerank scratch");
    char *base = (char *)h->pr_scratch.p;
    int *status = (int *)base;
    int32_t *colptr = (int32_t *)(base + 16);
    int32_t *rowidx = colptr + (m + 1);
    size_t offd = (size_t)(16 + sizeof(int32_t) * (m + 1 + nnz_cap) + 15) & ~(size_t)15;
    double *val = (double *)(base + offd);
    double *work = val + nnz_cap;
    const size_t lds = m <= PR_LDS_M ? sizeof(double) * 5 * (size_t)m + sizeof(int32_t) * (size_t)(m + 1) : 0;
    const int threads = m <= 256 ? 256 : PR_THREADS;   // small graphs: cheaper block barriers
    hipLaunchKernelGGL(k_pagerank, dim3(1), dim3(threads), lds, h->stream, A, (int)m, lda, indptr, indices,
                       data, damping, n_iter, tol, colptr, rowidx, val, work, scores, nnz_cap, status);
    PCG_HIP(h, hipGetLastError());
    int st = 0;
    PCG_HIP(h, hipMemcpyAsync(&st, status, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    if (st == 1) return pcg_fail(h, PCG_ERR_INVALID, "The input matrix is empty.");
    if (st == 3) return pcg_fail(h, PCG_ERR_INVALID, "pcg_pagerank_csr: malformed CSR (indptr order or column index)");
    if (st == 2) return pcg_fail(h, PCG_ERR_INVALID, "pcg_pagerank_csr: nnz is smaller than the non-zeros in indptr");
    return PCG_OK;
}

extern "C" int pcg_pagerank_dense(pcg_handle *h, const double *A, int64_t m, int64_t lda, double damping,
                                  int n_iter, double tol, double *scores) {
    if (!h || !A || !scores || m < 1 || lda < m || m > (1 << 15))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_pagerank_dense: invalid arguments");
    if (m > MAX_LEAVES * 64) return pcg_fail(h, PCG_ERR_INVALID, "m too large");
    return pagerank_common(h, A, nullptr, nullptr, nullptr, m, lda, 0, damping, n_iter, tol, scores);
}

extern "C" int pcg_pagerank_csr(pcg_handle *h, const int32_t *indptr, const int32_t *indices, const double *data,
                                int64_t m, int64_t nnz, double damping, int n_iter, double tol, double *scores) {
    if (!h || !indptr || !indices || !data || !scores || m < 1 || m > (1 << 15) || nnz < 0)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_pagerank_csr: invalid arguments");
    return pagerank_common(h, nullptr, indptr, indices, data, m, 0, nnz, damping, n_iter, tol, scores);
}

extern "C" int pcg_random_walk(pcg_handle *h, const double *P, int64_t m, int64_t ldp, int64_t start,
                               int64_t num_loop, uint64_t state_hi, uint64_t state_lo, uint64_t inc_hi,
                               uint64_t inc_lo, int64_t *counts) {
    if (!h || !P || !counts || m < 1 || ldp < m || start < 0 || start >= m || num_loop < 0)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_random_walk: invalid arguments");
    PCG_HIP(h, hipSetDevice(h->device));
    const size_t bytes = sizeof(double) * (size_t)m * m + 64;
    if (!pcg_ensure(h, h->pr_scratch, bytes)) return pcg_fail(h, PCG_ERR_OOM, "random walk scratch");
    int *uniform = (int *)h->pr_scratch.p;
    double *cdf = (double *)((char *)h->pr_scratch.p + 64);
    const int one = 1;
    PCG_HIP(h, hipMemcpyAsync(uniform, &one, sizeof(int), hipMemcpyHostToDevice, h->stream));
    PCG_HIP(h, hipMemsetAsync(counts, 0, sizeof(int64_t) * m, h->stream));
    hipLaunchKernelGGL(k_rw_cdf, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, h->stream, P, (int)m, ldp, cdf,
                       uniform);
    int uni = 0;
    PCG_HIP(h, hipMemcpyAsync(&uni, uniform, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    if (num_loop > 0) {
        if (uni)
            hipLaunchKernelGGL(k_rw_parallel, dim3((unsigned)((num_loop + 255) / 256)), dim3(256), 0, h->stream, cdf,
                               (int)m, state_hi, state_lo, inc_hi, inc_lo, num_loop,
                               (unsigned long long *)counts);
        else
            hipLaunchKernelGGL(k_rw_serial, dim3(1), dim3(64), 0, h->stream, cdf, (int)m, start, state_hi, state_lo,
                               inc_hi, inc_lo, num_loop, (unsigned long long *)counts);
    }
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}
