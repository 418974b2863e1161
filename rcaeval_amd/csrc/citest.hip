// citest.hip — batched Fisher-z CI tests on an arbitrary list of (x, y, S).
//
// The skeleton kernels (skeleton.hip) enumerate their own work; everything else that calls
// causal-learn's `cg.ci_test(i, j, S)` / `FisherZ.__call__` [U] with sets it builds itself —
// UCSepset priority 3/4 (`find_cond_sets_without_mid` / `_with_mid`,
// lib/causallearn/graph/GraphClass.py:190-204), the order-dependent stable=False skeleton
// (SkeletonDiscovery.py:112-131), FCI's possible-d-sep stage — goes through this entry.
// One lane owns one test: gather C[var, var] (var = [a, b] + S), LU with partial pivoting
// in numpy.linalg.inv's (dgesv) order, columns 0 and 1 of the inverse, then the reference
// p expression (fisherz_dev.h). Per-lane matrices live in a handle-owned global scratch
// (m <= 32: up to 8.5 KB per lane, L2-resident for the lanes in flight).
#include <hip/hip_runtime.h>

#include "fisherz_dev.h"
#include "handle.h"

namespace {

constexpr int BATCH_BLOCK = 128;
constexpr int BATCH_MAX_LANES = 256 * 128;   // lanes in flight (scratch = lanes * (m^2 + 2m))

__global__ __launch_bounds__(BATCH_BLOCK) void k_fisherz_batch(const double *C, int64_t n, int64_t ldc,
                                                               int64_t N, const int32_t *tests, int stride,
                                                               int64_t count, int mmax, double *scratch,
                                                               double *pout, int32_t *status) {
    const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t lanes = (int64_t)gridDim.x * blockDim.x;
    double *A = scratch + lane * (int64_t)(mmax * mmax + 2 * mmax);
    int piv[PCG_MAX_LEVEL_DEPTH + 2];
    int var[PCG_MAX_LEVEL_DEPTH + 2];
    for (int64_t t = lane; t < count; t += lanes) {
        const int32_t *row = tests + t * (int64_t)stride;
        const int a = row[0], b = row[1], d = row[2];
        int bad = (d < 0 || d > PCG_MAX_LEVEL_DEPTH || d + 3 > stride || a < 0 || b < 0 || a >= n || b >= n ||
                   a == b);
        if (!bad) {
            var[0] = a;
            var[1] = b;
            for (int q = 0; q < d; ++q) {
                const int s = row[3 + q];
                bad |= (s < 0 || s >= n || s == a || s == b);
                var[2 + q] = s;
            }
        }
        if (bad) {                       // refused on the device, never dereferenced
            pout[t] = __builtin_nan("");
            status[t] = 3;
            continue;
        }
        const int m = d + 2;
        double *B0 = A + m * m, *B1 = B0 + m;
        for (int r = 0; r < m; ++r)
            for (int c = 0; c < m; ++c) A[r * m + c] = C[(int64_t)var[r] * ldc + var[c]];
        double i00, i01, i11, p = __builtin_nan("");
        int err = 0;
        if (pcg_lu_inv01(A, m, piv, B0, B1, &i00, &i01, &i11)) {
            err = 1;                      // LinAlgError -> ValueError
        } else {
            const double prod = i00 * i11;
            const int64_t dof = N - d - 3;
            if (prod < 0.0 || dof < 0) {
                err = 2;                  // math.sqrt of a negative -> ValueError
            } else {
                p = pcg_pvalue_from_r(-i01 / sqrt(prod), sqrt((double)dof), &err);
            }
        }
        pout[t] = p;
        status[t] = err;
    }
}

}  // namespace

extern "C" int pcg_fisherz_batch(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                                 const int32_t *tests, int32_t stride, int64_t count, double *p,
                                 int32_t *status) {
    if (!h) return PCG_ERR_INVALID;
    if (count < 0 || n < 2 || ldc < n || stride < 3 || stride > PCG_MAX_LEVEL_DEPTH + 3)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_fisherz_batch: bad shape (n=%lld ldc=%lld stride=%d count=%lld)",
                        (long long)n, (long long)ldc, stride, (long long)count);
    if (count == 0) return PCG_OK;
    if (!C || !tests || !p || !status) return pcg_fail(h, PCG_ERR_INVALID, "pcg_fisherz_batch: null pointer");
    PCG_HIP(h, hipSetDevice(h->device));
    const int mmax = stride - 1;                            // d <= stride - 3
    const int64_t lanes = std::min<int64_t>(BATCH_MAX_LANES, (count + BATCH_BLOCK - 1) / BATCH_BLOCK * BATCH_BLOCK);
    const size_t per = (size_t)mmax * mmax + 2 * (size_t)mmax;
    if (!pcg_ensure(h, h->batch_scratch, sizeof(double) * per * (size_t)lanes))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_fisherz_batch: scratch allocation failed");
    hipLaunchKernelGGL(k_fisherz_batch, dim3((unsigned)(lanes / BATCH_BLOCK)), dim3(BATCH_BLOCK), 0, h->stream, C,
                       n, ldc, N, tests, (int)stride, count, mmax, (double *)h->batch_scratch.p, p, status);
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}
