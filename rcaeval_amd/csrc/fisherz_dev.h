// fisherz_dev.h — device-side Fisher-z arithmetic shared by the skeleton kernels.
//
// causal-learn 0.1.3.3 FisherZ.__call__ [U] (call sites RCAEval/e2e/pc_pagerank.py:19,
// RCAEval/graph_construction/pc.py:15):
//   inv = np.linalg.inv(C[ix_(var,var)]); r = -inv[0,1]/sqrt(inv[0,0]*inv[1,1])
//   Z = 0.5*log((1+r)/(1-r)); X = sqrt(N-|S|-3)*|Z|; p = 2*(1 - norm.cdf(|X|))
// norm.cdf = cephes ndtr: x = a/sqrt2, z = |x|; z < 1/sqrt2 ? 0.5+0.5 erf(x)
//                                                         : (y = 0.5 erfc(z), x>0 ? 1-y : y)
// The cancellation 2*(1 - (1 - y)) is reproduced on purpose.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcgpu.h"

#define PCG_SQRT1_2 0.70710678118654752440

// The reference arithmetic is evaluated without fused multiply-add contraction (plain mul then
// add/sub, as the C oracle and an x86-64 build of cephes / unblocked LAPACK evaluate it): on an
// ill-conditioned sub-matrix an FMA in the LU moves p by ~cond * 2^-53, which is what the
// parity tests would otherwise see (tests/test_gpu_skeleton.py near-collinear cases).
__device__ __forceinline__ double pcg_pvalue_from_X(double X) {
#pragma clang fp contract(off)
    const double a = fabs(X);
    const double x = a * PCG_SQRT1_2;
    const double z = fabs(x);
    double y;
    if (z < PCG_SQRT1_2) {
        y = 0.5 + 0.5 * erf(x);
    } else {
        y = 0.5 * erfc(z);
        if (x > 0) y = 1.0 - y;
    }
    return 2.0 * (1.0 - y);
}

// p from a partial correlation r with the reference's expression. err: 2 = math domain.
__device__ __forceinline__ double pcg_pvalue_from_r(double r, double sqrt_dof, int *err) {
#pragma clang fp contract(off)
    const double ratio = (1.0 + r) / (1.0 - r);
    if (ratio <= 0.0) {           // math.log(<= 0) raises ValueError
        *err = 2;
        return __builtin_nan("");
    }
    const double Z = 0.5 * log(ratio);
    return pcg_pvalue_from_X(sqrt_dof * fabs(Z));
}

// Exact path: numpy.linalg.inv (LAPACK dgesv with B = I) on the m x m matrix A (row-major,
// m = d + 2, in caller-provided scratch, destroyed), columns 0 and 1 only: LU with partial
// pivoting (first max |a|, dgetf2 order), forward/back substitution (dgetrs order).
// Returns 0 ok, 1 exactly singular (LAPACK INFO > 0 -> LinAlgError -> ValueError).
__device__ inline int pcg_lu_inv01(double *A, int m, int *piv, double *B0, double *B1,
                                   double *i00, double *i01, double *i11) {
#pragma clang fp contract(off)
    int info = 0;
    for (int j = 0; j < m; ++j) {
        int p = j;
        double best = fabs(A[j * m + j]);
        for (int i = j + 1; i < m; ++i) {
            const double v = fabs(A[i * m + j]);
            if (v > best) { best = v; p = i; }
        }
        piv[j] = p;
        if (A[p * m + j] != 0.0) {
            if (p != j)
                for (int k = 0; k < m; ++k) {
                    const double t = A[j * m + k];
                    A[j * m + k] = A[p * m + k];
                    A[p * m + k] = t;
                }
            const double rcp = 1.0 / A[j * m + j];
            for (int i = j + 1; i < m; ++i) A[i * m + j] *= rcp;
        } else if (!info) {
            info = j + 1;
        }
        for (int i = j + 1; i < m; ++i) {
            const double l = A[i * m + j];
            for (int k = j + 1; k < m; ++k) A[i * m + k] -= l * A[j * m + k];
        }
    }
    if (info) return 1;
    for (int c = 0; c < 2; ++c) {
        double *B = c ? B1 : B0;
        for (int i = 0; i < m; ++i) B[i] = (i == c) ? 1.0 : 0.0;
        for (int i = 0; i < m; ++i) {
            const int p = piv[i];
            if (p != i) { const double t = B[i]; B[i] = B[p]; B[p] = t; }
        }
        for (int i = 0; i < m; ++i)
            for (int k = 0; k < i; ++k) B[i] -= A[i * m + k] * B[k];
        for (int i = m - 1; i >= 0; --i) {
            for (int k = i + 1; k < m; ++k) B[i] -= A[i * m + k] * B[k];
            B[i] /= A[i * m + i];
        }
    }
    *i00 = B0[0];
    *i01 = B1[0];
    *i11 = B1[1];
    return 0;
}

// pcg_lu_inv01 with the matrix in registers (M = d + 2 known at compile time): the same
// operations in the same order (pivot search, row swap, scaling, elimination, dgetrs
// substitutions), the dynamic pivot row selected instead of indexed — bitwise the same result.
template <int M>
__device__ inline int pcg_lu_inv01_reg(double (&A)[M][M], double *i00, double *i01, double *i11) {
#pragma clang fp contract(off)
    int info = 0;
    int piv[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        int p = j;
        double best = fabs(A[j][j]);
#pragma unroll
        for (int i = j + 1; i < M; ++i) {
            const double v = fabs(A[i][j]);
            if (v > best) { best = v; p = i; }
        }
        piv[j] = p;
        double rp[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
            double t = A[j][k];
#pragma unroll
            for (int i = j + 1; i < M; ++i)
                if (p == i) t = A[i][k];
            rp[k] = t;
        }
        if (rp[j] != 0.0) {
            if (p != j) {
#pragma unroll
                for (int k = 0; k < M; ++k) {
#pragma unroll
                    for (int i = j + 1; i < M; ++i)
                        if (p == i) A[i][k] = A[j][k];
                    A[j][k] = rp[k];
                }
            }
            const double rcp = 1.0 / A[j][j];
#pragma unroll
            for (int i = j + 1; i < M; ++i) A[i][j] *= rcp;
        } else if (!info) {
            info = j + 1;
        }
#pragma unroll
        for (int i = j + 1; i < M; ++i) {
            const double l = A[i][j];
#pragma unroll
            for (int k = j + 1; k < M; ++k) A[i][k] -= l * A[j][k];
        }
    }
    if (info) return 1;
    double B0[M], B1[M];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        double B[M];
#pragma unroll
        for (int i = 0; i < M; ++i) B[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int p = piv[i];
            if (p != i) {
                double bp = B[i];
#pragma unroll
                for (int q = i + 1; q < M; ++q)
                    if (p == q) bp = B[q];
#pragma unroll
                for (int q = i + 1; q < M; ++q)
                    if (p == q) B[q] = B[i];
                B[i] = bp;
            }
        }
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
            for (int k = 0; k < i; ++k) B[i] -= A[i][k] * B[k];
#pragma unroll
        for (int i = M - 1; i >= 0; --i) {
#pragma unroll
            for (int k = i + 1; k < M; ++k) B[i] -= A[i][k] * B[k];
            B[i] /= A[i][i];
        }
#pragma unroll
        for (int i = 0; i < M; ++i) (c ? B1 : B0)[i] = B[i];
    }
    *i00 = B0[0];
    *i01 = B1[0];
    *i11 = B1[1];
    return 0;
}

// Binomial table: binom[c * PCG_BK + k] = C(c, k), saturated at UINT64_MAX.
#define PCG_BK (PCG_MAX_LEVEL_DEPTH + 1)

__device__ __forceinline__ uint64_t pcg_binom(const uint64_t *tab, int c, int k) {
    return (c < k || c < 0) ? 0ull : tab[(int64_t)c * PCG_BK + k];
}

// Colex unranking of a d-subset of {0..D-1}: rank = sum_i C(c_i, i), c_1 < ... < c_d.
// Writes k[0..d-1] ascending (k[i] = c_{i+1}).
template <int DM>
__device__ __forceinline__ void pcg_unrank_colex(uint64_t rank, int d, int D, const uint64_t *tab,
                                                 int (&k)[DM]) {
    int hi = D;  // c_i < hi
#pragma unroll
    for (int ii = DM - 1; ii >= 0; --ii) {
        if (ii < d) {
            const int i = ii + 1;  // subset position (1-based) holding c_i
            // largest c in [ii, hi-1] with C(c, i) <= rank
            int lo = ii, up = hi - 1;
            while (lo < up) {
                const int mid = (lo + up + 1) >> 1;
                if (pcg_binom(tab, mid, i) <= rank) lo = mid; else up = mid - 1;
            }
            k[ii] = lo;
            rank -= pcg_binom(tab, lo, i);
            hi = lo;
        }
    }
}
