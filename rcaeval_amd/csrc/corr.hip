// corr.hip — K1: numpy.corrcoef(data.T) on MI355X fp64 MFMA.
//
// Replaces FisherZ.__init__'s `self.correlation_matrix = np.corrcoef(data.T)` [U]
// (causal-learn 0.1.3.3 utils/cit.py). numpy's order:
//   avg = X.mean(axis=1); X -= avg; c = dot(X, X.T); c *= 1/(N-1);
//   s = sqrt(diag(c)); c /= s[:, None]; c /= s[None, :]; clip(c, -1, 1)
// X here is the caller's N x n (time x metrics) array, so c = Xc^T Xc.
//
// GEMM: 64 x 64 output tile per 256-thread block (4 waves, 32 x 32 per wave = 2 x 2
// v_mfma_f64_16x16x4_f64 tiles), K (time) staged through LDS in 16-row slabs, double
// buffered; the mean subtraction is fused into the staging load. Only upper-triangle
// tiles are computed (c is symmetric); the epilogue mirrors them. Roofline: MFMA fp64
// (2*N*n^2 flops); bytes 8*N*n*(n/64) staged per tile row, L2-served.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "handle.h"

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int TILE = 64;
constexpr int KT = 16;
constexpr int PAD = 1;  // LDS row padding (doubles) against bank conflicts
constexpr int MEAN_ROWS = 256;

// partial column sums over row chunks (deterministic two-pass mean)
__global__ void k_colsum_partial(const double *X, int64_t N, int n, int64_t ldx, double *part) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.y * MEAN_ROWS;
    if (j >= n) return;
    const int64_t r1 = std::min<int64_t>(r0 + MEAN_ROWS, N);
    double s = 0.0;
    for (int64_t t = r0; t < r1; ++t) s += X[t * ldx + j];
    part[(int64_t)blockIdx.y * n + j] = s;
}

__global__ void k_colmean(const double *part, int nchunks, int n, int64_t N, double *mean) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    double s = 0.0;
    for (int c = 0; c < nchunks; ++c) s += part[(int64_t)c * n + j];
    mean[j] = s / (double)N;
}

__device__ __forceinline__ void tile_of(int t, int T, int &bi, int &bj) {
    // t-th upper-triangle tile (bi <= bj), row-major over bi
    int row = 0, rem = t;
    while (rem >= T - row) { rem -= T - row; ++row; }
    bi = row;
    bj = row + rem;
}

__global__ __launch_bounds__(256) void k_xtx(const double *X, int64_t N, int n, int64_t ldx,
                                            const double *mean, int ntiles, int64_t kchunk, double *G,
                                            int64_t ldg, int64_t slab_stride) {
    __shared__ double As[2][KT][TILE + PAD];
    __shared__ double Bs[2][KT][TILE + PAD];
    const int T = (n + TILE - 1) / TILE;
    int bi, bj;
    tile_of(blockIdx.x % ntiles, T, bi, bj);
    const int slab = blockIdx.x / ntiles;           // split-K slice
    const int64_t kbeg = (int64_t)slab * kchunk;
    const int64_t kend = std::min<int64_t>(N, kbeg + kchunk);
    G += (int64_t)slab * slab_stride;
    const int i0 = bi * TILE, j0 = bj * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;

    // staging: 16 x 64 slab = 1024 doubles per operand, 4 per thread
    const int sc = tid & 63;          // column within the tile
    const int sr = tid >> 6;          // rows sr, sr+4, sr+8, sr+12
    const double ma = (i0 + sc < n) ? mean[i0 + sc] : 0.0;
    const double mb = (j0 + sc < n) ? mean[j0 + sc] : 0.0;
    const bool va = i0 + sc < n, vb = j0 + sc < n;

    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

    double ra[4], rb[4];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t t = t0 + sr + 4 * q;
            const bool vt = t < kend;
            ra[q] = (vt && va) ? X[t * ldx + i0 + sc] - ma : 0.0;
            rb[q] = (vt && vb) ? X[t * ldx + j0 + sc] - mb : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            As[buf][sr + 4 * q][sc] = ra[q];
            Bs[buf][sr + 4 * q][sc] = rb[q];
        }
    };

    const int64_t nk = (kend - kbeg + KT - 1) / KT;
    load(kbeg);
    store(0);
    __syncthreads();
    const int fr = lane & 15, fk = lane >> 4;
    for (int64_t kk = 0; kk < nk; ++kk) {
        const int buf = (int)(kk & 1);
        if (kk + 1 < nk) load(kbeg + (kk + 1) * KT);
#pragma unroll
        for (int k4 = 0; k4 < KT; k4 += 4) {
            double a0 = As[buf][k4 + fk][wr + fr];
            double a1 = As[buf][k4 + fk][wr + 16 + fr];
            double b0 = Bs[buf][k4 + fk][wc + fr];
            double b1 = Bs[buf][k4 + fk][wc + 16 + fr];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (kk + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    // epilogue: C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * r
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wr + 16 * a + (lane >> 4) + 4 * r;
                const int j = j0 + wc + 16 * b + (lane & 15);
                if (i < n && j < n) {
                    const double v = acc[a][b][r];
                    if (bi != bj) {
                        G[(int64_t)i * ldg + j] = v;
                        G[(int64_t)j * ldg + i] = v;
                    } else if (i <= j) {
                        G[(int64_t)i * ldg + j] = v;
                        G[(int64_t)j * ldg + i] = v;
                    }
                }
            }
}

// sd_i = sqrt(c_ii) with c = (sum of split-K slabs) * 1/(N-1)
__global__ void k_stddev(const double *G, int64_t ldg, int64_t slab_stride, int ks, int n, double scale,
                         double *sd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = 0.0;
    for (int s = 0; s < ks; ++s) v += G[(int64_t)s * slab_stride + (int64_t)i * ldg + i];
    sd[i] = sqrt(v * scale);
}

// C_ij = clip(((sum_s G_s,ij) * 1/(N-1) / sd_i) / sd_j, -1, 1)   (numpy corrcoef order)
__global__ void k_normalize(const double *G, int64_t ldg, int64_t slab_stride, int ks, double *C, int64_t ldc,
                            int n, double scale, const double *sd) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n) return;
    double g = 0.0;
    for (int s = 0; s < ks; ++s) g += G[(int64_t)s * slab_stride + (int64_t)i * ldg + j];
    double v = (g * scale) / sd[i];
    v = v / sd[j];
    C[(int64_t)i * ldc + j] = v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v);  // NaN passes through
}

}  // namespace

extern "C" int pcg_corr(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C,
                        int64_t ldc) {
    if (!h || !X || !C || N < 2 || n < 1 || ldx < n || ldc < n || n > (1 << 24))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_corr: invalid arguments");
    PCG_HIP(h, hipSetDevice(h->device));
    const int nchunks = (int)((N + MEAN_ROWS - 1) / MEAN_ROWS);
    if (!pcg_ensure(h, h->colmean, sizeof(double) * ((size_t)n * (nchunks + 2))))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_corr scratch");
    double *part = (double *)h->colmean.p;
    double *mean = part + (size_t)n * nchunks;
    double *sd = mean + n;
    const int nn = (int)n;
    hipLaunchKernelGGL(k_colsum_partial, dim3((nn + 255) / 256, nchunks), dim3(256), 0, h->stream, X, N, nn,
                       ldx, part);
    hipLaunchKernelGGL(k_colmean, dim3((nn + 255) / 256), dim3(256), 0, h->stream, part, nchunks, nn, N, mean);
    const int T = (nn + TILE - 1) / TILE;
    const int ntiles = T * (T + 1) / 2;
    // split K so that the grid covers the chip (~8 blocks per CU); slabs summed in order later
    int ks = (int)std::min<int64_t>(std::max<int64_t>(1, (2048 + ntiles - 1) / ntiles), std::max<int64_t>(1, N / 512));
    ks = std::min(ks, 16);
    const int64_t kchunk = (((N + ks - 1) / ks) + KT - 1) / KT * KT;
    ks = (int)((N + kchunk - 1) / kchunk);
    double *G = C;
    int64_t ldg = ldc, stride = 0;
    if (ks > 1) {
        stride = (int64_t)nn * nn;
        if (!pcg_ensure(h, h->pr_scratch, sizeof(double) * (size_t)stride * ks))
            return pcg_fail(h, PCG_ERR_OOM, "pcg_corr split-K slabs");
        G = (double *)h->pr_scratch.p;
        ldg = nn;
    }
    const double scale = 1.0 / (double)(N - 1);
    hipLaunchKernelGGL(k_xtx, dim3(ntiles * ks), dim3(256), 0, h->stream, X, N, nn, ldx, mean, ntiles, kchunk, G,
                       ldg, stride);
    hipLaunchKernelGGL(k_stddev, dim3((nn + 255) / 256), dim3(256), 0, h->stream, G, ldg, stride, ks, nn, scale, sd);
    hipLaunchKernelGGL(k_normalize, dim3((nn + 255) / 256, nn), dim3(256), 0, h->stream, G, ldg, stride, ks, C, ldc,
                       nn, scale, sd);
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}
