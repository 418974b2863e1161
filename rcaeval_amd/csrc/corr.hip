// corr.hip — K1: numpy.corrcoef(data.T) on MI355X fp64 MFMA.
//
// Replaces FisherZ.__init__'s `self.correlation_matrix = np.corrcoef(data.T)` [U]
// (causal-learn 0.1.3.3 utils/cit.py). numpy's order:
//   avg = X.mean(axis=1); X -= avg; c = dot(X, X.T); c *= 1/(N-1);
//   s = sqrt(diag(c)); c /= s[:, None]; c /= s[None, :]; clip(c, -1, 1)
// X here is the caller's N x n (time x metrics) array, so c = Xc^T Xc.
//
// GEMM: 64 x 64 output tile per 256-thread block (2 x 2 waves, 32 x 32 per wave = 2 x 2
// v_mfma_f64_16x16x4_f64 tiles), K (time) staged through LDS in 4-row slabs, double buffered,
// with the mean subtraction fused into the staging load. Only upper-triangle tiles are computed
// (c is symmetric) and only their upper triangle is written; the normalisation mirrors it
// (k_normalize_tiles, which also takes sd from the slab diagonals). K is split into fixed slabs
// (a function of n and N only, so every world size sums the same slabs in the same order);
// ~4096 blocks at n = 2000 (528 tiles x 8 slabs) keep ~8 small blocks resident per CU, which
// hides the staging latency far better than 128 x 128 tiles at 2 blocks per CU. Blocks are
// ordered XCD-major (blockIdx % 8 is the XCD the dispatcher picks), so each XCD walks whole
// slabs and reads its rows of X from HBM about once instead of once per XCD.
// Roofline: MFMA fp64 (2*N*n^2 algorithmic flops; the upper-tile work 528 * 16 * N/4 MFMAs).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "handle.h"

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

#ifndef PCG_K1_TILE
#define PCG_K1_TILE 64
#endif
#ifndef PCG_K1_XCD
#define PCG_K1_XCD 1        // 1: XCD-major block order (each XCD walks whole split-K slabs)
#endif
#ifndef PCG_K1_KS
#define PCG_K1_KS 0         // >0: force the split-K slab count (experiments)
#endif
constexpr int TILE = PCG_K1_TILE;
constexpr int WT = TILE / 32;          // 16x16 MFMA tiles per wave dimension (2 x 2 waves per block)
constexpr int RS = 256 / TILE;         // staging row step
#ifndef PCG_K1_BLOCKS
#define PCG_K1_BLOCKS 4096       // target k_xtx grid (tiles x split-K slabs)
#endif
#ifndef PCG_K1_MAXKS
#define PCG_K1_MAXKS 16
#endif
#ifndef PCG_K1_SLAB_BUDGET
#define PCG_K1_SLAB_BUDGET (64ll << 20)   // bytes of split-K partial slabs beyond PCG_K1_MAXKS
#endif
#ifndef PCG_K1_MINROWS
#define PCG_K1_MINROWS 32   // fewest rows per split-K slab
#endif
#ifndef PCG_K1_KT
#define PCG_K1_KT 4
#endif
constexpr int KT = PCG_K1_KT;
constexpr int PAD = 1;  // LDS row padding (doubles) against bank conflicts
#ifndef PCG_MEAN_ROWS
#define PCG_MEAN_ROWS 64
#endif
#ifndef PCG_COLSUM_UNROLL
#define PCG_COLSUM_UNROLL 8
#endif
constexpr int MEAN_ROWS = PCG_MEAN_ROWS;   // rows per partial column sum (N = 10k: 157 chunks x 8 column blocks)
constexpr int CS_U = PCG_COLSUM_UNROLL;    // loads in flight per thread (k_colsum_partial)

// partial column sums over row chunks (deterministic two-pass mean); with pmax / pmin also the
// chunk's column maximum and minimum (the int8 digit path's exponents)
__global__ __launch_bounds__(256) void k_colsum_partial(const double *X, int64_t N, int n, int64_t ldx, double *part,
                                                       double *pmax, double *pmin) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.y * MEAN_ROWS;
    if (j >= n) return;
    const int64_t r1 = std::min<int64_t>(r0 + MEAN_ROWS, N);
    double s = 0.0, mx = -INFINITY, mn = INFINITY;
    int64_t t = r0;
    for (; t + CS_U <= r1; t += CS_U) {     // CS_U loads in flight, summed in row order
        double v[CS_U];
#pragma unroll
        for (int k = 0; k < CS_U; ++k) v[k] = X[(t + k) * ldx + j];
#pragma unroll
        for (int k = 0; k < CS_U; ++k) {
            s += v[k];
            mx = fmax(mx, v[k]);
            mn = fmin(mn, v[k]);
        }
    }
    for (; t < r1; ++t) {
        const double v = X[t * ldx + j];
        s += v;
        mx = fmax(mx, v);
        mn = fmin(mn, v);
    }
    part[(int64_t)blockIdx.y * n + j] = s;
    if (pmax) {
        pmax[(int64_t)blockIdx.y * n + j] = mx;
        pmin[(int64_t)blockIdx.y * n + j] = mn;
    }
}

// digit exponent of column j: 2^e > max_t |fl(X_tj - mean_j)| = max(fl(max - mean), fl(mean - min))
// (rounding is monotone, so the extremes of the centred column are the centred extremes);
// K1_NONFINITE marks a column whose mean or range is not finite (numpy: that row and column of
// C are NaN)
constexpr int K1_NONFINITE = -100000;

// mean_j = (sum of the chunk partials) / N and, with pmax / pmin, the exponent e_j: 16 columns per
// block, 16 contiguous partitions of the chunk list per column (8 loads in flight each), the
// partition sums added in partition order through LDS
__global__ __launch_bounds__(256) void k_colstats(const double *part, const double *pmax, const double *pmin,
                                                 int nchunks, int n, int64_t N, double *mean, int *expo) {
    __shared__ double sq[3][16][17];
    const int c = threadIdx.x & 15, p = threadIdx.x >> 4;
    const int j = blockIdx.x * 16 + c;
    const int per = (nchunks + 15) / 16;
    const int lo = min(nchunks, p * per), hi = min(nchunks, lo + per);
    double s = 0.0, mx = -INFINITY, mn = INFINITY;
    if (j < n) {
        int k = lo;
        for (; k + 8 <= hi; k += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(k + u) * n + j];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; k < hi; ++k) s += part[(int64_t)k * n + j];
        if (expo)
            for (k = lo; k < hi; ++k) {
                mx = fmax(mx, pmax[(int64_t)k * n + j]);
                mn = fmin(mn, pmin[(int64_t)k * n + j]);
            }
    }
    sq[0][p][c] = s;
    sq[1][p][c] = mx;
    sq[2][p][c] = mn;
    __syncthreads();
    if (p != 0 || j >= n) return;
    double t = 0.0;
    mx = -INFINITY;
    mn = INFINITY;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        t += sq[0][q][c];
        mx = fmax(mx, sq[1][q][c]);
        mn = fmin(mn, sq[2][q][c]);
    }
    const double m = t / (double)N;
    mean[j] = m;
    if (!expo) return;
    const double amax = fmax(mx - m, m - mn);
    int e = 0;
    if (!isfinite(m) || !isfinite(amax)) e = K1_NONFINITE;
    else if (amax > 0.0) frexp(amax, &e);     // amax = f 2^e, f in [0.5, 1): |centred| / 2^e < 1
    expo[j] = e;
}

__device__ __forceinline__ void tile_of(int t, int T, int &bi, int &bj) {
    // t-th upper-triangle tile (bi <= bj), row-major over bi
    int row = 0, rem = t;
    while (rem >= T - row) { rem -= T - row; ++row; }
    bi = row;
    bj = row + rem;
}

// tl == nullptr: all upper-triangle tiles, upper triangle into G (single GPU). Otherwise tl lists
// (bi, bj, packed tile row) triples of one rank's share: rows go to packed position, no mirror.
__global__ __launch_bounds__(256) void k_xtx(const double *X, int64_t N, int n, int64_t ldx,
                                            const double *mean, int ntiles, int nslabs, int64_t kchunk,
                                            double *G, int64_t ldg, int64_t slab_stride, const int32_t *tl) {
    __shared__ double As[2][KT][TILE + PAD];
    __shared__ double Bs[2][KT][TILE + PAD];
    const int T = (n + TILE - 1) / TILE;
    int bi, bj, pbi = -1;
    int lin = blockIdx.x;
    if (PCG_K1_XCD) {       // blocks go round-robin over the 8 XCDs: give XCD x a contiguous run
        const int per = gridDim.x / 8;
        lin = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (lin >= ntiles * nslabs) return;
    }
    if (tl) {
        const int t = lin % ntiles;
        bi = tl[3 * t];
        bj = tl[3 * t + 1];
        pbi = tl[3 * t + 2];
    } else {
        tile_of(lin % ntiles, T, bi, bj);
    }
    const int slab = lin / ntiles;                  // split-K slice
    const int64_t kbeg = (int64_t)slab * kchunk;
    const int64_t kend = std::min<int64_t>(N, kbeg + kchunk);
    G += (int64_t)slab * slab_stride;
    const int i0 = bi * TILE, j0 = bj * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = (wave >> 1) * (TILE / 2), wc = (wave & 1) * (TILE / 2);

    // staging: KT x TILE slab per operand, KT/RS rows per thread (coalesced row segments)
    const int sc = tid % TILE;        // column within the tile
    const int sr = tid / TILE;        // rows sr, sr+RS, ...
    const double ma = (i0 + sc < n) ? mean[i0 + sc] : 0.0;
    const double mb = (j0 + sc < n) ? mean[j0 + sc] : 0.0;
    const bool va = i0 + sc < n, vb = j0 + sc < n;

    // each wave owns a TILE/2 square sub-tile = WT x WT MFMA 16x16 tiles
    d4 acc[WT][WT];
#pragma unroll
    for (int a = 0; a < WT; ++a)
#pragma unroll
        for (int b = 0; b < WT; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

    double ra[KT / RS], rb[KT / RS];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int q = 0; q < KT / RS; ++q) {
            const int64_t t = t0 + sr + RS * q;
            const bool vt = t < kend;
            ra[q] = (vt && va) ? X[t * ldx + i0 + sc] - ma : 0.0;
            rb[q] = (vt && vb) ? X[t * ldx + j0 + sc] - mb : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < KT / RS; ++q) {
            As[buf][sr + RS * q][sc] = ra[q];
            Bs[buf][sr + RS * q][sc] = rb[q];
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
            double av[WT], bv[WT];
#pragma unroll
            for (int q = 0; q < WT; ++q) {
                av[q] = As[buf][k4 + fk][wr + 16 * q + fr];
                bv[q] = Bs[buf][k4 + fk][wc + 16 * q + fr];
            }
#pragma unroll
            for (int a = 0; a < WT; ++a)
#pragma unroll
                for (int b = 0; b < WT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        if (kk + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    // epilogue: C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * r
#pragma unroll
    for (int a = 0; a < WT; ++a)
#pragma unroll
        for (int b = 0; b < WT; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wr + 16 * a + (lane >> 4) + 4 * r;
                const int j = j0 + wc + 16 * b + (lane & 15);
                if (i < n && j < n) {
                    const double v = acc[a][b][r];
                    if (pbi >= 0) {
                        G[((int64_t)pbi * TILE + (i - i0)) * ldg + j] = v;
                    } else if (bi != bj || i <= j) {
                        G[(int64_t)i * ldg + j] = v;   // upper triangle only: k_normalize_tiles mirrors
                    }
                }
            }
}

// ---------------------------------------------------------------------------------------
// K1 on the int8 matrix cores ("digit GEMM", PCG_K1_I8; Ozaki-style splitting).
//
// Each centred value v = fl(X_tj - mean_j) (numpy's own subtraction) is written exactly as
// v = 2^e_j * sum_{p=1..9} d_p 2^(-7p) + r, with signed digits d_p in [-127, 127] (truncation:
// y = v 2^-e_j in (-1, 1); d_p = trunc(128 y_{p-1}), y_p = 128 y_{p-1} - d_p, every step exact in
// fp64) and |r| < 2^(e_j - 63). The Gram entry is then
//     G_ij = sum_t v_ti v_tj ~= sum_{p + q <= 10} 2^(e_i + e_j - 7(p + q)) * (D_p^T D_q)_ij
// where every D_p^T D_q is an int8 GEMM accumulated EXACTLY in int32 (v_mfma_i32_32x32x32_i8):
// the products of one level l = p + q share a scale, so they share one int32 accumulator
// (at most 9 products x K x 127^2 < 2^31 for K <= K1_I8_MAXK rows per split-K slab). The dropped
// levels p + q > 10 and the remainders r bound the error by ~50 * 2^-63 * 2^(e_i + e_j) per
// row pair, i.e. relative to the fp64 Gram ~1e-17 x (max|v| / rms v)^2 -- far below fp64
// dot-product rounding. The levels are combined in fp64 from the smallest (exact int32 ->
// fp64, exact power-of-two scaling, 8 rounded adds), then the split-K slabs and the numpy-order
// normalisation run as in the fp64 path (k_normalize_tiles / k_slab_sum / k_gather_finish).
// Cost: 45 int8 GEMMs of the upper triangle = 45 x N n^2 int8 MACs at 2x the BF16 MFMA rate
// (vs N n^2 fp64 MACs at 1/32 of it), plus one pass that writes 9 digit planes.
#ifndef PCG_K1_DIG
#define PCG_K1_DIG 9          // digits per value (7 bits each); A/B knob
#endif
constexpr int K1_DIG = PCG_K1_DIG;
constexpr int K1_LEVELS = K1_DIG;            // p + q = 2 .. K1_DIG + 1
constexpr int K1_TB = 32;                    // rows (t) per digit block = the MFMA K
constexpr int K1_I8_MAXK = 14336;            // rows per slab: 9 * 14336 * 127^2 < 2^31
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

// t-th upper-triangle tile in supertile order: 8 x 8 groups of tiles (upper triangle of the
// group grid, row-major; inside a group row-major, bi <= bj on the diagonal groups). An XCD runs
// a contiguous run of blocks, so its ~64 resident blocks share 8 row panels and 8 column panels
// per K block (k_xtx's row-major order shares one row panel and streams 64 column panels).
#ifndef PCG_K1_SUPER
#define PCG_K1_SUPER 8
#endif
__device__ __forceinline__ void tile_of_super(int t, int T, int &bi, int &bj) {
    constexpr int S = PCG_K1_SUPER;
    const int ST = (T + S - 1) / S;
    for (int si = 0; si < ST; ++si)
        for (int sj = si; sj < ST; ++sj) {
            const int r0 = si * S, r1 = min(T, r0 + S), c0 = sj * S, c1 = min(T, c0 + S);
            const int m = r1 - r0, w = c1 - c0;
            const int cnt = si == sj ? m * (m + 1) / 2 : m * w;
            if (t >= cnt) { t -= cnt; continue; }
            if (si == sj) {
                int row = 0;
                while (t >= m - row) { t -= m - row; ++row; }
                bi = r0 + row;
                bj = r0 + row + t;
            } else {
                bi = r0 + t / w;
                bj = c0 + t % w;
            }
            return;
        }
    bi = bj = 0;
}

// digit planes, blocked for the GEMM: Dg[((p * CB + cb) * TB + tb) * 2048 + (tt >> 4) * 1024 + c * 16
// + (tt & 15)] is digit p of column 64 cb + c at row 32 tb + tt (2 KB blocks, k-half major like the
// CRT residue planes: conflict-free fragment reads); rows past N and columns past n are zero. One
// block: 64 columns x 64 rows, transposed through LDS.
__global__ __launch_bounds__(256) void k_digits(const double *X, int64_t N, int n, int64_t ldx, const double *mean,
                                               const int *expo, int CB, int TB, int8_t *Dg) {
    __shared__ __attribute__((aligned(16))) int8_t tile[K1_DIG][2][2][64][16];   // [p][tb][k-half][col][t]
    const int cb = blockIdx.x, t64 = blockIdx.y;
    const int c = threadIdx.x & 63, r4 = threadIdx.x >> 6;
    const int j = cb * 64 + c;
    const bool vj = j < n;
    const int e = vj ? expo[j] : 0;
    const bool live = vj && e != K1_NONFINITE;
    const double m = vj ? mean[j] : 0.0;
    // this thread: rows 16 r4 .. 16 r4 + 15 of column c; the 16 digits of one plane pack into
    // one 16-byte LDS store
    double y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t t = (int64_t)t64 * 64 + r4 * 16 + i;
        y[i] = (live && t < N) ? ldexp(X[t * ldx + j] - m, -e) : 0.0;
    }
#pragma unroll
    for (int p = 0; p < K1_DIG; ++p) {
        v4i pk = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            y[i] *= 128.0;
            const double d = trunc(y[i]);
            y[i] -= d;
            pk[i >> 2] |= ((int)d & 255) << (8 * (i & 3));
        }
        *reinterpret_cast<v4i *>(&tile[p][r4 >> 1][r4 & 1][c][0]) = pk;
    }
    __syncthreads();
    // 9 x 2 blocks of 2 KB out: 16-byte stores, consecutive threads on consecutive addresses
    const v4i *src = reinterpret_cast<const v4i *>(&tile[0][0][0][0]);
    for (int q = threadIdx.x; q < K1_DIG * 2 * 128; q += 256) {
        const int blk = q >> 7, w = q & 127;         // blk = p * 2 + half
        const int p = blk >> 1, tb = t64 * 2 + (blk & 1);
        if (tb >= TB) continue;
        v4i *dst = reinterpret_cast<v4i *>(Dg + (((int64_t)p * CB + cb) * TB + tb) * 2048);
        dst[w] = src[q];
    }
}

// the digit GEMM of one 64 x 64 upper-triangle tile and one split-K slab (k_xtx's tiling, block
// order and output conventions). 4 waves, each a 32 x 32 quarter: lane (r = l & 31, h = l >> 5)
// feeds row / column r, rows t = 16h .. 16h + 15 of the block (A and B take the same k layout,
// so the MFMA's k order inside a lane does not matter). LDS: two stages x 18 digit blocks.
__global__ __launch_bounds__(256, 2) void k_xtx_i8(const int8_t *Dg, int CB, int TB, int n, const int *expo,
                                                 int ntiles, int nslabs, int kb, double *G, int64_t ldg,
                                                 int64_t slab_stride, const int32_t *tl, int super_order) {
    __shared__ __attribute__((aligned(16))) int8_t st[2][2 * K1_DIG][2048];
    const int T = (n + 63) / 64;
    int bi, bj, pbi = -1;
    int lin = blockIdx.x;
    if (PCG_K1_XCD) {
        const int per = gridDim.x / 8;
        lin = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (lin >= ntiles * nslabs) return;
    }
    if (tl) {
        const int t = lin % ntiles;
        bi = tl[3 * t];
        bj = tl[3 * t + 1];
        pbi = tl[3 * t + 2];
    } else if (super_order) {
        tile_of_super(lin % ntiles, T, bi, bj);
    } else {
        tile_of(lin % ntiles, T, bi, bj);
    }
    const int slab = lin / ntiles;
    const int tb0 = slab * kb, tb1 = min(TB, tb0 + kb);
    G += (int64_t)slab * slab_stride;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;

    v16i acc[K1_LEVELS];
#pragma unroll
    for (int l = 0; l < K1_LEVELS; ++l)
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[l][k] = 0;

    // staging: 18 blocks of 2 KB = 2304 16-byte words, 9 per thread; thread tid moves words
    // q * 256 + tid, i.e. block (q * 256 + tid) >> 7 (a digit of tile row bi for blocks < 9, of
    // tile column bj after), word (q * 256 + tid) & 127
    const v4i *srcq[K1_DIG];
#pragma unroll
    for (int q = 0; q < K1_DIG; ++q) {
        const int o = q * 256 + tid;
        const int blk = o >> 7, w = o & 127;
        const int p = blk < K1_DIG ? blk : blk - K1_DIG;
        const int cbk = blk < K1_DIG ? bi : bj;
        srcq[q] = reinterpret_cast<const v4i *>(Dg + ((int64_t)p * CB + cbk) * TB * 2048) + w;
    }
    v4i pre[K1_DIG];
#define K1_LOAD(tb_)                                                                   \
    _Pragma("unroll") for (int q = 0; q < K1_DIG; ++q) pre[q] = srcq[q][(int64_t)(tb_) * 128];
#define K1_STORE(buf_)                                                                 \
    _Pragma("unroll") for (int q = 0; q < K1_DIG; ++q)                                 \
        reinterpret_cast<v4i *>(&st[(buf_)][0][0])[q * 256 + tid] = pre[q];
    if (tb0 < tb1) {
        K1_LOAD(tb0);
        K1_STORE(0);
    }
    __syncthreads();
    for (int tb = tb0; tb < tb1; ++tb) {
        const int buf = (tb - tb0) & 1;
        if (tb + 1 < tb1) { K1_LOAD(tb + 1); }
        v4i bq[K1_DIG];
#pragma unroll
        for (int q = 0; q < K1_DIG; ++q)
            bq[q] = *reinterpret_cast<const v4i *>(&st[buf][K1_DIG + q][hh * 1024 + (wc + r) * 16]);
#pragma unroll
        for (int p = 0; p < K1_DIG; ++p) {
            const v4i ap = *reinterpret_cast<const v4i *>(&st[buf][p][hh * 1024 + (wr + r) * 16]);
#pragma unroll
            for (int q = 0; q < K1_DIG - p; ++q)         // level p + q (0-based) <= K1_DIG - 1
                acc[p + q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ap, bq[q], acc[p + q], 0, 0, 0);
        }
        if (tb + 1 < tb1) { K1_STORE(buf ^ 1); }
        __syncthreads();
    }
#undef K1_LOAD
#undef K1_STORE
    // epilogue: C/D map of the 32 x 32 forms: col = lane & 31, row = (k & 3) + 8 (k >> 2) + 4 h
    const int j = bj * 64 + wc + r;
    const int ej = j < n ? expo[j] : 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int i = bi * 64 + wr + (k & 3) + 8 * (k >> 2) + 4 * hh;
        if (i >= n || j >= n) continue;
        const int ei = expo[i];
        double v = 0.0;
        if (ei == K1_NONFINITE || ej == K1_NONFINITE) {
            v = NAN;
        } else {
#pragma unroll
            for (int l = K1_LEVELS - 1; l >= 0; --l)   // smallest level first; level l is p + q = l + 2
                v += ldexp((double)acc[l][k], ei + ej - 7 * (l + 2));
        }
        if (pbi >= 0) {
            G[((int64_t)pbi * 64 + (i - bi * 64)) * ldg + j] = v;
        } else if (bi != bj || i <= j) {
            G[(int64_t)i * ldg + j] = v;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K1 on the int8 matrix cores, CRT form (PCG_K1_CRT, the default for n >= 256; the Ozaki
// scheme II split: linear in the number of moduli instead of quadratic in the digits).
//
// Each centred value is truncated to a b-bit integer on its column's scale,
//     a_tj = trunc(v_tj 2^(b - e_j)),  |a_tj| < 2^b,  v_tj = fl(X_tj - mean_j),
// and the integer Gram A^T A is computed EXACTLY through the Chinese remainder theorem. For k
// pairwise coprime moduli m_i <= 256 with M = prod m_i > 2 N 4^b, (A^T A) mod m_i is one int8
// GEMM of the balanced residue planes (a mod m_i in [-128, 127]) accumulated exactly in int32
// (|sum| <= rows x 128^2 < 2^31 per split-K slab), and the k residues determine every entry
// (|G| < N 4^b < M / 2): x = sum_i z_i M_i - q M with M_i = M / m_i, z_i = r_i M_i^-1 mod m_i
// and q = round(sum_i z_i / m_i), built in 32-bit limbs and rounded to fp64 once,
// G_ij = x 2^(e_i + e_j - 2b). The only error is the truncation, 2^-b of the column scale
// (b >= 56; b = 59 with k = 17 at N = 10^4); the digit path's 45 GEMMs become k.
// Kernels: k_residues (the k residue planes, the digit path's blocked layout), k_xtx_crt
// (one 256 x 256 upper tile x one modulus x one split-K slab per 512-thread block, operands
// staged by LDS-DMA through an 8-slot ring of k-blocks, 6 in flight; the residue
// sums of the slab written mod m as bytes in the MFMA's own lane order), k_crt_finish (slab sums,
// the CRT rebuild, the upper triangle of G), then k_normalize_tiles as for the other paths.
// A result is the correctly rounded fp64 of the exact truncated Gram, so every tile split,
// slab split and world size gives the same bits.
constexpr int CRT_KMAX = 24;               // moduli (M < 2^192)
constexpr int CRT_L = 6;                   // 32-bit limbs of M
constexpr int CRT_T = 256;                 // output tile
constexpr int CRT_KB = 4;                  // a slab's k-blocks are a multiple of this (the plan's split-K rounding)
#ifndef PCG_CRT_PR
#define PCG_CRT_PR 8
#endif
constexpr int CRT_PR = PCG_CRT_PR;         // LDS ring slots of one k-block (16 KB: A and B, 4 column blocks x 2 KB each)
#ifndef PCG_CRT_KP
#define PCG_CRT_KP 1
#endif
constexpr int CRT_KP = PCG_CRT_KP;         // k-blocks per phase (one block barrier each)
constexpr int CRT_PL = CRT_PR - 2 * CRT_KP;   // k-blocks in flight (a slot is restaged >= 2 phases after its last read)
static_assert(CRT_PR * 16384 <= 160 * 1024 && CRT_PL >= CRT_KP && CRT_PL % CRT_KP == 0, "CRT LDS ring");
constexpr int CRT_MAXKB = 4095;            // k-blocks per slab: 4095 x 32 x 128^2 < 2^31
constexpr int CRT_UNIT = CRT_T * CRT_T;    // residue bytes per (tile, modulus, slab)
static const int kCrtModuli[CRT_KMAX] = {256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217,
                                         211, 199, 197, 193, 191, 181, 179, 173, 167, 163, 157, 151};

struct CrtTab {
    int k, b, L;                    // moduli, bits of |a|, limbs of M
    int m[CRT_KMAX];
    int y[CRT_KMAX];                // (M / m_i)^-1 mod m_i
    float finv[CRT_KMAX];           // fl(1 / m_i)
    double dinv[CRT_KMAX];
    uint32_t wlo[CRT_KMAX], whi[CRT_KMAX];   // bytes 2^(8q) mod m_i, 2^(32 + 8q) mod m_i (q = 0..3)
    uint32_t cneg[CRT_KMAX];        // -(2^b mod m_i) as u32: the offset's residue, subtracted in the dot
    uint32_t Mi[CRT_KMAX][2 * CRT_L];   // M / m_i, little-endian 16-bit limbs (one per word)
    uint32_t M[2 * CRT_L];
};

// the CRT sum of one entry: S = sum_i z_i M_i in 16-bit limb accumulators (z_i < 256, limbs
// < 2^16: full-rate 24-bit multiply-adds, sums < 24 x 2^24), fs = sum_i z_i / m_i
// (L = tab.L 32-bit limbs, a template parameter: no per-limb branches)
template <int L>
struct CrtAcc {
    uint32_t l[2 * L];
    float fs;      // |x| / M <= 0.4966 (the plan's 0.01-bit margin): fp32's ~1e-6 error picks q exactly
};

template <int L>
__device__ __forceinline__ void crt_acc_init(CrtAcc<L> &a) {
#pragma unroll
    for (int l = 0; l < 2 * L; ++l) a.l[l] = 0;
    a.fs = 0.0f;
}

template <int L>
__device__ __forceinline__ void crt_acc_add(CrtAcc<L> &a, uint32_t z, int mi, const CrtTab &tab) {
    a.fs = fmaf((float)z, tab.finv[mi], a.fs);
#pragma unroll
    for (int l = 0; l < 2 * L; ++l) a.l[l] = __umul24(z, tab.Mi[mi][l]) + a.l[l];
}

// G = x 2^(ei + ej - 2b) with x = S - q M, q = round(fs): |x| < M / 2, rounded to fp64 once
template <int L>
__device__ __forceinline__ double crt_value(const CrtAcc<L> &a, const CrtTab &tab, int ei, int ej) {
    const int32_t qq = (int32_t)floorf(a.fs + 0.5f);
    uint32_t lim[CRT_L];
    int32_t carry = 0;
#pragma unroll
    for (int l = 0; l < CRT_L; ++l) {          // 16-bit carries (every term < 2^29), two limbs per word
        int32_t v0 = carry, v1;
        if (l < L) v0 += (int32_t)a.l[2 * l] - qq * (int32_t)tab.M[2 * l];
        const uint32_t lo = (uint32_t)v0 & 0xffffu;
        v1 = v0 >> 16;                          // arithmetic: the sign carries on
        if (l < L) v1 += (int32_t)a.l[2 * l + 1] - qq * (int32_t)tab.M[2 * l + 1];
        lim[l] = lo | ((uint32_t)v1 << 16);
        carry = v1 >> 16;
    }
    const bool negx = carry < 0;
    if (negx) {                                 // magnitude: two's complement
        uint64_t c = 1;
#pragma unroll
        for (int l = 0; l < CRT_L; ++l) {
            const uint64_t v = (uint64_t)(~lim[l]) + c;
            lim[l] = (uint32_t)v;
            c = v >> 32;
        }
    }
    int top = -1;
#pragma unroll
    for (int l = 0; l < CRT_L; ++l)
        if (lim[l]) top = l;
    if (top < 0) return 0.0;
    // the top 96 bits (limbs top, top-1, top-2), normalised; the rest as a sticky bit
    uint32_t l2 = 0, l1 = 0, l0 = 0;
    bool sticky = false;
#pragma unroll
    for (int l = 0; l < CRT_L; ++l) {
        if (l == top) l2 = lim[l];
        if (l == top - 1) l1 = lim[l];
        if (l == top - 2) l0 = lim[l];
        if (l < top - 2 && lim[l]) sticky = true;
    }
    const int sh = __builtin_clz(l2);
    uint64_t h64 = ((uint64_t)l2 << 32) | l1;
    uint32_t low = l0;
    if (sh) {
        h64 = (h64 << sh) | (low >> (32 - sh));
        low <<= sh;
    }
    if (low || sticky) h64 |= 1;                // below the 53-bit rounding point
    const double mag = fma((double)(uint32_t)(h64 >> 32), 0x1p32, (double)(uint32_t)h64);
    const double gv = ldexp(mag, 32 * (top - 1) - sh + ei + ej - 2 * tab.b);
    return negx ? -gv : gv;
}

// numpy.corrcoef's order: ((g * 1/(N-1)) / sd_row) / sd_col, clipped (NaN passes)
__device__ __forceinline__ double corr_of(double g, double scale, double sr, double sc) {
    double v = (g * scale) / sr;
    v = v / sc;
    return v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v);
}

// s mod m for 0 <= s < 2^20, all in fp32 (exact integers; the quotient off by at most one each way)
__device__ __forceinline__ uint32_t crt_mod(uint32_t s, int m, float finv) {
    const float x = (float)s, fm = (float)m;
    float r = fmaf(floorf(x * finv), -fm, x);
    r = r < 0.0f ? r + fm : r;
    r = r >= fm ? r - fm : r;
    return (uint32_t)r;
}

// residue planes in 2 KB blocks of 64 columns x 32 rows, k-half major:
// R[((mi * CBp + cb) * TB + tb) * 2048 + (tt >> 4) * 1024 + c * 16 + (tt & 15)] = a mod m_i
// (balanced, int8) of column 64 cb + c at row 32 tb + tt; zero past n and N. A lane's MFMA
// fragment (16 rows of one column) is 16 contiguous bytes and a half-wave's 32 columns are one
// contiguous 512 B (no LDS bank conflicts; the column-major [c][32] form conflicts 2-way). One
// thread = 16 rows of one column; a wave stores two contiguous 512 B runs.
__global__ __launch_bounds__(256) void k_residues(const double *X, int64_t N, int n, int64_t ldx, const double *mean,
                                                 const int *expo, int CBp, int TB, CrtTab tab, int m0, int m1,
                                                 int8_t *R) {
    const int cb = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = 32 * (w & 1) + (lane >> 1), half = lane & 1;
    const int tb = blockIdx.y * 2 + (w >> 1);
    const int j = cb * 64 + c;
    const bool vj = j < n;
    const int e = vj ? expo[j] : 0;
    const bool live = vj && e != K1_NONFINITE;
    const double mu = live ? mean[j] : 0.0;
    // offset binary: (hi, lo) = a + 2^b in [1, 2^(b+1)), so every residue is of a nonnegative
    // integer and the offset's residue 2^b mod m is subtracted inside the dot product (tab.cneg)
    uint32_t lo[16], hi[16];
    const uint32_t B = 1u << (tab.b - 32);
    const int64_t t0 = (int64_t)tb * 32 + 16 * half;
    const double *xp = X + t0 * ldx + j;                 // rows t0 + i at xp + i ldx (uniform stride)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const double v = (live && t0 + i < N) ? xp[(int64_t)i * ldx] - mu : 0.0;
        const double y = ldexp(fabs(v), tab.b - e);      // < 2^b <= 2^63, exact scaling
        const uint32_t h = (uint32_t)(y * 0x1p-32);      // truncating conversions: |a| = trunc(y)
        const uint32_t l = (uint32_t)(y - (double)h * 0x1p32);   // exact difference (multiples of ulp(y))
        const bool neg = v < 0.0;
        lo[i] = neg ? 0u - l : l;
        hi[i] = neg ? B - h - (l != 0u) : B + h;
    }
    const int64_t plane = (int64_t)CBp * TB * 2048;
    int8_t *dst = R + ((int64_t)cb * TB + tb) * 2048 + half * 1024 + c * 16;
    // bytes: the low byte of each of 4 words packed into one word (v_perm_b32)
    auto pack4 = [](uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
        const uint32_t w01 = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);
        const uint32_t w23 = __builtin_amdgcn_perm(b3, b2, 0x0c0c0400u);
        return __builtin_amdgcn_perm(w23, w01, 0x05040100u);
    };
    for (int mi = m0; mi < m1; ++mi) {           // this launch's moduli
        v4i pk;
        const int m = tab.m[mi];
        if (m == 256) {          // the low byte (2^b = 0 mod 256)
#pragma unroll
            for (int q = 0; q < 4; ++q) pk[q] = (int)pack4(lo[4 * q], lo[4 * q + 1], lo[4 * q + 2], lo[4 * q + 3]);
        } else {
            // odd m: s = a + 2^b - (2^b mod m) = a (mod m), |s| < 8 x 255^2 (exact in fp32), r = s - m
            // rint(s / m) in [-(m-1)/2, (m-1)/2] (s / m is never a half-integer for odd m, and
            // fl(1/m) moves it by < 1/(32 m)); rint and the byte via the 1.5 x 2^23 magic constant
            const f2 fi = {tab.finv[mi], tab.finv[mi]};
            const f2 nm = {-(float)m, -(float)m};
            const f2 mg = {12582912.0f, 12582912.0f};
            const uint32_t wl = tab.wlo[mi], wh = tab.whi[mi], cn = tab.cneg[mi];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t bb[4];
#pragma unroll
                for (int u = 0; u < 4; u += 2) {
                    const int i = 4 * q + u;
                    const float x0 = (float)(int)__builtin_amdgcn_udot4(
                        lo[i], wl, __builtin_amdgcn_udot4(hi[i], wh, cn, false), false);
                    const float x1 = (float)(int)__builtin_amdgcn_udot4(
                        lo[i + 1], wl, __builtin_amdgcn_udot4(hi[i + 1], wh, cn, false), false);
                    const f2 x = {x0, x1};
                    const f2 qv = __builtin_elementwise_fma(x, fi, mg) - mg;    // rint(s / m)
                    const f2 rv = __builtin_elementwise_fma(qv, nm, x) + mg;
                    // (through named floats: this compiler's __builtin_bit_cast of a vector
                    // component reads component 0)
                    const float r0 = rv.x, r1 = rv.y;
                    bb[u] = __float_as_uint(r0);
                    bb[u + 1] = __float_as_uint(r1);
                }
                pk[q] = (int)pack4(bb[0], bb[1], bb[2], bb[3]);
            }
        }
        *reinterpret_cast<v4i *>(dst + mi * plane) = pk;
    }
}

// the residue GEMM of one 256 x 256 upper tile, one modulus and one split-K slab. 8 waves as 2 x 4,
// each 128 x 64 (4 x 2 v_mfma_i32_32x32x32_i8 tiles, 128 accumulators); one k-block per phase
// from an 8-slot LDS ring (6 k-blocks in flight). Units u = (mi * ks + slab) * ntiles + tile (modulus-major: a modulus group is
// one contiguous run), this launch runs u0 .. u0 + nu - 1
// (a rank's share) and writes unit u0 + l at out + l * CRT_UNIT, in lane order:
// byte ((w * 4 + a) * 2 + b) * 1024 + lane * 16 + kk = accumulator kk of MFMA tile (a, b) of wave w.
__global__ __launch_bounds__(512, 1) void k_xtx_crt(const int8_t *R, int TB, int64_t plane, int T, int ntiles, int ks,
                                                  int kb, CrtTab tab, int64_t u0, int64_t nu, uint8_t *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int64_t lin = blockIdx.x;
    {   // XCD-contiguous runs: an XCD's resident blocks share the modulus and slab (all panels in its L2)
        const int64_t per = gridDim.x / 8;
        lin = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (lin >= nu) return;
    }
    const int64_t u = u0 + lin;
    const int t = (int)(u % ntiles);
    const int64_t sm = u / ntiles;
    const int mi = (int)(sm / ks), slab = (int)(sm % ks);
    int bi, bj;
    tile_of(t, T, bi, bj);
    const int tb0 = slab * kb, tb1 = min(TB, tb0 + kb);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, hh = lane >> 5;
    const int wr = w >> 2, wc = w & 3;

    v16i acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[a][b][q] = 0;

    // staging by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip): a ring slot is one k-block,
    // A then B, each 4 column blocks x 2 KB; a thread's DMA word is column block tid >> 7, 16-byte
    // word tid & 127 of its 2 KB block — lane-linear per wave, as the DMA writes, in the planes'
    // k-half-major order
    const int8_t *Rm = R + (int64_t)mi * plane;
    const int8_t *srcA = Rm + (int64_t)(bi * 4 + (tid >> 7)) * TB * 2048 + (tid & 127) * 16;
    const int8_t *srcB = Rm + (int64_t)(bj * 4 + (tid >> 7)) * TB * 2048 + (tid & 127) * 16;
    const int nkb = tb1 - tb0;
    // one phase per k-block p: stage k-block p + PL (2 DMAs per thread: its A and B words) into
    // ring slot (p + PL) % PR; wait (counted, never 0) until this thread's DMAs of k-block p + 1
    // landed; barrier (every wave's DMAs of p + 1 visible, every wave past its reads of the slot
    // being restaged: those were for k-block p + PL - PR <= p - 2, consumed before phase p - 1's
    // barrier); then p's 8 MFMAs on the fragments read during phase p - 1, interleaved with the
    // 6 fragment reads of k-block p + 1. The tail re-stages the last k-block (uniform counts).
    auto stage = [&](int g) {
        const int64_t tb = tb0 + min(g, nkb - 1);
        unsigned char *dst = smem + (g % CRT_PR) * 16384 + w * 1024;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(srcA + tb * 2048),
                                         (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(srcB + tb * 2048),
                                         (__attribute__((address_space(3))) void *)(dst + 8192), 16, 0, 0);
    };
    const unsigned char *fa0 = smem + (2 * wr * 2048 + hh * 1024 + r * 16);
    const unsigned char *fb0 = smem + (8192 + wc * 2048 + hh * 1024 + r * 16);
    v4i af[2][CRT_KP][4], bf[2][CRT_KP][2];
    // the fragments of k-blocks g .. g + KP - 1 into buffer sl
    auto frag = [&](int g, int sl) {
#pragma unroll
        for (int kk = 0; kk < CRT_KP; ++kk) {
            const int off = ((g + kk) % CRT_PR) * 16384;
#pragma unroll
            for (int a = 0; a < 4; ++a)
                af[sl][kk][a] = *reinterpret_cast<const v4i *>(fa0 + off + (a >> 1) * 2048 + (a & 1) * 512);
#pragma unroll
            for (int b = 0; b < 2; ++b) bf[sl][kk][b] = *reinterpret_cast<const v4i *>(fb0 + off + b * 512);
        }
    };
    // (KP > 1: a phase covers KP k-blocks — one barrier per KP k-blocks; a slot is restaged two
    // phases after the phase whose fragment reads were its last; the tail's k-blocks past nkb are
    // re-staged copies of the last one and their MFMAs are skipped)
#pragma unroll
    for (int g = 0; g < CRT_PL; ++g) stage(g);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (CRT_PL - CRT_KP)) : "memory");   // the first phase's k-blocks
    __builtin_amdgcn_s_barrier();
    frag(0, 0);
    for (int p = 0; p < nkb; p += 2 * CRT_KP) {
        // two phases per iteration, so the fragment buffers stay compile-time (first phase: buffer 0)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int q = p + h2 * CRT_KP;
            if (q < nkb) {
#pragma unroll
                for (int kk = 0; kk < CRT_KP; ++kk) stage(q + CRT_PL + kk);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (CRT_PL - CRT_KP)) : "memory");   // the next phase's
                __builtin_amdgcn_s_barrier();
                const bool nxt = q + CRT_KP < nkb;
                if (nxt) frag(q + CRT_KP, h2 ^ 1);
#pragma unroll
                for (int kk = 0; kk < CRT_KP; ++kk) {
                    if (kk > 0 && q + kk >= nkb) break;      // (wave-uniform)
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[h2][kk][a], bf[h2][kk][b], acc[a][b],
                                                                              0, 0, 0);
                }
                if (nxt) {
#pragma unroll
                    for (int u = 0; u < 6 * CRT_KP; ++u) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 2 * CRT_KP, 0);
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land in LDS after the block ends
    // epilogue: the slab's sums mod m as bytes, 16 per lane per MFMA tile (one 16-byte store)
    const int m = tab.m[mi];
    const float fm = (float)m, finv = tab.finv[mi];
    const int c16 = (int)((tab.wlo[mi] >> 16) & 0xffu);      // 2^16 mod m
    uint8_t *o = out + lin * CRT_UNIT + (int64_t)w * 8192 + lane * 16;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            v4i pk = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int v = acc[a][b][q];
                uint32_t rr;
                if (m == 256) {
                    rr = (uint32_t)v & 255u;
                } else {
                    // |v| < 2^31: t = (v >> 16)(2^16 mod m) + (v & 0xffff) = v (mod m) with |t| < 2^24
                    // (24-bit multiply), so t and t - q m are exact in fp32; q = rint(t fl(1/m)) is off
                    // the exact quotient by < 2^-7, so t - q m lies in (-m/2 - 1, m/2 + 1)
                    const int t = __mul24(v >> 16, c16) + (v & 0xffff);
                    const float tf = (float)t;
                    int x = (int)fmaf(-rintf(tf * finv), fm, tf);
                    x += x < 0 ? m : 0;
                    x -= x >= m ? m : 0;
                    rr = (uint32_t)x;
                }
                pk[q >> 2] |= (int)(rr << (8 * (q & 3)));
            }
            *reinterpret_cast<v4i *>(o + (a * 2 + b) * 1024) = pk;
        }
}

// byte offset of entry (li, lj) of a unit (the lane order of k_xtx_crt's epilogue)
__device__ __forceinline__ int crt_unit_offset(int li, int lj) {
    const int wr = li >> 7, a = (li >> 5) & 3, rr = li & 31;
    const int hh = (rr >> 2) & 1, q = (rr & 3) | ((rr >> 3) << 2);
    const int wc = lj >> 6, b = (lj >> 5) & 1, r = lj & 31;
    return ((((wr * 4 + wc) * 4 + a) * 2 + b) * 64 + r + 32 * hh) * 16 + q;
}

// sd_i = sqrt(G_ii / (N - 1)) from the diagonal entries' residues (one thread per i; every
// residue load issued before the first use)
template <int L>
__global__ __launch_bounds__(256) void k_crt_diag(const uint8_t *Rs, int T, int ntiles, int ks, CrtTab tab,
                                                 const int *expo, int n, double scale, double *sd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int bi = i / CRT_T;
    const int t = bi * T - bi * (bi - 1) / 2;          // tile (bi, bi), row-major upper triangle
    const int ei = expo[i];
    if (ei == K1_NONFINITE) {
        sd[i] = NAN;
        return;
    }
    const int k = tab.k;
    const int64_t ustride = (int64_t)ntiles * CRT_UNIT;
    const uint8_t *src = Rs + (int64_t)t * CRT_UNIT + crt_unit_offset(i % CRT_T, i % CRT_T);
    uint32_t sv[CRT_KMAX];
#pragma unroll
    for (int mi = 0; mi < CRT_KMAX; ++mi) sv[mi] = 0;
    for (int s = 0; s < ks; ++s) {
        uint32_t b[CRT_KMAX];             // unconditional loads (see k_crt_finish)
#pragma unroll
        for (int mi = 0; mi < CRT_KMAX; ++mi) b[mi] = src[((int64_t)min(mi, k - 1) * ks + s) * ustride];
#pragma unroll
        for (int mi = 0; mi < CRT_KMAX; ++mi) sv[mi] += b[mi];
    }
    CrtAcc<L> acc;
    crt_acc_init(acc);
#pragma unroll
    for (int mi = 0; mi < CRT_KMAX; ++mi)
        if (mi < k) crt_acc_add(acc, crt_mod(__umul24(sv[mi], (uint32_t)tab.y[mi]), tab.m[mi], tab.finv[mi]), mi, tab);
    sd[i] = sqrt(crt_value(acc, tab, ei, ei) * scale);
}

// the CRT rebuild fused with the normalisation: one thread = 4 entries (one 32-bit word of a
// 16-byte lane word of the units: the same column j, 4 consecutive rows i); residues summed over
// the ks slabs in u16 lanes, moduli outermost (each modulus' constants read once, 4 independent
// chains); writes C_ij and its mirror C_ji, each in numpy's division order
template <int L>
__global__ __launch_bounds__(256) void k_crt_finish(const uint8_t *Rs, int T, int ntiles, int ks, CrtTab tab,
                                                   const int *expo, int n, const double *sd, double scale, double *C,
                                                   int64_t ldc) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int t = (int)(gid >> 14), rem = (int)((gid >> 2) & 4095), g = (int)(gid & 3);
    if (t >= ntiles) return;
    int bi, bj;
    tile_of(t, T, bi, bj);
    const int lane = rem & 63, wab = rem >> 6;
    const int r = lane & 31, hh = lane >> 5;
    // ((w * 4 + a) * 2 + b), w = 4 wr + wc: k_xtx_crt's epilogue order
    const int b = wab & 1, a = (wab >> 1) & 3, wr = wab >> 5, wc = (wab >> 3) & 3;
    const int j = bj * CRT_T + wc * 64 + b * 32 + r;
    // this word: accumulators q = 4 g .. 4 g + 3, rows ibase + (q & 3) + 8 (q >> 2) = ibase + q4 + 8 g
    const int ibase = bi * CRT_T + wr * 128 + a * 32 + 4 * hh + 8 * g;
    if (j >= n || ibase > j) return;
    const int k = tab.k;
    const int ej = expo[j];
    const int64_t ustride = (int64_t)ntiles * CRT_UNIT;          // next (modulus, slab)
    const uint8_t *src = Rs + (int64_t)t * CRT_UNIT + rem * 16 + 4 * g;
    // the ks slab bytes of the 4 entries, summed in u16 lanes; every load issued before the first use
    uint32_t se[CRT_KMAX], so[CRT_KMAX];
#pragma unroll
    for (int mi = 0; mi < CRT_KMAX; ++mi) se[mi] = so[mi] = 0;
    for (int s = 0; s < ks; ++s) {
        // unconditional loads (moduli past k re-read modulus k - 1 and are never used): a guarded
        // load would be a branch with its own vmcnt(0)
        uint32_t wd[CRT_KMAX];
#pragma unroll
        for (int mi = 0; mi < CRT_KMAX; ++mi)
            wd[mi] = *reinterpret_cast<const uint32_t *>(src + ((int64_t)min(mi, k - 1) * ks + s) * ustride);
#pragma unroll
        for (int mi = 0; mi < CRT_KMAX; ++mi) {
            se[mi] += wd[mi] & 0x00ff00ffu;
            so[mi] += (wd[mi] >> 8) & 0x00ff00ffu;
        }
    }
    CrtAcc<L> acc[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) crt_acc_init(acc[q4]);
#pragma unroll
    for (int mi = 0; mi < CRT_KMAX; ++mi) {
        if (mi >= k) continue;
        const int m = tab.m[mi];
        const float fi = tab.finv[mi];
        const uint32_t y = (uint32_t)tab.y[mi];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const uint32_t sv = (((q4 & 1) ? so[mi] : se[mi]) >> (16 * (q4 >> 1))) & 0xffffu;   // < ks x 255
            // z = r M_i^-1 mod m with r = sv mod m: one reduction of sv y < 2^20
            crt_acc_add(acc[q4], crt_mod(__umul24(sv, y), m, fi), mi, tab);
        }
    }
    const double sj = sd[j];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
        const int i = ibase + q4;
        if (i > j) break;
        const int ei = expo[i];
        const double gv = (ei == K1_NONFINITE || ej == K1_NONFINITE) ? NAN : crt_value(acc[q4], tab, ei, ej);
        const double si = sd[i];
        C[(int64_t)i * ldc + j] = corr_of(gv, scale, si, sj);
        if (i != j) C[(int64_t)j * ldc + i] = corr_of(gv, scale, sj, si);
    }
}

// slab split of the digit GEMM: a function of (n, N) only (every world size sums the same slabs
// in the same order), rows per slab a multiple of the 32-row digit block and <= K1_I8_MAXK
int split_k_i8(const int64_t *tune, int n, int64_t N, int *kb_out) {
    const int T = (n + 63) / 64;
    const int ntiles = T * (T + 1) / 2;
    const int TB = (int)((N + 63) / 64 * 2);
    int ks = (int)std::max<int64_t>(1, (PCG_K1_BLOCKS + ntiles / 2) / ntiles);
    if (tune[PCG_TUNE_K1_I8_KS] > 0) ks = (int)tune[PCG_TUNE_K1_I8_KS];   // PCG_TUNE_K1_I8_KS
    ks = std::min(ks, std::max(1, TB / 2));          // >= 64 rows per slab
    ks = std::min(ks, 256);
    int kb = (TB + ks - 1) / ks;
    kb = std::min(kb, K1_I8_MAXK / K1_TB);
    *kb_out = kb;
    return (TB + kb - 1) / kb;
}

// the knobs of a handle, or the built-in / environment defaults for a null handle (the host-only
// pcg_corr_shard_bytes / pcg_k1_plan_signature calls)
struct K1Tune {
    int64_t v[PCG_TUNE_COUNT];
    explicit K1Tune(const pcg_handle *h) {
        if (h) memcpy(v, h->tune, sizeof(v));
        else pcg_tuning_defaults(v);
    }
};

// the CRT path's plan: a function of (n, N) only, so every rank and world size agrees
struct CrtPlan {
    CrtTab tab;
    int T = 0, ntiles = 0, ks = 0, kb = 0, TB = 0, CBp = 0;
    int64_t units = 0;
};

// little-endian 32-bit limb helpers for the host tables
static void big_mul_small(uint32_t *x, int L, uint32_t m) {
    uint64_t c = 0;
    for (int l = 0; l < L; ++l) {
        const uint64_t v = (uint64_t)x[l] * m + c;
        x[l] = (uint32_t)v;
        c = v >> 32;
    }
}
static uint32_t big_div_small(const uint32_t *x, int L, uint32_t m, uint32_t *q) {   // q = x / m, returns x % m
    uint64_t r = 0;
    for (int l = L - 1; l >= 0; --l) {
        const uint64_t v = (r << 32) | x[l];
        q[l] = (uint32_t)(v / m);
        r = v % m;
    }
    return (uint32_t)r;
}

// the plan's knobs are the handle's (pcg_corr_sharded agrees the resulting plan's signature
// across ranks before its all-gather, so ranks with different knobs fail together)
static bool crt_plan_build(const int64_t *tune, int n, int64_t N, CrtPlan &p);

// the plan is a pure function of (n, N) and five knobs; building it (modular inverses, the limb
// tables) costs ~25 us of host time, which sat before K1's first launch on every call: one cached
// plan per host thread
bool crt_plan(const int64_t *tune, int n, int64_t N, CrtPlan &p) {
    struct Entry {
        int64_t key[7];
        bool ok;
        CrtPlan plan;
    };
    thread_local Entry e{{-1, -1, -1, -1, -1, -1, -1}, false, CrtPlan{}};
    const int64_t key[7] = {n, N, tune[PCG_TUNE_K1_I8], tune[PCG_TUNE_K1_CRT], tune[PCG_TUNE_K1_CRT_MINN],
                            tune[PCG_TUNE_K1_CRT_BITS], tune[PCG_TUNE_K1_CRT_KS]};
    if (memcmp(key, e.key, sizeof(key)) != 0) {
        e.ok = crt_plan_build(tune, n, N, e.plan);
        memcpy(e.key, key, sizeof(key));
    }
    if (e.ok) p = e.plan;
    return e.ok;
}

static bool crt_plan_build(const int64_t *tune, int n, int64_t N, CrtPlan &p) {
    if (!tune[PCG_TUNE_K1_I8] || !tune[PCG_TUNE_K1_CRT] || n < tune[PCG_TUNE_K1_CRT_MINN]) return false;
    const int bmin = (int)std::min<int64_t>(63, std::max<int64_t>(32, tune[PCG_TUNE_K1_CRT_BITS]));   // k_residues: b in [32, 63]
    // k: the fewest moduli whose product leaves b >= bmin bits per value, M > 2 N 4^b (0.01 bit margin)
    double lm = 0.0;
    int k = 0, b = 0;
    for (; k < CRT_KMAX; ++k) {
        lm += std::log2((double)kCrtModuli[k]);
        b = (int)std::floor((lm - std::log2((double)N) - 1.0 - 0.01) / 2.0);
        if (b >= bmin) { ++k; break; }
    }
    if (b < bmin) return false;
    b = std::min(b, 63);
    CrtTab &t = p.tab;
    memset(&t, 0, sizeof(t));
    t.k = k;
    t.b = b;
    uint32_t M[CRT_L] = {1, 0, 0, 0, 0, 0};
    for (int i = 0; i < k; ++i) big_mul_small(M, CRT_L, (uint32_t)kCrtModuli[i]);
    t.L = (int)std::floor(lm / 32.0) + 1;      // M < 2^(32 L - 1)... at least one spare bit
    if (lm > 32.0 * t.L - 1.0) ++t.L;
    if (t.L > CRT_L) return false;
    for (int l = 0; l < CRT_L; ++l) {
        t.M[2 * l] = M[l] & 0xffffu;
        t.M[2 * l + 1] = M[l] >> 16;
    }
    for (int i = 0; i < k; ++i) {
        const uint32_t m = (uint32_t)kCrtModuli[i];
        t.m[i] = (int)m;
        t.finv[i] = 1.0f / (float)m;
        t.dinv[i] = 1.0 / (double)m;
        uint32_t Mi32[CRT_L], mq[CRT_L];
        big_div_small(M, CRT_L, m, Mi32);        // exact: m divides M
        for (int l = 0; l < CRT_L; ++l) {
            t.Mi[i][2 * l] = Mi32[l] & 0xffffu;
            t.Mi[i][2 * l + 1] = Mi32[l] >> 16;
        }
        const uint32_t mim = big_div_small(Mi32, CRT_L, m, mq);      // (M / m) mod m
        t.y[i] = 0;
        for (uint32_t y = 1; y < m; ++y)
            if ((mim * y) % m == 1) { t.y[i] = (int)y; break; }
        uint32_t wl = 0, wh = 0;
        for (int q = 0; q < 4; ++q) {
            uint64_t p1 = 1, p2 = 1;
            for (int s = 0; s < 8 * q; ++s) p1 = (p1 * 2) % m;
            for (int s = 0; s < 32 + 8 * q; ++s) p2 = (p2 * 2) % m;
            wl |= (uint32_t)p1 << (8 * q);
            wh |= (uint32_t)p2 << (8 * q);
        }
        t.wlo[i] = wl;
        t.whi[i] = wh;
        uint64_t pb = 1;
        for (int s2 = 0; s2 < b; ++s2) pb = (pb * 2) % m;
        t.cneg[i] = 0u - (uint32_t)pb;
    }
    p.T = (n + CRT_T - 1) / CRT_T;
    p.ntiles = p.T * (p.T + 1) / 2;
    p.CBp = p.T * 4;
    p.TB = (int)((N + 63) / 64 * 2);
    // split-K: rounds of 256 resident blocks x k-blocks per slab (~0.3 us each) + the residue bytes
    // each unit writes and k_crt_finish reads (128 KB, ~0.026 us of chip bandwidth)
    // a forced count (PCG_TUNE_K1_CRT_KS) that the k-block rounding cannot reach takes the nearest
    // achievable count (it used to fall back to one slab silently)
    int best = 1;
    double best_cost = 1e300;
    const int force = (int)tune[PCG_TUNE_K1_CRT_KS];
    for (int ks = 1; ks <= 16; ++ks) {
        int kbk = (p.TB + ks - 1) / ks;
        kbk = (kbk + CRT_KB - 1) / CRT_KB * CRT_KB;
        const int kse = (p.TB + kbk - 1) / kbk;
        if (kse != ks || kbk > CRT_MAXKB) continue;
        const int64_t U = (int64_t)p.ntiles * k * ks;
        const double cost = force > 0 ? (double)std::abs(ks - force)
                                      : (double)((U + 255) / 256) * kbk * 0.3 + (double)U * 0.026;
        if (cost < best_cost) {
            best_cost = cost;
            best = ks;
        }
    }
    {
        int kbk = (p.TB + best - 1) / best;
        kbk = (kbk + CRT_KB - 1) / CRT_KB * CRT_KB;
        if (kbk > CRT_MAXKB) return false;     // N beyond 16 slabs of 131k rows: the digit path
        p.kb = kbk;
        p.ks = (p.TB + kbk - 1) / kbk;
    }
    p.units = (int64_t)p.ntiles * k * p.ks;
    return true;
}

// the residue planes of X into h->k1_digits
// the residue planes of moduli m0 .. m1 - 1 into h->k1_digits (allocated for all k)
int crt_residues(pcg_handle *h, const CrtPlan &p, const double *X, int64_t N, int nn, int64_t ldx, const double *mean,
                 const int *expo, int m0, int m1, hipStream_t st, const int8_t **R) {
    const size_t bytes = (size_t)p.tab.k * p.CBp * p.TB * 2048;
    if (!pcg_ensure(h, h->k1_digits, bytes)) return pcg_fail(h, PCG_ERR_OOM, "K1 residue planes (%zu bytes)", bytes);
    hipLaunchKernelGGL(k_residues, dim3((unsigned)p.CBp, (unsigned)(p.TB / 2)), dim3(256), 0, st, X, N, nn, ldx, mean,
                       expo, p.CBp, p.TB, p.tab, m0, m1, (int8_t *)h->k1_digits.p);
    *R = (const int8_t *)h->k1_digits.p;
    return PCG_OK;
}

// units u0 .. u0 + nu - 1 of the residue GEMM into out
void crt_gemm(pcg_handle *h, const CrtPlan &p, const int8_t *R, int64_t u0, int64_t nu, uint8_t *out) {
    if (nu <= 0) return;
    const int64_t plane = (int64_t)p.CBp * p.TB * 2048;
    hipLaunchKernelGGL(k_xtx_crt, dim3((unsigned)((nu + 7) / 8 * 8)), dim3(512), CRT_PR * 16384, h->stream, R,
                       p.TB, plane, p.T, p.ntiles, p.ks, p.kb, p.tab, u0, nu, out);
}

// C from the units' residues: the diagonal (sd) first, then every upper entry and its mirror
void crt_finish(pcg_handle *h, const CrtPlan &p, const uint8_t *Rs, const int *expo, int nn, int64_t N, double *sd,
                double *C, int64_t ldc) {
    const double scale = 1.0 / (double)(N - 1);
    const int64_t threads = (int64_t)p.ntiles * 16384;
#define CRT_LAUNCH(L_)                                                                                       \
    do {                                                                                                     \
        hipLaunchKernelGGL((k_crt_diag<L_>), dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, h->stream, Rs, \
                           p.T, p.ntiles, p.ks, p.tab, expo, nn, scale, sd);                                  \
        hipLaunchKernelGGL((k_crt_finish<L_>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,         \
                           h->stream, Rs, p.T, p.ntiles, p.ks, p.tab, expo, nn, (const double *)sd, scale, C, \
                           ldc);                                                                              \
    } while (0)
    if (p.tab.L <= 4) { CRT_LAUNCH(4); }
    else if (p.tab.L == 5) { CRT_LAUNCH(5); }
    else { CRT_LAUNCH(6); }
#undef CRT_LAUNCH
}

// digits of X (all columns) into h->k1_digits; returns the plane geometry
int k1_digits(pcg_handle *h, const double *X, int64_t N, int nn, int64_t ldx, const double *mean, const int *expo,
              int *CB, int *TB, const int8_t **Dg) {
    *CB = (nn + 63) / 64;
    *TB = (int)((N + 63) / 64 * 2);
    const size_t bytes = (size_t)K1_DIG * *CB * *TB * 2048;
    if (!pcg_ensure(h, h->k1_digits, bytes)) return pcg_fail(h, PCG_ERR_OOM, "K1 digit planes (%zu bytes)", bytes);
    hipLaunchKernelGGL(k_digits, dim3((unsigned)*CB, (unsigned)(*TB / 2)), dim3(256), 0, h->stream, X, N, nn, ldx,
                       mean, expo, *CB, *TB, (int8_t *)h->k1_digits.p);
    *Dg = (const int8_t *)h->k1_digits.p;
    return PCG_OK;
}

// C_ij = clip(((sum_s G_s,ij) * 1/(N-1) / sd_i) / sd_j, -1, 1)   (numpy corrcoef order)
// G holds the upper triangle only (i <= j). One block per 64 x 64 tile pair (bi <= bj): the
// slab sums of the upper tile go through LDS so both C[i][j] and C[j][i] are written as
// coalesced rows; each side keeps numpy's own division order ((g * scale) / sd_row) / sd_col,
// so C is not forced to be bitwise symmetric (numpy's is not either).
constexpr int NT = 64;
__device__ __forceinline__ double slab_diag_sd(const double *G, int64_t ldg, int64_t slab_stride, int ks, int i,
                                               double scale) {
    double v = 0.0;    // sd_i = sqrt(c_ii), c = (sum of split-K slabs in slab order) * 1/(N-1)
    for (int s = 0; s < ks; ++s) v += G[(int64_t)s * slab_stride + (int64_t)i * ldg + i];
    return sqrt(v * scale);
}

__global__ __launch_bounds__(256) void k_normalize_tiles(const double *G, int64_t ldg, int64_t slab_stride, int ks,
                                                         double *C, int64_t ldc, int n, double scale) {
    __shared__ double t[NT][NT + 1];
    __shared__ double sdr[NT], sdc[NT];
    const int T = (n + NT - 1) / NT;
    int bi = 0, bj = 0;
    {   // upper-triangle tile index -> (bi, bj), row-major over bi
        int r = blockIdx.x;
        while (r >= T - bi) { r -= T - bi; ++bi; }
        bj = bi + r;
    }
    const int i0 = bi * NT, j0 = bj * NT;
    const int c = threadIdx.x & 63, r4 = threadIdx.x >> 6;
    if (r4 == 0 && i0 + c < n) sdr[c] = slab_diag_sd(G, ldg, slab_stride, ks, i0 + c, scale);
    if (r4 == 1 && j0 + c < n) sdc[c] = slab_diag_sd(G, ldg, slab_stride, ks, j0 + c, scale);
    {   // all 16 rows of this thread in flight per slab; slabs summed in order 0..ks-1
        constexpr int RPT = NT / 4;
        double g[RPT];
        bool live[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int rr = r4 + 4 * q, i = i0 + rr, j = j0 + c;
            live[q] = i < n && j < n && (bi != bj || rr <= c);
            g[q] = 0.0;
        }
        // four slabs' loads in flight at a time (small n splits K into up to 256 slabs); the adds
        // stay in slab order
        const int64_t off0 = (int64_t)(i0 + r4) * ldg + j0 + c;
        int s = 0;
        for (; s + 4 <= ks; s += 4) {
            double v[4][RPT];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int q = 0; q < RPT; ++q)
                    v[k][q] = live[q] ? G[(int64_t)(s + k) * slab_stride + off0 + (int64_t)4 * q * ldg] : 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int q = 0; q < RPT; ++q) g[q] += v[k][q];
        }
        for (; s < ks; ++s) {
            const double *Gs = G + (int64_t)s * slab_stride;
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if (live[q]) g[q] += Gs[off0 + (int64_t)4 * q * ldg];
        }
#pragma unroll
        for (int q = 0; q < RPT; ++q) t[r4 + 4 * q][c] = g[q];
    }
    __syncthreads();
    for (int rr = r4; rr < NT; rr += 4) {
        const int i = i0 + rr, j = j0 + c;          // upper side: row i, column j
        if (i < n && j < n && (bi != bj || rr <= c)) {
            double v = (t[rr][c] * scale) / sdr[rr];
            v = v / sdc[c];
            C[(int64_t)i * ldc + j] = v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v);  // NaN passes through
        }
        const int p = j0 + rr, q = i0 + c;          // lower side: row p (tile bj), column q (tile bi)
        if (p < n && q < n && (bi != bj || c < rr)) {
            double v = (t[c][rr] * scale) / sdc[rr];
            v = v / sdr[c];
            C[(int64_t)p * ldc + q] = v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v);
        }
    }
}

// packed[r][j] = sum_s G_s[r][j] in slab order (the order k_normalize_tiles uses)
__global__ void k_slab_sum(const double *G, int64_t slab_stride, int ks, int64_t count, double *out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    double g = 0.0;
    for (int s = 0; s < ks; ++s) g += G[(int64_t)s * slab_stride + e];
    out[e] = g;
}

// zig-zag owner of tile row r among `world` ranks (2 rows per rank per period of 2*world):
// rank q owns rows m == q and m == 2*world-1-q of every period, so the upper-triangle work
// (T - r tiles in row r) is balanced
__host__ __device__ __forceinline__ void shard_slot(int r, int world, int &owner, int &local) {
    const int period = 2 * world, q = r / period, m = r % period;
    owner = m < world ? m : period - 1 - m;
    local = 2 * q + (m < world ? 0 : 1);
}

// C from the gathered packed Gram rows of every rank: unpack (upper from the owner of the
// smaller tile row), sd from the diagonal, normalize + clip in numpy.corrcoef order —
// bitwise the single-GPU pcg_corr result (same slab split, same summation order)
__global__ void k_gather_finish_sd(const double *Gg, int64_t rows_per_rank, int n, int world, double scale,
                                   double *sd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int owner, local;
    shard_slot(i / TILE, world, owner, local);
    const double g = Gg[((int64_t)owner * rows_per_rank + (int64_t)local * TILE + (i % TILE)) * n + i];
    sd[i] = sqrt(g * scale);
}

__global__ void k_gather_finish(const double *Gg, int64_t rows_per_rank, int n, int world, double scale,
                                const double *sd, double *C, int64_t ldc) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n) return;
    // (p, q) = the position the single-GPU path computes (upper tile, i <= j inside diagonal
    // tiles) and mirrors
    const bool up = (i / TILE) < (j / TILE) || ((i / TILE) == (j / TILE) && i <= j);
    const int p = up ? i : j, q = up ? j : i;
    int owner, local;
    shard_slot(p / TILE, world, owner, local);
    const double g = Gg[((int64_t)owner * rows_per_rank + (int64_t)local * TILE + (p % TILE)) * n + q];
    double v = (g * scale) / sd[i];
    v = v / sd[j];
    C[(int64_t)i * ldc + j] = v > 1.0 ? 1.0 : (v < -1.0 ? -1.0 : v);
}

// split-K factor: a function of the problem only (n, N), so every world size sums the
// same slabs in the same order; ~2048 blocks in all (n = 2000: 136 upper tiles x 15) fill
// 256 CUs x 2 blocks in four even rounds, and 1/2/4/8 ranks in whole rounds, with
// little tail at 1..8 ranks
int split_k(int n, int64_t N, int64_t *kchunk_out) {
    const int T = (n + TILE - 1) / TILE;
    const int ntiles = T * (T + 1) / 2;
    // slab cap: PCG_K1_MAXKS for large n (each slab is a full n x n partial); small n (the RQ2
    // cases: one tile, tens of variables) may split K much further so the grid is not a
    // handful of blocks walking thousands of rows each
    const int64_t slab_bytes = (int64_t)T * TILE * T * TILE * 8;
    const int maxks = (int)std::min<int64_t>(256, std::max<int64_t>(PCG_K1_MAXKS, PCG_K1_SLAB_BUDGET / slab_bytes));
    int ks = (int)std::min<int64_t>(std::max<int64_t>(1, (PCG_K1_BLOCKS + ntiles / 2) / ntiles),
                                    std::max<int64_t>(1, N / PCG_K1_MINROWS));
    ks = std::min(ks, maxks);
    if (PCG_K1_KS > 0) ks = (int)std::min<int64_t>(PCG_K1_KS, std::max<int64_t>(1, N / KT));
    const int64_t kchunk = (((N + ks - 1) / ks) + KT - 1) / KT * KT;
    *kchunk_out = kchunk;
    return (int)((N + kchunk - 1) / kchunk);
}

unsigned xtx_grid(int blocks) { return PCG_K1_XCD ? (unsigned)((blocks + 7) / 8 * 8) : (unsigned)blocks; }

// column means (and, for the digit path, the per-column digit exponents)
int column_means(pcg_handle *h, const double *X, int64_t N, int nn, int64_t ldx, double **mean_out,
                 int **expo_out = nullptr) {
    const int nchunks = (int)((N + MEAN_ROWS - 1) / MEAN_ROWS);
    const size_t parts = (size_t)nn * nchunks * (expo_out ? 3 : 1);
    h->k1_stamp_ok = false;          // h->colmean is rewritten: no shard's exponents survive
    if (!pcg_ensure(h, h->colmean, sizeof(double) * (parts + nn) + sizeof(int) * nn))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_corr scratch");
    double *part = (double *)h->colmean.p;
    double *mean = part + parts;
    double *pmax = expo_out ? part + (size_t)nn * nchunks : nullptr;
    double *pmin = expo_out ? pmax + (size_t)nn * nchunks : nullptr;
    hipLaunchKernelGGL(k_colsum_partial, dim3((nn + 255) / 256, nchunks), dim3(256), 0, h->stream, X, N, nn, ldx,
                       part, pmax, pmin);
    int *expo = expo_out ? reinterpret_cast<int *>(mean + nn) : nullptr;
    hipLaunchKernelGGL(k_colstats, dim3((nn + 15) / 16), dim3(256), 0, h->stream, (const double *)part,
                       (const double *)pmax, (const double *)pmin, nchunks, nn, N, mean, expo);
    if (expo_out) *expo_out = expo;
    *mean_out = mean;
    return PCG_OK;
}

}  // namespace

// a signature of K1's plan for (n, N) (path, and the CRT path's k, b, split-K and unit count):
// ranks whose environments select different plans would all-gather mismatched units
int64_t k1_plan_signature(const pcg_handle *h, int64_t n, int64_t N) {
    const K1Tune t(h);
    CrtPlan cp;
    if (crt_plan(t.v, (int)n, N, cp))
        return ((int64_t)1 << 62) | ((int64_t)cp.tab.k << 48) | ((int64_t)cp.tab.b << 40) | ((int64_t)cp.ks << 32) |
               (cp.units & 0xffffffffll);
    if (!t.v[PCG_TUNE_K1_I8]) return 2;
    int kb = 0;                               // the digit path: its slab split and tile order
    const int ks = split_k_i8(t.v, (int)n, N, &kb);
    return ((int64_t)1 << 61) | ((int64_t)ks << 32) | ((int64_t)kb << 8) | (t.v[PCG_TUNE_K1_SUPER_ORDER] ? 1 : 0);
}

extern "C" int pcg_k1_plan_signature(pcg_handle *h, int64_t n, int64_t N, int64_t *signature) {
    if (n < 1 || N < 2 || n > (1 << 24) || !signature) return pcg_fail(h, PCG_ERR_INVALID, "pcg_k1_plan_signature");
    *signature = k1_plan_signature(h, n, N);
    return PCG_OK;
}

extern "C" int pcg_corr_shard_rows(int64_t n, int world, int64_t *rows_per_rank) {
    if (n < 1 || world < 1 || !rows_per_rank) return PCG_ERR_INVALID;
    const int64_t T = (n + TILE - 1) / TILE;
    *rows_per_rank = (int64_t)TILE * 2 * ((T + 2 * world - 1) / (2 * world));
    return PCG_OK;
}

// bytes of one rank's share (the pcg_corr_shard buffer; the all-gather moves world x this): the
// CRT path's residue units, else the digit / fp64 path's packed Gram rows
extern "C" int pcg_corr_shard_bytes(pcg_handle *h, int64_t n, int64_t N, int world, int64_t *bytes_per_rank) {
    if (n < 1 || N < 2 || world < 1 || n > (1 << 24) || !bytes_per_rank) return PCG_ERR_INVALID;
    const K1Tune t(h);
    CrtPlan cp;
    if (crt_plan(t.v, (int)n, N, cp)) {
        *bytes_per_rank = (cp.units + world - 1) / world * (int64_t)CRT_UNIT;
        return PCG_OK;
    }
    int64_t rows = 0;
    pcg_corr_shard_rows(n, world, &rows);
    *bytes_per_rank = rows * n * (int64_t)sizeof(double);
    return PCG_OK;
}

// the per-column exponents column_means left in h->colmean (the CRT finish of a shard call)
static int *colmean_expo(pcg_handle *h, int64_t N, int nn) {
    const int nchunks = (int)((N + MEAN_ROWS - 1) / MEAN_ROWS);
    return reinterpret_cast<int *>((double *)h->colmean.p + (size_t)nn * nchunks * 3 + nn);
}

extern "C" int pcg_corr_shard(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, int rank,
                              int world, double *packed) {
    if (!h || !X || !packed || N < 2 || n < 1 || ldx < n || n > (1 << 24) || world < 1 || rank < 0 ||
        rank >= world)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_corr_shard: invalid arguments");
    PCG_HIP(h, hipSetDevice(h->device));
    const int nn = (int)n;
    CrtPlan cp;
    if (crt_plan(h->tune, nn, N, cp)) {     // this rank's contiguous run of (tile, modulus, slab) units
        double *mean;
        int *expo = nullptr;
        int rc = column_means(h, X, N, nn, ldx, &mean, &expo);
        if (rc) return rc;
        h->k1_stamp[0] = N;
        h->k1_stamp[1] = nn;
        h->k1_stamp[2] = cp.tab.k;
        h->k1_stamp[3] = ((int64_t)cp.tab.b << 32) | ((int64_t)cp.ks << 16) | cp.kb;
        h->k1_stamp_ok = true;
        const int8_t *R = nullptr;
        rc = crt_residues(h, cp, X, N, nn, ldx, mean, expo, 0, cp.tab.k, h->stream, &R);
        if (rc) return rc;
        const int64_t per = (cp.units + world - 1) / world, u0 = per * rank;
        crt_gemm(h, cp, R, u0, std::min<int64_t>(per, cp.units - u0), (uint8_t *)packed);
        PCG_HIP(h, hipGetLastError());
        PCG_HIP(h, hipStreamSynchronize(h->stream));
        return PCG_OK;
    }
    int64_t rows = 0;
    pcg_corr_shard_rows(n, world, &rows);
    PCG_HIP(h, hipMemsetAsync(packed, 0, sizeof(double) * rows * nn, h->stream));
    const int T = (nn + TILE - 1) / TILE;
    std::vector<int32_t> tl;
    for (int bi = 0; bi < T; ++bi) {
        int owner, local;
        shard_slot(bi, world, owner, local);
        if (owner != rank) continue;
        for (int bj = bi; bj < T; ++bj) {
            tl.push_back(bi);
            tl.push_back(bj);
            tl.push_back(local);
        }
    }
    const int ntiles = (int)(tl.size() / 3);
    if (ntiles == 0) return PCG_OK;
    const bool i8 = h->tune[PCG_TUNE_K1_I8] != 0;
    double *mean;
    int *expo = nullptr;
    int rc = column_means(h, X, N, nn, ldx, &mean, i8 ? &expo : nullptr);
    if (rc) return rc;
    int64_t kchunk = 0;
    int kb = 0;
    const int ks = i8 ? split_k_i8(h->tune, nn, N, &kb) : split_k(nn, N, &kchunk);
    const int64_t stride = rows * nn;
    if (!pcg_ensure(h, h->pr_scratch, sizeof(double) * ((size_t)stride * (ks > 1 ? ks : 0) + tl.size())))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_corr_shard slabs");
    double *G = ks > 1 ? (double *)h->pr_scratch.p : packed;
    int32_t *tld = reinterpret_cast<int32_t *>((double *)h->pr_scratch.p + (ks > 1 ? (size_t)stride * ks : 0));
    PCG_HIP(h, hipMemcpyAsync(tld, tl.data(), sizeof(int32_t) * tl.size(), hipMemcpyHostToDevice, h->stream));
    if (ks > 1) PCG_HIP(h, hipMemsetAsync(G, 0, sizeof(double) * (size_t)stride * ks, h->stream));
    if (i8) {
        int CB = 0, TB = 0;
        const int8_t *Dg = nullptr;
        rc = k1_digits(h, X, N, nn, ldx, mean, expo, &CB, &TB, &Dg);
        if (rc) return rc;
        hipLaunchKernelGGL(k_xtx_i8, dim3(xtx_grid(ntiles * ks)), dim3(256), 0, h->stream, Dg, CB, TB, nn,
                           (const int *)expo, ntiles, ks, kb, G, (int64_t)nn, stride, (const int32_t *)tld, 0);
    } else {
        hipLaunchKernelGGL(k_xtx, dim3(xtx_grid(ntiles * ks)), dim3(256), 0, h->stream, X, N, nn, ldx, mean, ntiles,
                           ks, kchunk, G, (int64_t)nn, stride, (const int32_t *)tld);
    }
    if (ks > 1)
        hipLaunchKernelGGL(k_slab_sum, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, h->stream, G, stride,
                           ks, stride, packed);
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}

extern "C" int pcg_corr_shard_finish(pcg_handle *h, const double *gathered, int64_t N, int64_t n, int world,
                                     double *C, int64_t ldc) {
    if (!h || !gathered || !C || N < 2 || n < 1 || ldc < n || world < 1)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_corr_shard_finish: invalid arguments");
    PCG_HIP(h, hipSetDevice(h->device));
    const int nn = (int)n;
    const double scale = 1.0 / (double)(N - 1);
    CrtPlan cp;
    if (crt_plan(h->tune, nn, N, cp)) {     // gathered = every unit in canonical order; exponents from pcg_corr_shard
        if (!h->k1_stamp_ok || h->k1_stamp[0] != N || h->k1_stamp[1] != nn || h->k1_stamp[2] != cp.tab.k ||
            h->k1_stamp[3] != (((int64_t)cp.tab.b << 32) | ((int64_t)cp.ks << 16) | cp.kb))
            return pcg_fail(h, PCG_ERR_INVALID,
                            "pcg_corr_shard_finish: no CRT-mode pcg_corr_shard of (N %lld, n %lld) on this handle since "
                            "the last K1 call", (long long)N, (long long)n);
        if (!pcg_ensure(h, h->pr_scratch, sizeof(double) * (size_t)(nn + 32)))
            return pcg_fail(h, PCG_ERR_OOM, "pcg_corr_shard_finish scratch");
        crt_finish(h, cp, (const uint8_t *)gathered, colmean_expo(h, N, nn), nn, N, (double *)h->pr_scratch.p, C,
                   ldc);
        PCG_HIP(h, hipGetLastError());
        PCG_HIP(h, hipStreamSynchronize(h->stream));
        return PCG_OK;
    }
    int64_t rows = 0;
    pcg_corr_shard_rows(n, world, &rows);
    h->k1_stamp_ok = false;          // sd overwrites h->colmean
    if (!pcg_ensure(h, h->colmean, sizeof(double) * ((size_t)nn * 2)))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_corr scratch");
    double *sd = (double *)h->colmean.p;
    hipLaunchKernelGGL(k_gather_finish_sd, dim3((nn + 255) / 256), dim3(256), 0, h->stream, gathered, rows, nn,
                       world, scale, sd);
    hipLaunchKernelGGL(k_gather_finish, dim3((nn + 255) / 256, nn), dim3(256), 0, h->stream, gathered, rows, nn,
                       world, scale, (const double *)sd, C, ldc);
    PCG_HIP(h, hipGetLastError());
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}

// The native sharded K1 (comm.hip pcg_corr_sharded) on the CRT path, in three steps with no host
// sync: corr_shard_crt_prepare sizes every buffer the launches use (so the only local failure, an
// allocation, happens before any collective), corr_shard_crt_enqueue launches this rank's share —
// the column statistics, the residue planes of ONLY the moduli its unit run touches (units are
// modulus-major: at 8 ranks a rank forms ~1/8 of the 17 planes), its units of the GEMM — and
// corr_shard_crt_finish_enqueue rebuilds C from the all-gathered units. *crt = false: K1 takes the
// digit / fp64 path here and the caller uses pcg_corr_shard / pcg_corr_shard_finish instead.
int corr_shard_crt_prepare(pcg_handle *h, int64_t N, int64_t n, int world, bool *crt, int64_t *unit_bytes) {
    CrtPlan cp;
    *crt = crt_plan(h->tune, (int)n, N, cp);
    if (!*crt) return PCG_OK;
    const int nn = (int)n;
    const int nchunks = (int)((N + MEAN_ROWS - 1) / MEAN_ROWS);
    const size_t parts = (size_t)nn * nchunks * 3;
    if (!pcg_ensure(h, h->colmean, sizeof(double) * (parts + nn) + sizeof(int) * nn) ||
        !pcg_ensure(h, h->k1_digits, (size_t)cp.tab.k * cp.CBp * cp.TB * 2048) ||
        !pcg_ensure(h, h->pr_scratch, sizeof(double) * (size_t)(nn + 32)))
        return pcg_fail(h, PCG_ERR_OOM, "sharded K1 scratch (n %lld, N %lld)", (long long)n, (long long)N);
    *unit_bytes = (cp.units + world - 1) / world * (int64_t)CRT_UNIT;
    return PCG_OK;
}

int corr_shard_crt_enqueue(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, int rank, int world,
                           double *packed) {
    const int nn = (int)n;
    CrtPlan cp;
    if (!crt_plan(h->tune, nn, N, cp)) return pcg_fail(h, PCG_ERR_INVALID, "sharded K1: not the CRT path");
    double *mean;
    int *expo = nullptr;
    int rc = column_means(h, X, N, nn, ldx, &mean, &expo);
    if (rc) return rc;
    h->k1_stamp[0] = N;
    h->k1_stamp[1] = nn;
    h->k1_stamp[2] = cp.tab.k;
    h->k1_stamp[3] = ((int64_t)cp.tab.b << 32) | ((int64_t)cp.ks << 16) | cp.kb;
    h->k1_stamp_ok = true;
    const int64_t per = (cp.units + world - 1) / world, u0 = per * rank;
    const int64_t nu = std::max<int64_t>(std::min<int64_t>(per, cp.units - u0), 0);
    if (nu > 0) {
        const int64_t um = (int64_t)cp.ntiles * cp.ks;       // units per modulus
        const int m0 = (int)(u0 / um), m1 = (int)((u0 + nu - 1) / um) + 1;
        const int8_t *R = nullptr;
        rc = crt_residues(h, cp, X, N, nn, ldx, mean, expo, m0, m1, h->stream, &R);
        if (rc) return rc;
        crt_gemm(h, cp, R, u0, nu, (uint8_t *)packed);
    }
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

int corr_shard_crt_finish_enqueue(pcg_handle *h, const double *gathered, int64_t N, int64_t n, double *C,
                                  int64_t ldc) {
    const int nn = (int)n;
    CrtPlan cp;
    if (!crt_plan(h->tune, nn, N, cp) || !h->k1_stamp_ok)
        return pcg_fail(h, PCG_ERR_INVALID, "sharded K1 finish: no CRT-mode shard on this handle");
    crt_finish(h, cp, (const uint8_t *)gathered, colmean_expo(h, N, nn), nn, N, (double *)h->pr_scratch.p, C, ldc);
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

// K1 launched on the handle's stream without a host sync (the fused pcg_pc_skeleton path)
int pcg_corr_launch(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C, int64_t ldc) {
    if (!h || !X || !C || N < 2 || n < 1 || ldx < n || ldc < n || n > (1 << 24))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_corr: invalid arguments");
    PCG_HIP(h, hipSetDevice(h->device));
    const int nn = (int)n;
    const double scale = 1.0 / (double)(N - 1);
    CrtPlan cp;
    if (crt_plan(h->tune, nn, N, cp)) {
        double *mean;
        int *expo = nullptr;
        int rc = column_means(h, X, N, nn, ldx, &mean, &expo);
        if (rc) return rc;
        const size_t sbytes = sizeof(double) * (size_t)(nn + 32);
        if (!pcg_ensure(h, h->pr_scratch, sbytes + (size_t)cp.units * CRT_UNIT))
            return pcg_fail(h, PCG_ERR_OOM, "pcg_corr CRT scratch");
        double *sd = (double *)h->pr_scratch.p;
        uint8_t *Rs = (uint8_t *)h->pr_scratch.p + sbytes;
        // (round 4 measured the residue planes of modulus groups on the aux stream beside the GEMM:
        // slower — the co-resident residue blocks delay the GEMM's waves — and removed it in round 5)
        const int8_t *R = nullptr;
        rc = crt_residues(h, cp, X, N, nn, ldx, mean, expo, 0, cp.tab.k, h->stream, &R);
        if (rc) return rc;
        crt_gemm(h, cp, R, 0, cp.units, Rs);
        crt_finish(h, cp, Rs, expo, nn, N, sd, C, ldc);
        PCG_HIP(h, hipGetLastError());
        return PCG_OK;
    }
    const bool i8 = h->tune[PCG_TUNE_K1_I8] != 0;
    double *mean;
    int *expo = nullptr;
    int rc = column_means(h, X, N, nn, ldx, &mean, i8 ? &expo : nullptr);
    if (rc) return rc;
    const int T = (nn + TILE - 1) / TILE;
    const int ntiles = T * (T + 1) / 2;
    int64_t kchunk = 0;
    int kb = 0;
    const int ks = i8 ? split_k_i8(h->tune, nn, N, &kb) : split_k(nn, N, &kchunk);
    double *G = C;
    int64_t ldg = ldc, stride = 0;
    if (ks > 1) {
        stride = (int64_t)nn * nn;
        if (!pcg_ensure(h, h->pr_scratch, sizeof(double) * (size_t)stride * ks))
            return pcg_fail(h, PCG_ERR_OOM, "pcg_corr split-K slabs");
        G = (double *)h->pr_scratch.p;
        ldg = nn;
    }
    if (i8) {
        int CB = 0, TB = 0;
        const int8_t *Dg = nullptr;
        rc = k1_digits(h, X, N, nn, ldx, mean, expo, &CB, &TB, &Dg);
        if (rc) return rc;
        hipLaunchKernelGGL(k_xtx_i8, dim3(xtx_grid(ntiles * ks)), dim3(256), 0, h->stream, Dg, CB, TB, nn,
                           (const int *)expo, ntiles, ks, kb, G, ldg, stride, (const int32_t *)nullptr,
                           h->tune[PCG_TUNE_K1_SUPER_ORDER] != 0 ? 1 : 0);
    } else {
        hipLaunchKernelGGL(k_xtx, dim3(xtx_grid(ntiles * ks)), dim3(256), 0, h->stream, X, N, nn, ldx, mean, ntiles,
                           ks, kchunk, G, ldg, stride, (const int32_t *)nullptr);
    }
    const int T64 = (nn + NT - 1) / NT;
    hipLaunchKernelGGL(k_normalize_tiles, dim3(T64 * (T64 + 1) / 2), dim3(256), 0, h->stream, G, ldg, stride, ks, C,
                       ldc, nn, scale);
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

extern "C" int pcg_corr(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C,
                        int64_t ldc) {
    const int rc = pcg_corr_launch(h, X, N, n, ldx, C, ldc);
    if (rc) return rc;
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return PCG_OK;
}
