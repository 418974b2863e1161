// barrier.hip — the bit-packed level barrier of the edge-sharded skeleton (multi-GPU).
//
// Within a depth every rank evaluates an owner-disjoint slice of the work list and raises
// removal flags (n x n bytes, both triangles) for the pairs it found independent
// (SkeletonDiscovery.py:124-128; removals deferred to :141-144). The merge across ranks is a
// bitwise OR of those flags. RCCL has no OR, so instead of an all-reduce(MAX) of the n*n
// bytes (4 MB at n = 2000) every rank packs its upper triangle into bits and the ranks
// all-gather the packed words:
//
//   packed layout: row x keeps words w = x/64 .. W-1 of its 64-bit row mask (bits y > x only),
//   rows back to back (offs(x) = x*W - sum_{r<x} floor(r/64)), then ONE status word whose
//   bytes are the level status bytes that follow the flags (overflow, singular, domain) plus
//   byte 3 = "this rank failed locally" — so a rank whose begin / run failed still takes part
//   in the collective and every rank leaves the depth with the same verdict.
//
// n = 2000: 32 032 words + 1 = 256 KB per rank (vs 4 MB), all-gathered over xGMI.
// pcg_level_merge ORs the world copies and writes the symmetric byte flags back (64 x 64
// tiles, transposed through LDS so both triangle halves are written as coalesced rows).
#include <hip/hip_runtime.h>

#include "handle.h"

namespace {

__host__ __device__ inline int64_t packed_row_offset(int64_t x, int64_t W) {
    const int64_t q = x >> 6;
    return x * W - (64 * q * (q - 1) / 2 + (x - 64 * q) * q);
}

__host__ inline int64_t packed_words_of(int64_t n) {
    const int64_t W = (n + 63) / 64;
    return packed_row_offset(n, W) + 1;   // + the status word
}

// one wave per (x, w >= x/64): lane b reads rm[x][64w + b] (a coalesced 64-byte segment)
__global__ __launch_bounds__(256) void k_pack_flags(const uint8_t *rm, int n, int W, uint64_t *packed) {
    const int lane = threadIdx.x & 63;
    const int64_t word = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;   // wave-uniform
    if (word >= (int64_t)n * W) return;
    const int x = (int)(word / W), w = (int)(word % W);
    if (w < (x >> 6)) return;
    const int y = w * 64 + lane;
    const bool f = y > x && y < n && rm[(int64_t)x * n + y] != 0;
    const unsigned long long m = __ballot(f);
    if (lane == 0) packed[packed_row_offset(x, W) + (w - (x >> 6))] = m;
}

__global__ void k_pack_status(const uint8_t *status, int local_error, uint64_t *word) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t v = 0;
    for (int k = 0; k < 3; ++k) v |= (uint64_t)(status[k] != 0) << (8 * k);
    if (local_error) v |= 1ull << 24;
    *word = v;
}

// one block per 64 x 64 tile (bi <= bj) of the pair triangle
__global__ __launch_bounds__(256) void k_merge_flags(const uint64_t *gathered, int64_t P, int world, int n, int W,
                                                     uint8_t *rm) {
    __shared__ uint64_t rows[64];
    __shared__ uint8_t tr[64][65];
    int bi = 0, rem = blockIdx.x;
    while (rem >= W - bi) { rem -= W - bi; ++bi; }   // tile rows have W - bi tiles each
    const int bj = bi + rem;
    const int tid = threadIdx.x;
    if (tid < 64) {
        const int x = 64 * bi + tid;
        uint64_t v = 0;
        if (x < n) {
            const int64_t idx = packed_row_offset(x, W) + (bj - bi);
            for (int r = 0; r < world; ++r) v |= gathered[(int64_t)r * P + idx];
        }
        rows[tid] = v;
    }
    __syncthreads();
    // upper tile (bi, bj): row x = 64 bi + r, columns 64 bj + c; diagonal tile: min/max
    for (int e = tid; e < 64 * 64; e += blockDim.x) {
        const int r = e >> 6, c = e & 63;
        const int x = 64 * bi + r, y = 64 * bj + c;
        uint8_t b;
        if (bi != bj) b = (uint8_t)((rows[r] >> c) & 1ull);
        else b = c > r ? (uint8_t)((rows[r] >> c) & 1ull) : (c < r ? (uint8_t)((rows[c] >> r) & 1ull) : 0);
        if (x < n && y < n) rm[(int64_t)x * n + y] = b;
        tr[c][r] = b;
    }
    if (bi == bj) return;
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += blockDim.x) {
        const int r = e >> 6, c = e & 63;   // row 64 bj + r, column 64 bi + c
        const int x = 64 * bj + r, y = 64 * bi + c;
        if (x < n && y < n) rm[(int64_t)x * n + y] = tr[r][c];
    }
}

__global__ void k_merge_status(const uint64_t *gathered, int64_t P, int world, uint8_t *status) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t v = 0;
    for (int r = 0; r < world; ++r) v |= gathered[(int64_t)r * P + P - 1];
    for (int k = 0; k < 8; ++k) status[k] = (uint8_t)((v >> (8 * k)) & 0xff);
}

uint8_t *removal_flags(pcg_handle *h) { return h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p; }

}  // namespace

extern "C" int pcg_level_packed_words(int64_t n, int64_t *words) {
    if (n < 2 || !words) return PCG_ERR_INVALID;
    *words = packed_words_of(n);
    return PCG_OK;
}

extern "C" int pcg_level_pack(pcg_handle *h, uint64_t *packed_dev, int local_error) {
    if (!h || !packed_dev || h->n < 2) return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_pack: invalid arguments");
    const int n = (int)h->n, W = h->W;
    const int64_t P = packed_words_of(n);
    uint8_t *rm = removal_flags(h);
    if (local_error || h->depth < 0) {
        // this rank's flags may be stale or never written: contribute nothing but the verdict
        PCG_HIP(h, hipMemsetAsync(packed_dev, 0, sizeof(uint64_t) * (P - 1), h->stream));
    } else {
        const int64_t waves = (int64_t)n * W;
        hipLaunchKernelGGL(k_pack_flags, dim3((unsigned)((waves * 64 + 255) / 256)), dim3(256), 0, h->stream, rm, n,
                           W, packed_dev);
    }
    hipLaunchKernelGGL(k_pack_status, dim3(1), dim3(64), 0, h->stream, rm + (int64_t)n * n, local_error ? 1 : 0,
                       packed_dev + (P - 1));
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

extern "C" int pcg_level_merge(pcg_handle *h, const uint64_t *gathered_dev, int world) {
    if (!h || !gathered_dev || world < 1 || h->n < 2)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_merge: invalid arguments");
    const int n = (int)h->n, W = h->W;
    const int64_t P = packed_words_of(n);
    uint8_t *rm = removal_flags(h);
    const unsigned tiles = (unsigned)(W * (W + 1) / 2);
    hipLaunchKernelGGL(k_merge_flags, dim3(tiles), dim3(256), 0, h->stream, gathered_dev, P, world, n, W, rm);
    hipLaunchKernelGGL(k_merge_status, dim3(1), dim3(64), 0, h->stream, gathered_dev, P, world, rm + (int64_t)n * n);
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}
