// skeleton.hip — level-synchronous stable PC skeleton on MI355X (gfx950).
//
// Replaces causal-learn skeleton_discovery(stable=True) + FisherZ [U]; the loop it
// restates is lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:70-144 and the helpers
// lib/causallearn/graph/GraphClass.py:78-106 (cache key, neighbors, max_degree).
//
// Device layout (HBM, all handle-owned except C and removed_level):
//   C        n x n fp64 correlation (caller)           diag  n fp64 (C[i,i])
//   adj      n x W u64 adjacency bitmask (W = ceil(n/64)); the level barrier state
//   deg/off  n int32 degrees, n+1 int32 CSR offsets;   nbr   sum(deg) int32, ascending
//   rm       n x n uint8 removal flags of the current depth (merged across ranks)
//   ug       sum(deg) x W u64: per ordered adjacent pair (x -> y) the union of independent
//            S seen from x's side (global node bits) — SkeletonDiscovery.py:129-130,135-136
//   cpre     n+1 int64 chunk prefix: node x owns chunks [cpre[x], cpre[x+1])
//
// Work decomposition at depth d >= 1 ("x-side" order of the reference loop):
//   a chunk = (node x, bs consecutive colex ranks of d-subsets S of adj(x)); one lane = one S.
//   Each lane factors C_SS once (Cholesky in registers), u = L^-1 C_Sx, then sweeps every
//   y in adj(x) \ S: v = L^-1 C_Sy, c_xx = 1-u.u, c_yy = C_yy - v.v, c_xy = C_xy - u.v, and
//   r = c_xy / sqrt(c_xx c_yy) is the partial correlation (= -inv01/sqrt(inv00 inv11)).
//   The block stages row C[y, adj(x)] + adj(y) in LDS (double-buffered, register prefetch),
//   so every per-test operand comes from LDS; only the once-per-lane gathers hit L2/HBM.
//   Dedup = the reference's memo: (x, y, S) is skipped on x's side when y < x and S is a
//   subset of adj(y) — node y evaluates it and ORs the result into both sides' unions.
//
// Decision (default): p > alpha  <=>  r^2 < tanh(z_{1-a/2}/sqrt(N-d-3))^2; tests within a
// relative 1e-6 band of the threshold, with a failed Cholesky, |r| ~ 1, NaN, or any other
// edge case go to the exact path (LU like numpy.linalg.inv + the reference p expression).
// PCG_FLAG_FULL_P computes the p-value of every test inline instead.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <type_traits>

#include "fisherz_dev.h"
#include "handle.h"

namespace {

constexpr int MODE_DECIDE = 0;
#ifndef PCG_COND_TAU
#define PCG_COND_TAU 1e-4     // conditioning guard of the fast paths (see decide)
#endif
constexpr int MODE_FULLP = 1;
constexpr int MODE_EXACT = 2;
// candidates c per lane task in k_level_lds_t, per depth (measured, tools/variant_bench.sh):
// depth 2 groups of 6 (round 2: 0.314 -> 0.282 ms vs 8, which had been -28 % vs 4); depth 3 groups of 6 (fp32 sweep: 0.715 -> 0.688 ms vs 4; the fp64 form measured 4 ~ 6, 8 +15 %);
// depth 4 groups of 6 at 3 waves/SIMD (168 VGPRs): fp64 VALU from one wave issues at most every
// ~8 cycles with a ~50-cycle dependent latency (tools/micro/valu_occ.hip), so a third wave of 6
// chains beats two waves of 8 (4.03 vs 4.29 ms; groups of 4 at 3 waves 4.46 ms)
#ifndef PCG_TG2
#define PCG_TG2 6
#endif
#ifndef PCG_TG_WC
#define PCG_TG_WC 0   // T-group sweep: project candidates with w_c = C_TT^-1 M[T][c] (see k_level_lds_t)
#endif
#ifndef PCG_TG_Y2
#define PCG_TG_Y2 0   // T-group sweep: two y per iteration at the depths whose bit is set (1 << d)
#endif
#ifndef PCG_TG_SGPR
#define PCG_TG_SGPR 0x18 // T-group sweep, depths whose bit (1 << d) is set: per-y bookkeeping as wave
                         // lane masks (SALU) instead of per-lane bits
#endif
#ifndef PCG_TG_SGPR_WIDE
#define PCG_TG_SGPR_WIDE PCG_TG_SGPR   // the same for the wide (128-bit mask) class
#endif
#ifndef PCG_TG_SPLIT
#define PCG_TG_SPLIT 0   // lane-mask sweep: split the y range around a shared candidate window (spills: slower)
#endif
#ifndef PCG_TG3
#define PCG_TG3 6
#endif
#ifndef PCG_TG4
#define PCG_TG4 6
#endif
__host__ __device__ constexpr int tg_of_depth(int d) { return d == 2 ? PCG_TG2 : (d == 3 ? PCG_TG3 : PCG_TG4); }
static_assert((PCG_TG2 == 4 || PCG_TG2 == 6 || PCG_TG2 == 8) && (PCG_TG3 == 4 || PCG_TG3 == 6 || PCG_TG3 == 8) &&
                  (PCG_TG4 == 4 || PCG_TG4 == 6 || PCG_TG4 == 8),
              "k_level_lds_t candidate groups of 4, 6 or 8");

struct LevelArgs {
    const double *C;
    int64_t ldc;
    const double *diag;
    const uint64_t *adj;
    int W;
    int n;
    int d;
    int bs;                      // lanes (S ranks) per chunk
    const int32_t *deg;
    const int32_t *off;
    const int32_t *nbr;
    const int64_t *cpre;
    const uint64_t *binom;
    uint8_t *rm;
    uint64_t *ug;
    DevCounters *ctr;
    DeferredEntry *deferred;
    int64_t def_cap;
    ScreenEntry *screen;         // fp32 sweep -> fp64 screen list
    int64_t scr_cap;
    pcg_record *records;
    int64_t rec_cap;
    pcg_record *nearl;
    int64_t near_cap;
    double lo2, hi2;             // decision band on r^2
    double tau;                  // conditioning guard (see decide)
    double s_amgm, inv_s;        // fp32 screen: AM-GM scale ~ |c_xy| at the threshold (k_level_lds_f)
    double alpha, sqrt_dof;
    int dof_negative;
    int record;
    int64_t rec_mod, rec_res;    // record sample: canonical pair (a, b) with (a*n + b) % rec_mod == rec_res
    int64_t chunk_lo;            // first chunk of this launch (within its class)
    int spl;                     // S ranks per lane (LDS-resident kernel)
    int lds_btab_off;            // byte offset of the LDS binomial table (LDS-resident kernel)
    // depth 4's per-node compact blocks (k_node_blocks)
    const int64_t *bo;           // n + 1 offsets of the compact blocks (doubles)
    double *cblk;                // per node: C[adj(x) + x, adj(x) + x], stride D + 1, x last
    uint64_t *lmk;               // per node: local adjacency masks of adj(x), at off[x]
    int img;                     // cblk holds fp32 LDS images of k_level_lds_f (tgf_image_bytes each) instead
    // k_level_lds_f's dispatch order (a launch over the whole narrow class): block b runs the b-th
    // chunk of the nodes taken by degree, largest first (nord: nodes, nps: their chunk prefix), so
    // the level's last blocks are its shortest ones
    const int32_t *nord, *nps;
    int nm;
    int stamp_end;               // block 0 stamps ctr->t_run1 at entry (the kernel bracket's end)
};

// the kernel bracket's end (skeleton_once with PCG_KBRACKET = 0): one store by one thread
__device__ __forceinline__ void stamp_run_end(const LevelArgs &a) {
    if (a.stamp_end && blockIdx.x == 0 && threadIdx.x == 0) a.ctr->t_run1 = wall_clock64();
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// the wave's LDS slot of the one-wave-per-set kernels: the L rows of the current set (md x (md + 1)),
// reused by the exact path (m x m matrix, two solution columns, m variable ids; m <= md + 2)
constexpr int WAVE_SLOT_DOUBLES(int md) {
    return (md + 2) * (md + 2) + 3 * (md + 2) > md * (md + 1) ? (md + 2) * (md + 2) + 3 * (md + 2) : md * (md + 1);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// per-kernel test / independence counters: one atomic pair per BLOCK (wave sums staged in
// LDS). Per-wave atomics on the two counter words queue at the L2 when many blocks end together
// (measured: 40 us at depth 0, 0.35 ms for depth 1's 5 400 blocks). Every thread must call it.
__device__ __forceinline__ void block_flush_counts(DevCounters *ctr, unsigned long long tests,
                                                   unsigned long long indep) {
    __shared__ unsigned long long s_cnt[2][16];
    tests = wave_sum(tests);
    indep = wave_sum(indep);
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_cnt[0][w] = tests;
        s_cnt[1][w] = indep;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, i = 0;
        for (int k = 0; k < nw; ++k) {
            t += s_cnt[0][k];
            i += s_cnt[1][k];
        }
        if (t) atomicAdd(&ctr->tests, t);
        if (i) atomicAdd(&ctr->indep, i);
    }
}

__device__ __forceinline__ int find_in_sorted(const int32_t *a, int len, int v) {
    int lo = 0, hi = len - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// wave-aggregated like push_deferred: one counter atomic per call site and wave (the records of
// every test of a sampled pair arrive together from one wave's lanes)
__device__ __forceinline__ void push_record(pcg_record *buf, int64_t cap, unsigned long long *ctr,
                                            int a, int b, int d, const int *S, double p) {
    const unsigned long long act = __ballot(1);
    const int leader = __ffsll((long long)act) - 1;
    const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(act >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)act, 0u));
    unsigned long long base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(act));
    base = __shfl(base, leader);
    const unsigned long long slot = base + rank;
    if ((int64_t)slot < cap) {
        pcg_record &r = buf[slot];
        r.a = a; r.b = b; r.d = d;
        for (int i = 0; i < PCG_MAX_DEPTH; ++i) r.s[i] = i < d ? S[i] : -1;
        r.p = p;
    }
}

// PCG_FLAG_RECORD keeps every unique test, or the fixed pair sample of pcg_set_record_sample
__device__ __forceinline__ bool rec_on(const LevelArgs &a, int lo, int hi) {
    return a.record && (a.rec_mod <= 1 || ((int64_t)lo * a.n + hi) % a.rec_mod == a.rec_res);
}

// wave-aggregated: the lanes active at the call take consecutive slots from ONE counter atomic (the
// record routing puts every test of a sampled pair here — ~1e6 per config-5 run — and a returning
// atomic per entry on the one list counter serialises at its L2 channel)
__device__ __forceinline__ void push_deferred(const LevelArgs &a, int x, int y, const int *S, int d) {
    const unsigned long long act = __ballot(1);
    const int leader = __ffsll((long long)act) - 1;
    const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(act >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)act, 0u));
    unsigned long long base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&a.ctr->deferred, (unsigned long long)__popcll(act));
    base = __shfl(base, leader);
    const unsigned long long slot = base + rank;
    if ((int64_t)slot < a.def_cap) {
        DeferredEntry &e = a.deferred[slot];
        e.x = x; e.y = y;
        for (int i = 0; i < PCG_MAX_DEPTH; ++i) e.s[i] = i < d ? S[i] : -1;
    }
}

#ifndef PCG_SCREEN_ABL
#define PCG_SCREEN_ABL 0   // timing ablation only (wrong results): the fp32 sweep's screen pushes dropped
#endif
__device__ __forceinline__ void push_screen(const LevelArgs &a, int x, int y, const int *S, int d) {
    if (PCG_SCREEN_ABL) return;
    const unsigned long long slot = atomicAdd(&a.ctr->screened, 1ull);
    if ((int64_t)slot < a.scr_cap) {
        ScreenEntry &e = a.screen[slot];
        e.x = x; e.y = y;
        for (int i = 0; i < 4; ++i) e.s[i] = i < d ? S[i] : -1;
    }
}

// k_level_lds_f's screen list entries are staged in a per-block LDS buffer and appended to the
// global list with ONE counter atomic per block at its end: one returning atomic per entry on the
// single list counter serialised at its L2 channel (config 5 depth 3: 8.9e4 pushes, kernel 0.68 ms;
// 0.44 ms with the pushes dropped). A full buffer falls back to the per-entry push
#ifndef PCG_SCREEN_BUF
#define PCG_SCREEN_BUF 96
#endif
__device__ __forceinline__ void push_screen_blk(const LevelArgs &a, ScreenEntry *buf, unsigned *cnt, int x, int y,
                                                const int *S, int d) {
    const unsigned k = atomicAdd(cnt, 1u);
    if (k < (unsigned)PCG_SCREEN_BUF) {
        ScreenEntry &e = buf[k];
        e.x = x; e.y = y;
        for (int i = 0; i < 4; ++i) e.s[i] = i < d ? S[i] : -1;
    } else {
        push_screen(a, x, y, S, d);
    }
}
// the block's buffered entries to the global list (every thread calls it after a block barrier)
__device__ __forceinline__ void flush_screen_blk(const LevelArgs &a, const ScreenEntry *buf, const unsigned *cnt,
                                                 unsigned long long *base) {
    const unsigned nbuf = min(*cnt, (unsigned)PCG_SCREEN_BUF);
    if (!nbuf) return;                                  // (block-uniform)
    if (threadIdx.x == 0) *base = atomicAdd(&a.ctr->screened, (unsigned long long)nbuf);
    __syncthreads();
    const unsigned long long b0 = *base;
    for (unsigned i = threadIdx.x; i < nbuf; i += blockDim.x)
        if ((int64_t)(b0 + i) < a.scr_cap) a.screen[b0 + i] = buf[i];
}

// error bits (1 singular, 2 domain) into the level counters and into the status bytes that
// follow the n*n removal flags, so a multi-GPU merge spreads them to every rank
__device__ __forceinline__ void flag_error(const LevelArgs &a, int err) {
    atomicOr(&a.ctr->error, (unsigned long long)err);
    uint8_t *status = a.rm + (int64_t)a.n * a.n;
    if (err & 1) status[1] = 1;
    if (err & 2) status[2] = 1;
}

// (group, t0) pairs of k_level_lds_t for a node of degree D at depth DM: t0 in
// [g*TG + 1, D - DM + 1] for every group g with g*TG <= D - DM
__host__ __device__ inline int tg_pairs(int D, int DM) {
    int s = 0;
    for (int cb = 0; cb <= D - DM; cb += tg_of_depth(DM)) {
        const int m = D - (DM - 1) - cb;
        if (m > 0) s += m;
    }
    return s;
}

// 0 dependent, 1 independent, 2 exact path. p written in FULL_P mode.
// Conditioning guard: the Cholesky-based partial correlation is trusted only when
//   g * min(c_xx, c_yy) * (1 - r^2) >= tau,   g = the smallest pivot^2 of C_SS,
// i.e. c_xx c_yy - c_xy^2 > kg with kg = tau / g (correlation diagonals are 1). Below it
// (near-collinear S, x or y given S nearly determined, |r| ~ 1) the test goes to the exact LU
// path, so decisions never rest on a cancellation-dominated r^2: with tau = 1e-4 the
// backward-error bound of the factorisation keeps r^2 within ~1e-8 relative of the LU value,
// far inside the +-1e-6 band (a test with near-duplicate columns pins this).
template <int MODE>
__device__ __forceinline__ int decide(const LevelArgs &a, double cxy, double cxx, double cyy, double kg,
                                      double *p) {
    if (MODE == MODE_EXACT) return 2;
    const double den = cxx * cyy;
    if (!(den > 0.0)) return 2;
    const double num = cxy * cxy;
    if (!(den - num > kg)) return 2;
    if (MODE == MODE_DECIDE) {
        if (num < a.lo2 * den) return 1;
        if (num > a.hi2 * den) return 0;
        return 2;
    } else {
        const double r = cxy / sqrt(den);
        int err = 0;
        const double pv = pcg_pvalue_from_r(r, a.sqrt_dof, &err);
        if (err) return 2;
        *p = pv;
        return pv > a.alpha ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------------------
// utility kernels
// byte fill by a grid-stride loop: unaligned head and tail bytewise, the body in 16-byte stores
__device__ __forceinline__ void fill_bytes(uint8_t *p, int64_t bytes, uint8_t v, int64_t tid, int64_t nth) {
    const int64_t head = std::min<int64_t>(bytes, (int64_t)((16 - ((uintptr_t)p & 15)) & 15));
    const int64_t body = (bytes - head) / 16;
    if (tid < head) p[tid] = v;
    uint4 *q = reinterpret_cast<uint4 *>(p + head);
    const unsigned w = 0x01010101u * v;
    for (int64_t i = tid; i < body; i += nth) q[i] = make_uint4(w, w, w, w);
    const int64_t t0 = head + body * 16;
    if (tid < bytes - t0) p[t0 + tid] = v;
}

// the skeleton's initial state in one launch: complete-graph adjacency bits, diag(C), degrees
// n - 1, removed_level = -1, removal flags + status bytes = 0, export row counter = 0
// rm |= banned off the diagonal (n x n bytes), grid-stride
__global__ __launch_bounds__(256) void k_or_flags(const uint8_t *banned, int64_t n, uint8_t *rm) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * n; i += (int64_t)gridDim.x * blockDim.x)
        if (banned[i] && i / n != i % n) rm[i] = 1;
}

__global__ __launch_bounds__(256) void k_init(uint64_t *adj, int n, int W, const double *C, int64_t ldc, double *diag,
                                              int32_t *deg, int8_t *rl, uint8_t *rm, int64_t rm_bytes,
                                              unsigned long long *exp_ctr) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nth = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = tid; i < (int64_t)n * W; i += nth) {
        const int x = (int)(i / W), w = (int)(i % W);
        const int base = w * 64;
        const int rem = n - base;
        uint64_t m = rem >= 64 ? ~0ull : ((1ull << rem) - 1ull);
        if (x >= base && x < base + 64) m &= ~(1ull << (x - base));
        adj[i] = m;
    }
    for (int64_t i = tid; i < n; i += nth) {
        diag[i] = C[i * ldc + i];
        deg[i] = n - 1;
    }
    fill_bytes(reinterpret_cast<uint8_t *>(rl), (int64_t)n * n, 0xFF, tid, nth);
    fill_bytes(rm, rm_bytes, 0, tid, nth);
    if (tid == 0) *exp_ctr = 0;
}

constexpr int EXPORT_GROUP = 8;     // union rows in flight per wave in the sepset export

// sepset export helpers: lane k of a wave owns CSR slot slot0 + k of node x; rows of removed
// slots are read with all 64 lanes, eight rows' loads in flight
// pass 1: the mask of the wave's removed slots whose W-word union row is non-empty
__device__ __forceinline__ unsigned long long export_keep(int64_t slot0, bool removed, const uint64_t *ug, int W) {
    const int lane = threadIdx.x & 63;
    unsigned long long keepm = 0;
    for (unsigned long long mm = __ballot(removed); mm;) {
        int ks[EXPORT_GROUP];
        int cnt = 0;
#pragma unroll
        for (int g = 0; g < EXPORT_GROUP; ++g) {
            ks[g] = mm ? __ffsll((long long)mm) - 1 : 0;
            if (mm) { mm &= mm - 1; ++cnt; }
        }
        uint64_t v[EXPORT_GROUP];
#pragma unroll
        for (int g = 0; g < EXPORT_GROUP; ++g) v[g] = 0ull;
        for (int w = lane; w < W; w += 64)
#pragma unroll
            for (int g = 0; g < EXPORT_GROUP; ++g)
                if (g < cnt) v[g] |= ug[(slot0 + ks[g]) * W + w];
#pragma unroll
        for (int g = 0; g < EXPORT_GROUP; ++g)
            if (g < cnt && __ballot(v[g] != 0ull)) keepm |= 1ull << ks[g];
    }
    return keepm;
}

// pass 2: copy the kept rows (already L2-resident from pass 1) to rows base, base + 1, ...
__device__ __forceinline__ void export_copy(int64_t slot0, unsigned long long keepm, int64_t base, int x, int y,
                                            const uint64_t *ug, int W, int32_t *xy, uint64_t *bits, int64_t cap) {
    const int lane = threadIdx.x & 63;
    if ((keepm >> lane) & 1ull) {      // the lane owning the slot writes its (x, y)
        const int64_t r = base + __popcll(keepm & ((1ull << lane) - 1ull));
        if (r < cap) {
            xy[2 * r] = x;
            xy[2 * r + 1] = y;
        }
    }
    for (unsigned long long mm = keepm; mm;) {
        int ks[EXPORT_GROUP];
        int cnt = 0;
#pragma unroll
        for (int g = 0; g < EXPORT_GROUP; ++g) {
            ks[g] = mm ? __ffsll((long long)mm) - 1 : 0;
            if (mm) { mm &= mm - 1; ++cnt; }
        }
        for (int w = lane; w < W; w += 64) {
            uint64_t v[EXPORT_GROUP];
#pragma unroll
            for (int g = 0; g < EXPORT_GROUP; ++g) v[g] = g < cnt ? ug[(slot0 + ks[g]) * W + w] : 0ull;
#pragma unroll
            for (int g = 0; g < EXPORT_GROUP; ++g) {
                if (g >= cnt) break;
                const int64_t r = base + __popcll(keepm & ((1ull << ks[g]) - 1ull));
                if (r < cap) bits[r * W + w] = v[g];
            }
        }
    }
}

// The sepset export of depth d, off the level loop's critical path (export stream, double-
// buffered CSR and union rows): one lane per CSR slot (x, y) of depth d's graph finds x, keeps
// the slot if the pair was removed at this depth (removed_level == d) and its union row is
// non-empty, and the wave appends its kept rows with one atomic on a counter that persists
// across depths (rows are read with all 64 lanes, eight in flight).
__global__ __launch_bounds__(256) void k_export(const int32_t *off, const int32_t *nbr, const int8_t *rl, int d,
                                                const uint64_t *ug, int n, int W, int64_t sumdeg, int32_t *xy,
                                                uint64_t *bits, int64_t cap, unsigned long long *ctr) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
    const int64_t slot = wave_base + lane;
    int x = -1, y = -1;
    bool removed = false;
    if (slot < sumdeg && slot < off[n]) {
        int lo = 0, hi = n;  // off[lo] <= slot < off[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (off[mid] <= slot) lo = mid; else hi = mid;
        }
        x = lo;
        y = nbr[slot];
        removed = rl[(int64_t)x * n + y] == (int8_t)d;
    }
    const unsigned long long keepm = export_keep(wave_base, removed, ug, W);
    if (!keepm) return;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(ctr, (unsigned long long)__popcll(keepm));
    base = __shfl(base, 0);
    export_copy(wave_base, keepm, (int64_t)base, x, y, ug, W, xy, bits, cap);
}

// The level barrier (SkeletonDiscovery.py:141-144), one 256-thread block per row x: rm row x ->
// adjacency words (a wave's ballot is the mask cleared from word (x, w)) + removed_level, deg[x]
// lowered by the row's removed count; rm is the last read here, so set bytes are cleared for the
// next depth.
__device__ __forceinline__ void close_rows(uint8_t *rm, uint64_t *adj, int32_t *deg, int8_t *rl, int n, int W, int d,
                                           int blk, int nblk, int *cleared) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int x = blk; x < n; x += nblk) {
        int mine = 0;
        for (int w = wave; w < W; w += 4) {
            const int y = w * 64 + lane;
            bool removed = false;
            if (y < n) {
                removed = rm[(int64_t)x * n + y] != 0;
                if (removed) {
                    rl[(int64_t)x * n + y] = (int8_t)d;
                    rm[(int64_t)x * n + y] = 0;
                }
            }
            const unsigned long long m = __ballot(removed);
            if (lane == 0 && m) {
                const uint64_t old = adj[(int64_t)x * W + w];
                adj[(int64_t)x * W + w] = old & ~m;
                mine += __popcll(old & m);
            }
        }
        if (lane == 0) cleared[wave] = mine;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int c = cleared[0] + cleared[1] + cleared[2] + cleared[3];
            if (c) deg[x] -= c;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_level_close(uint8_t *rm, uint64_t *adj, int32_t *deg, int8_t *rl, int n,
                                                     int W, int d) {
    __shared__ int cleared[4];
    close_rows(rm, adj, deg, rl, n, W, d, blockIdx.x, gridDim.x, cleared);
}

// The level barrier's summary and the next depth's CSR in one launch. Blocks 0 .. nfill-1
// (nfill = ceil(n/4); 0 at init: depth 0 reads no CSR):
// one wave per node x builds its ascending neighbour list from the adjacency row at offset
// sum(deg[0..x)) (each wave sums the prefix itself, so no grid-wide scan is waited for) and, with
// ug, clears the node's union rows when they lie inside the buffer's ug_rows rows (the last block
// reports whether all of them did, so the next depth skips its memset). The last block: the CSR offsets (exclusive scan of deg), the
// degrees, level counters and merged status bytes written into host-mapped memory, then — after
// a system-scope fence — the sequence number the host spins on (the host then enqueues work that
// the stream orders after the whole grid). Counters and status bytes are cleared once copied.
// the CSR part: node groups g = blk, blk + nblk, ... of 4 nodes (a wave per node)
__device__ __forceinline__ void summary_nodes(const int32_t *deg, int n, int W, const uint64_t *adj, int32_t *nbr,
                                              uint64_t *ug, int64_t ug_rows, int nfill, int blk, int nblk) {
    const int lane = threadIdx.x & 63;
    for (int g = blk; g < nfill; g += nblk) {
        const int x = g * 4 + (threadIdx.x >> 6);
        if (x >= n) continue;
        int ps = 0;
        for (int i = lane; i < x; i += 64) ps += deg[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ps += __shfl_xor(ps, o);
        int base = ps;
        const int dx = *(const volatile int32_t *)&deg[x];
        if (ug && (int64_t)base + dx <= ug_rows) {
            const int64_t lo = (int64_t)base * W, hi = (int64_t)(base + dx) * W;
            for (int64_t e = lo + lane; e < hi; e += 64) ug[e] = 0ull;
        }
        for (int w0 = 0; w0 < W; w0 += 64) {
            const int w = w0 + lane;
            uint64_t v = w < W ? adj[(int64_t)x * W + w] : 0ull;
            const int c = __popcll(v);
            int incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            const int tot = __shfl(incl, 63);
            int pos = base + incl - c;
            while (v) {
                const int b = __ffsll((long long)v) - 1;
                nbr[pos++] = w * 64 + b;
                v &= v - 1;
            }
            base += tot;
        }
    }
}

// the summary part (one block): CSR offsets, degrees, counters, status bytes -> host-mapped
// memory, then the sequence number
__device__ __forceinline__ void summary_block(const int32_t *deg, int n, int32_t *off, const uint64_t *ug,
                                              int64_t ug_rows, DevCounters *ctr, uint8_t *status, LevelSummary *out,
                                              int32_t *out_deg, unsigned long long seq, int nfill, int32_t *part) {
    const int tid = threadIdx.x;
    const int per = (n + 255) / 256;
    const int lo = min(n, tid * per), hi = min(n, lo + per);
    int32_t sum = 0;
    for (int i = lo; i < hi; ++i) {
        const int32_t v = deg[i];
        out_deg[i] = v;
        sum += v;
    }
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {        // inclusive Hillis-Steele scan of the chunk sums
        const int32_t v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int32_t acc = tid ? part[tid - 1] : 0;
    for (int i = lo; i < hi; ++i) { off[i] = acc; acc += deg[i]; }
    if (tid == 255) off[n] = part[255];
    if (tid == 0) {
        volatile unsigned long long *cw = reinterpret_cast<volatile unsigned long long *>(ctr);
        unsigned long long *ow = reinterpret_cast<unsigned long long *>(&out->ctr);
        constexpr int NW = (int)(sizeof(DevCounters) / sizeof(unsigned long long));
        const int near_w = (int)(offsetof(DevCounters, near_alpha) / sizeof(unsigned long long));
        for (int k = 0; k < NW; ++k) {
            ow[k] = cw[k];
            if (k != near_w) cw[k] = 0ull;    // the near-alpha list accumulates over the run
        }
        const volatile uint8_t *sv = status;
        for (int k = 0; k < 8; ++k) out->status[k] = status ? sv[k] : 0;
        out->ug_clean = ug != nullptr && nfill > 0 && (int64_t)part[255] <= ug_rows;
        if (status)
            for (int k = 0; k < PCG_RM_STATUS; ++k) status[k] = 0;
        out->stamp = wall_clock64();
    }
    __threadfence_system();
    __syncthreads();
    if (tid == 0) {
        __threadfence_system();
        __atomic_store_n(&out->seq, seq, __ATOMIC_RELEASE);
    }
}

__global__ __launch_bounds__(256) void k_summary_fill(const int32_t *deg, int n, int W, const uint64_t *adj,
                                                      int32_t *off, int32_t *nbr, uint64_t *ug, int64_t ug_rows,
                                                      DevCounters *ctr, uint8_t *status, LevelSummary *out,
                                                      int32_t *out_deg, unsigned long long seq, int nfill) {
    if ((int)blockIdx.x < nfill) {
        summary_nodes(deg, n, W, adj, nbr, ug, ug_rows, nfill, blockIdx.x, nfill);
        return;
    }
    __shared__ int32_t part[256];
    summary_block(deg, n, off, ug, ug_rows, ctr, status, out, out_deg, seq, nfill, part);
}

// The node owning a chunk: the last x < n with cpre[x] <= chunk (the caller checked chunk <
// cpre[n]). A wave samples 64 prefix entries per round and narrows to the ballot's last hit, so
// n = 2000 takes two dependent loads instead of a binary search's eleven (each an L2 round trip at
// the start of every block). Every lane of the wave must be active; the result is wave-uniform.
__device__ __forceinline__ int chunk_node(const int64_t *cpre, int n, int64_t chunk) {
    const int lane = threadIdx.x & 63;
    int lo = 0, hi = n;                                   // cpre[lo] <= chunk < cpre[hi]
    while (hi - lo > 1) {
        const int step = (hi - lo + 63) >> 6;
        const int idx = lo + lane * step;
        const bool le = idx < hi && cpre[idx] <= chunk;   // a prefix of the lanes (cpre ascends)
        const unsigned long long b = __ballot(le);        // lane 0 always set
        const int j = 63 - __builtin_clzll(b);
        lo += j * step;
        hi = min(hi, lo + step);
    }
    return lo;
}

// chunk_node over an int32 prefix (LevelArgs::nps)
__device__ __forceinline__ int chunk_node32(const int32_t *pre, int n, int v) {
    const int lane = threadIdx.x & 63;
    int lo = 0, hi = n;                                   // pre[lo] <= v < pre[hi]
    while (hi - lo > 1) {
        const int step = (hi - lo + 63) >> 6;
        const int idx = lo + lane * step;
        const bool le = idx < hi && pre[idx] <= v;
        const unsigned long long b = __ballot(le);
        const int j = 63 - __builtin_clzll(b);
        lo += j * step;
        hi = min(hi, lo + step);
    }
    return lo;
}

// Local adjacency masks of a narrow node (D <= 64): row t's bit k = adj(nxs[t], nxs[k]); a wave
// takes four rows at a time with their four loads in flight before the ballots (the one-row loop
// waited out one L2 round trip per row)
__device__ __forceinline__ void stage_lmask(const LevelArgs &a, const int32_t *nxs, int D, unsigned long long *lmask) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int kg = lane < D ? nxs[lane] : 0;
    for (int t0 = wv; t0 < D; t0 += 4 * nwv) {
        uint64_t w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = t0 + r * nwv;
            w[r] = (t < D && lane < D) ? a.adj[(int64_t)nxs[t] * a.W + (kg >> 6)] : 0ull;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = t0 + r * nwv;
            if (t >= D) break;                // wave-uniform
            const unsigned long long m = __ballot(lane < D && ((w[r] >> (kg & 63)) & 1ull));
            if (lane == 0) lmask[t] = m;
        }
    }
}

// ---------------------------------------------------------------------------------------
// depth 0: one chunk = one 64 x 64 tile (bi <= bj) of the pair triangle; node bi*64 owns the
// chunks of tile row bi. Decisions are staged in LDS so both rm[x][y] and its mirror
// rm[y][x] are written as coalesced 64-byte row segments (every removal byte of the tile
// pair is written, 0 or 1, by exactly this block).
template <int MODE>
__global__ __launch_bounds__(256) void k_level0(LevelArgs a) {
    __shared__ uint8_t flag[64][68];
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int bi = lo >> 6;
    const int bj = bi + (int)(chunk - a.cpre[lo]);
    const int x0 = bi * 64, y0 = bj * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int S0[1] = {0};
    unsigned long long tests = 0, indep = 0;
    const int y = y0 + tx;
    const double cyy = y < a.n ? a.diag[y] : 0.0;
    // the thread's 16 entries (and their rows' diagonals) are all loaded before the first test:
    // one memory latency per thread, not four
    double cv[16], dv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int x = x0 + ty + 4 * i;
        const bool in = x < a.n && y < a.n && y > x;
        cv[i] = in ? a.C[(int64_t)x * a.ldc + y] : 0.0;
        dv[i] = in ? a.diag[x] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = ty + 4 * i;
        const int x = x0 + r;
        uint8_t f = 0;
        if (x < a.n && y < a.n && y > x) {
            const double cxy = cv[i];
            double p = 0.0;
            const int dec = decide<MODE>(a, cxy, dv[i], cyy, a.tau, &p);
            ++tests;
            if (dec == 2) {
                push_deferred(a, x, y, S0, 0);
            } else {
                if (MODE == MODE_FULLP) {
                    if (rec_on(a, x, y)) push_record(a.records, a.rec_cap, &a.ctr->records, x, y, 0, S0, p);
                    if (fabs(p - a.alpha) < 1e-9) push_record(a.nearl, a.near_cap, &a.ctr->near_alpha, x, y, 0, S0, p);
                }
                if (dec == 1) { f = 1; ++indep; }
            }
        }
        flag[r][tx] = f;
    }
    __syncthreads();
    // rows x of the tile: rm[x][y0 + tx]; mirrored rows y: rm[y][x0 + tx] = flag[tx][y - y0]
#pragma unroll 4
    for (int r = ty; r < 64; r += 4) {
        const int x = x0 + r, yy = y0 + tx;
        if (x < a.n && yy < a.n && yy > x) a.rm[(int64_t)x * a.n + yy] = flag[r][tx];
        const int ym = y0 + r, xm = x0 + tx;
        if (ym < a.n && xm < a.n && ym > xm) a.rm[(int64_t)ym * a.n + xm] = flag[tx][r];
    }
    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// depth d >= 1. DM = compile-time upper bound of d (exact for DM <= 4).
template <int DM, int MODE>
__global__ __launch_bounds__(256) void k_level(LevelArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int bs = blockDim.x;
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)

    // node owning this chunk
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int x = lo;
    const int D = a.deg[x];
    const int d = DM <= 4 ? DM : a.d;
    const int W = a.W;
    const int E = D + W + 2;                      // staged u64 per y: row, adj(y), Cxy, Cyy
    const int32_t *nxg = a.nbr + a.off[x];

    // LDS carve: nxs[D] int32 (padded to 8B) | sbuf[2][E] u64 | scratch[nwaves][2][W] u64
    int32_t *nxs = reinterpret_cast<int32_t *>(smem);
    uint64_t *sbuf = reinterpret_cast<uint64_t *>(smem + (((size_t)D * 4 + 15) & ~(size_t)15));
    uint64_t *scr = sbuf + 2 * (size_t)E;
    uint64_t *sc_self = scr + (size_t)wave * 2 * W;
    uint64_t *sc_prop = sc_self + W;

    for (int i = tid; i < D; i += bs) nxs[i] = nxg[i];
    for (int i = lane; i < 2 * W; i += 64) sc_self[i] = 0;

    const uint64_t nS = pcg_binom(a.binom, D, d);
    const uint64_t rank = (uint64_t)(chunk - a.cpre[x]) * (uint64_t)bs + (uint64_t)tid;
    const bool active = rank < nS;

    int k[DM];      // local indices of S in adj(x), ascending
    int sg[DM];     // global ids
#pragma unroll
    for (int i = 0; i < DM; ++i) { k[i] = -1; sg[i] = 0; }
    if (active) pcg_unrank_colex<DM>(rank, d, D, a.binom, k);
    __syncthreads();  // nxs ready
#pragma unroll
    for (int i = 0; i < DM; ++i)
        if (i < d && active) sg[i] = nxs[k[i]];

    // Cholesky of C_SS (lower, packed by row), u = L^-1 C_Sx, c_xx = C_xx - u.u
    double L[DM][DM];
    double rinv[DM];
    double u[DM];
    bool chol_ok = active;
    double cxx = 0.0;
    double gmin = 1.0;   // smallest pivot^2 of C_SS (conditioning guard, see decide)
    if (active) {
#pragma unroll
        for (int j = 0; j < DM; ++j) {
            if (j < d) {
                const double *Cj = a.C + (int64_t)sg[j] * a.ldc;
                double s = a.diag[sg[j]];
#pragma unroll
                for (int q = 0; q < DM; ++q)
                    if (q < j) s -= L[j][q] * L[j][q];
                chol_ok = chol_ok && (s > 0.0);
                gmin = fmin(gmin, s);
                const double ljj = sqrt(s);
                rinv[j] = 1.0 / ljj;
                L[j][j] = ljj;
#pragma unroll
                for (int i = 0; i < DM; ++i) {
                    if (i > j && i < d) {
                        double t = Cj[sg[i]];
#pragma unroll
                        for (int q = 0; q < DM; ++q)
                            if (q < j) t -= L[i][q] * L[j][q];
                        L[i][j] = t * rinv[j];
                    }
                }
            }
        }
        const double *Cx = a.C + (int64_t)x * a.ldc;
        double uu = 0.0;
#pragma unroll
        for (int i = 0; i < DM; ++i) {
            if (i < d) {
                double t = Cx[sg[i]];
#pragma unroll
                for (int q = 0; q < DM; ++q)
                    if (q < i) t -= L[i][q] * u[q];
                u[i] = t * rinv[i];
                uu += u[i] * u[i];
            }
        }
        cxx = a.diag[x] - uu;
        chol_ok = chol_ok && (cxx == cxx);
    }
    const double kg = a.tau / gmin;

    unsigned long long tests = 0, indep = 0;
    const int nstage = (E + bs - 1) / bs;          // staged elements per thread
    constexpr int PF = 8;                          // held in registers (rest: direct)

    auto stage_val = [&](int e, int yg) -> uint64_t {
        if (e < D) return (uint64_t)__double_as_longlong(a.C[(int64_t)yg * a.ldc + nxs[e]]);
        e -= D;
        if (e < W) return a.adj[(int64_t)yg * W + e];
        e -= W;
        if (e == 0) return (uint64_t)__double_as_longlong(a.C[(int64_t)x * a.ldc + yg]);
        return (uint64_t)__double_as_longlong(a.diag[yg]);
    };

    // prologue: stage y = nxs[0] into buffer 0
    if (D > 0) {
        const int yg0 = nxs[0];
        for (int e = tid; e < E; e += bs) sbuf[e] = stage_val(e, yg0);
    }
    __syncthreads();

    for (int t = 0; t < D; ++t) {
        const uint64_t *cur = sbuf + (size_t)(t & 1) * E;
        uint64_t *nxt = sbuf + (size_t)((t + 1) & 1) * E;
        const bool more = t + 1 < D;
        const int ygn = more ? nxs[t + 1] : 0;
        uint64_t pf[PF];
        if (more) {
#pragma unroll
            for (int j = 0; j < PF; ++j) {
                const int e = tid + j * bs;
                if (j < nstage && e < E) pf[j] = stage_val(e, ygn);
            }
        }
        const int yg = nxs[t];
        bool is_indep = false, prop = false;
        if (active) {
            bool skip = !active;
#pragma unroll
            for (int i = 0; i < DM; ++i)
                if (i < d) skip = skip || (k[i] == t);
            bool in_y = true;
            if (!skip) {
#pragma unroll
                for (int i = 0; i < DM; ++i)
                    if (i < d) in_y = in_y && ((cur[D + (sg[i] >> 6)] >> (sg[i] & 63)) & 1ull);
                if (yg < x && in_y) skip = true;     // owned by node y (memo)
            }
            if (!skip) {
                ++tests;
                int dec = 2;
                double p = 0.0;
                if (chol_ok) {
                    double vv = 0.0, uv = 0.0, v[DM];
#pragma unroll
                    for (int i = 0; i < DM; ++i) {
                        if (i < d) {
                            double tt = __longlong_as_double((long long)cur[k[i]]);
#pragma unroll
                            for (int q = 0; q < DM; ++q)
                                if (q < i) tt -= L[i][q] * v[q];
                            v[i] = tt * rinv[i];
                            vv += v[i] * v[i];
                            uv += u[i] * v[i];
                        }
                    }
                    const double cxy = __longlong_as_double((long long)cur[D + W]) - uv;
                    const double cyy = __longlong_as_double((long long)cur[D + W + 1]) - vv;
                    dec = decide<MODE>(a, cxy, cxx, cyy, kg, &p);
                }
                if (dec == 2) {
                    push_deferred(a, x, yg, sg, d);
                } else {
                    if (MODE == MODE_FULLP) {
                        const int lo_ = x < yg ? x : yg, hi_ = x < yg ? yg : x;
                        if (rec_on(a, lo_, hi_)) push_record(a.records, a.rec_cap, &a.ctr->records, lo_, hi_, d, sg, p);
                        if (fabs(p - a.alpha) < 1e-9)
                            push_record(a.nearl, a.near_cap, &a.ctr->near_alpha, lo_, hi_, d, sg, p);
                    }
                    if (dec == 1) {
                        is_indep = true;
                        prop = in_y && (yg > x);
                        ++indep;
                    }
                }
            }
        }
        // sepset unions + removal flags (wave-uniform branch)
        const unsigned long long bal = __ballot(is_indep);
        if (bal) {
            if (lane == __ffsll((long long)bal) - 1) {
                a.rm[(int64_t)x * a.n + yg] = 1;
                a.rm[(int64_t)yg * a.n + x] = 1;
            }
            if (is_indep) {
#pragma unroll
                for (int i = 0; i < DM; ++i)
                    if (i < d) {
                        atomicOr(&sc_self[sg[i] >> 6], 1ull << (sg[i] & 63));
                        if (prop) atomicOr(&sc_prop[sg[i] >> 6], 1ull << (sg[i] & 63));
                    }
            }
            const unsigned long long balp = __ballot(prop);
            wave_sync();
            uint64_t *row = a.ug + ((int64_t)a.off[x] + t) * W;
            for (int w = lane; w < W; w += 64) {
                const uint64_t vsw = sc_self[w];
                if (vsw) { atomicOr(reinterpret_cast<unsigned long long *>(&row[w]), vsw); sc_self[w] = 0; }
            }
            if (balp) {
                const int slot = a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x);
                uint64_t *rowy = a.ug + (int64_t)slot * W;
                for (int w = lane; w < W; w += 64) {
                    const uint64_t vpw = sc_prop[w];
                    if (vpw) { atomicOr(reinterpret_cast<unsigned long long *>(&rowy[w]), vpw); sc_prop[w] = 0; }
                }
            }
            wave_sync();
        }
        if (more) {
#pragma unroll
            for (int j = 0; j < PF; ++j) {
                const int e = tid + j * bs;
                if (j < nstage && e < E) nxt[e] = pf[j];
            }
            for (int e = tid + PF * bs; e < E; e += bs) nxt[e] = stage_val(e, ygn);
        }
        __syncthreads();
    }

    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// depth 1, nodes with 64 < D <= L1_MAXD neighbours, threshold decision. Both tests of a
// neighbour pair {y, z} of x — (x, y | z) and (x, z | y) — read the same C[y][z] and the same
// adjacency bit (adj is symmetric), so a lane takes one unordered pair and evaluates both:
// half the scattered gathers of the per-test form, no barrier in the sweep. The node's
// per-neighbour terms (C_xk, C_kk, 1/sqrt(C_kk), u_k = C_xk/sqrt(C_kk), c_xx|k, ok_k) are
// staged in LDS once per block. Same arithmetic and decision as k_level<1, MODE_DECIDE>:
// for (x, y | z): v = C_yz / sqrt(C_zz), c_xy = C_xy - u_z v, c_yy = C_yy - v^2.
// A chunk is (x, a contiguous share of the D(D-1)/2 pairs, row-major over y < z).
constexpr int L1_MAXD = 1024;
#ifndef PCG_L1_ABL
#define PCG_L1_ABL 0      // timing ablation only (wrong results): k_level1_pairs without its independence writes
#endif
constexpr int L1_PB = 4;              // pairs in flight per lane (independent gathers; 8 and 16 measured slower)
size_t l1_lds_bytes(int D) { return (size_t)D * (4 + 5 * 8) + 16; }
// I32: every index of C, adj and rm fits 31 bits (n * ldc < 2^31): 32-bit offsets instead of
// 64-bit multiplies in the hot loop (the pair arithmetic is 32-bit always: D <= L1_MAXD)
template <bool I32>
__global__ __launch_bounds__(256) void k_level1_pairs(LevelArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int x = lo;
    const int D = a.deg[x];
    const int W = a.W;
    // per-neighbour terms, sized by this node's degree (the launch reserves the largest)
    double *s_cx = reinterpret_cast<double *>(smem);
    double *s_d = s_cx + D, *s_ri = s_d + D, *s_u = s_ri + D, *s_cxx = s_u + D;
    int32_t *s_nx = reinterpret_cast<int32_t *>(s_cxx + D);
    const int32_t *nx = a.nbr + a.off[x];
    const double *Cx = a.C + (int64_t)x * a.ldc;
    const double Cxx = a.diag[x];
    for (int k = tid; k < D; k += blockDim.x) {
        const int g = nx[k];
        const double s = a.diag[g];
        const double ri = 1.0 / sqrt(s);
        const double cxk = Cx[g];
        const double u = cxk * ri;
        const double cxx = Cxx - u * u;
        s_nx[k] = g;
        s_cx[k] = cxk;
        s_d[k] = s;
        s_ri[k] = ri;
        s_u[k] = u;
        s_cxx[k] = ((s > 0.0) && (cxx == cxx)) ? cxx : __builtin_nan("");   // NaN marks !chol_ok
    }
    __syncthreads();
    const int npairs = D * (D - 1) / 2;                    // < 2^19 (D <= L1_MAXD)
    const int nch = (int)(a.cpre[x + 1] - a.cpre[x]);
    const int c = (int)(chunk - a.cpre[x]);
    const int p0 = (int)((int64_t)npairs * c / nch), p1 = (int)((int64_t)npairs * (c + 1) / nch);
    unsigned tests = 0, indep = 0;
    const float twoD1 = 2.0f * D - 1.0f;
    auto rowstart = [&](int r) -> int { return r * (2 * D - 1 - r) / 2; };
    const int ldc = (int)a.ldc;

    for (int pb = p0 + tid; pb < p1; pb += L1_PB * (int)blockDim.x) {
        // L1_PB pairs per lane: indices first, then every gather, then the tests
        int ys[L1_PB], zs[L1_PB];
        double cyz[L1_PB];
        uint64_t aw[L1_PB];
#pragma unroll
        for (int q = 0; q < L1_PB; ++q) {
            const int p = pb + q * (int)blockDim.x;
            int y = 0, z = 1;
            if (p < p1) {
                // pair p -> (y, z), y < z: row y starts at y(2D - 1 - y)/2 (fp32 root, then exact fix-up)
                y = (int)floorf((twoD1 - sqrtf(fmaxf(twoD1 * twoD1 - 8.0f * (float)p, 0.0f))) * 0.5f);
                if (y < 0) y = 0;
                while (y > 0 && rowstart(y) > p) --y;
                while (rowstart(y + 1) <= p) ++y;
                z = y + 1 + (p - rowstart(y));
            }
            ys[q] = y;
            zs[q] = z;
        }
#pragma unroll
        for (int q = 0; q < L1_PB; ++q) {
            const int yg = s_nx[ys[q]], zg = s_nx[zs[q]];
            if constexpr (I32) {
                cyz[q] = a.C[(uint32_t)(yg * ldc + zg)];
                aw[q] = a.adj[(uint32_t)(yg * W + (zg >> 6))];
            } else {
                cyz[q] = a.C[(int64_t)yg * a.ldc + zg];
                aw[q] = a.adj[(int64_t)yg * W + (zg >> 6)];
            }
        }
#pragma unroll
        for (int q = 0; q < L1_PB; ++q) {
            if (pb + q * (int)blockDim.x >= p1) continue;
            const int y = ys[q], z = zs[q];
            const int yg = s_nx[y], zg = s_nx[z];
            const bool adj_yz = (aw[q] >> (zg & 63)) & 1ull;
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                // side 0: test (x, y | z); side 1: test (x, z | y)
                const int t = side ? z : y;        // the tested neighbour (local), S = {k}
                const int k = side ? y : z;
                const int tg = side ? zg : yg, kg = side ? yg : zg;
                if (tg < x && adj_yz) continue;    // memo: node tg owns (tg, x, {kg})
                ++tests;
                const double cxx = s_cxx[k];
                int dec = 2;
                if (cxx == cxx) {
                    double pv = 0.0;
                    const double v = cyz[q] * s_ri[k];
                    const double cxt = s_cx[t] - s_u[k] * v;
                    const double ctt = s_d[t] - v * v;
                    dec = decide<MODE_DECIDE>(a, cxt, cxx, ctt, a.tau * s_ri[k] * s_ri[k], &pv);
                }
                if (dec == 2) {
                    const int sg[1] = {kg};
                    push_deferred(a, x, tg, sg, 1);
                } else if (dec == 1) {
                    ++indep;
                    if (PCG_L1_ABL) continue;      // timing ablation only (wrong results)
                    a.rm[(int64_t)x * a.n + tg] = 1;
                    a.rm[(int64_t)tg * a.n + x] = 1;
                    unsigned long long *row = reinterpret_cast<unsigned long long *>(
                        a.ug + ((int64_t)a.off[x] + t) * W);
                    atomicOr(&row[kg >> 6], 1ull << (kg & 63));
                    if (adj_yz && tg > x) {        // S in adj(tg): also tg's side of the pair
                        const int slot = a.off[tg] + find_in_sorted(a.nbr + a.off[tg], a.deg[tg], x);
                        unsigned long long *rowt = reinterpret_cast<unsigned long long *>(a.ug + (int64_t)slot * W);
                        atomicOr(&rowt[kg >> 6], 1ull << (kg & 63));
                    }
                }
            }
        }
    }
    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// depth 1 by conditioning node (threshold mode, one rank over the whole level; PCG_L1Z). The
// tests (x, t | z) with z in adj(x) are grouped by z: block z stages row z of C and of adj (both
// contiguous) and walks x in adj(z), t in adj(x) \ {z}, so C_xt comes from the graph's per-edge
// copy cxe[off[x] + j] = C[x][nbr[x][j]] (k_edge_c, read in CSR order) and C_tz, adj(t, z) from
// LDS: the scattered C[y][z] gathers of k_level1_pairs become streams. Same tests (the memo
// rule: (x, t | z) belongs to t's side when t < x and z in adj(t)), same arithmetic and decision
// as k_level1_pairs; C_tz is read as C[z][t] (C need not be bitwise symmetric: a 1-ulp change
// of an operand moves r^2 by ~1e-16, far inside the decision band, and band tests take the exact
// path either way). The block's (x, j) items are flattened over a prefix of the x's degrees in
// LDS (per-x terms staged once), so every lane has work and its loads of U items are in flight
// together; the mirror union row of an independent pair is found from adj(t)'s bit rank (one
// round of independent loads) instead of a binary search of nbr(t) (dependent loads).
#ifndef PCG_L1Z
#define PCG_L1Z 1
#endif
#ifndef PCG_L1Z_ABL
#define PCG_L1Z_ABL 0     // timing ablation only (wrong results): 1 no mirror rows, 2 no independence writes
#endif
#ifndef PCG_L1Z_FLAT
#define PCG_L1Z_FLAT 1    // 1: the sweep's common path without branches (depth-1 kernel 0.095 -> 0.090 ms); 0: k_level1_pairs' branch structure
#endif
#ifndef PCG_L1Z_DTE
#define PCG_L1Z_DTE 1     // C_tt per edge in CSR order (k_edge_c) instead of a gather of diag[t] per item
#endif
#ifndef L1Z_U
#define L1Z_U 4           // items in flight per lane
#endif
#ifndef L1Z_BS
#define L1Z_BS 512        // threads per block (one block per z; 8 waves fill a CU's wave slots at 4 blocks)
#endif
size_t l1z_lds_bytes(int64_t n, int W, int maxd) {
    return sizeof(double) * ((size_t)n + 2 * (size_t)maxd) + sizeof(uint64_t) * (size_t)W +
           sizeof(int32_t) * (3 * (size_t)maxd + 1) + 16;
}

__global__ __launch_bounds__(256) void k_edge_c(const double *C, int64_t ldc, const int32_t *deg, const int32_t *off,
                                                const int32_t *nbr, int n, const double *diag, double *cxe, double *dte) {
    const int x = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (x >= n) return;
    const int lane = threadIdx.x & 63, D = deg[x], o = off[x];
    const double *Cx = C + (int64_t)x * ldc;
    for (int j = lane; j < D; j += 64) {
        const int t = nbr[o + j];
        cxe[o + j] = Cx[t];
        if (PCG_L1Z_DTE) dte[o + j] = diag[t];
    }
}

#ifndef L1Z_MCAP
#define L1Z_MCAP 512      // mirror entries a block defers to its end (LDS); past them it searches inline
#endif
__global__ __launch_bounds__(L1Z_BS) void k_level1_z(LevelArgs a, const double *cxe, const double *dte) {
    __shared__ int2 s_ml[L1Z_MCAP];
    __shared__ unsigned s_mn;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int z = blockIdx.x, n = a.n, W = a.W, tid = threadIdx.x, lane = tid & 63;
    const int Dz = a.deg[z];
    unsigned tests = 0, indep = 0;
    if (tid == 0) s_mn = 0;
    if (Dz > 0) {
        double *cz = reinterpret_cast<double *>(smem);        // row z of C
        double *su = cz + n, *scxx = su + Dz;                  // per x in adj(z): u, c_xx|z (NaN: no Cholesky)
        uint64_t *az = reinterpret_cast<uint64_t *>(scxx + Dz);   // row z of adj
        int32_t *sx = reinterpret_cast<int32_t *>(az + W), *sox = sx + Dz, *spre = sox + Dz;   // x, off[x], item prefix
        const double *Cz = a.C + (int64_t)z * a.ldc;
        for (int e = tid; e < n; e += blockDim.x) cz[e] = Cz[e];
        for (int e = tid; e < W; e += blockDim.x) az[e] = a.adj[(int64_t)z * W + e];
        const double s = a.diag[z];
        const double ri = 1.0 / sqrt(s);
        const int32_t *nz = a.nbr + a.off[z];
        for (int xi = tid; xi < Dz; xi += blockDim.x) {
            const int x = nz[xi];
            const double u = a.C[(int64_t)x * a.ldc + z] * ri;
            const double cxx = a.diag[x] - u * u;
            sx[xi] = x;
            sox[xi] = a.off[x];
            spre[xi] = a.deg[x];
            su[xi] = u;
            scxx[xi] = ((s > 0.0) && (cxx == cxx)) ? cxx : __builtin_nan("");
        }
        __syncthreads();
        if (tid < 64) {   // exclusive prefix of the degrees (wave 0)
            int carry = 0;
            for (int b = 0; b < Dz; b += 64) {
                const int i = b + lane;
                const int v = i < Dz ? spre[i] : 0;
                int incl = v;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(incl, o);
                    if (lane >= o) incl += t;
                }
                if (i < Dz) spre[i] = carry + incl - v;
                carry += __shfl(incl, 63);
            }
            if (lane == 0) spre[Dz] = carry;
        }
        __syncthreads();
        const int P = spre[Dz];
        const double kg = a.tau * ri * ri;
        const int sg[1] = {z};
        // each wave walks a contiguous share of the items, 64 * L1Z_U at a time (lane l, slot q:
        // item b + 64 q + l); a lane's items ascend, so its x cursor only moves forward (one LDS
        // compare per item while D_x >= 64) after one binary search at the wave's start
        const int nw = (int)(blockDim.x >> 6), wv = tid >> 6;
        const int per = (P + nw - 1) / nw;
        const int pw0 = min(P, wv * per), pw1 = min(P, pw0 + per);
        int xi = 0;
        {
            const int p = min(pw0 + lane, max(P - 1, 0));
            int lo = 0, hi = Dz;                       // spre[lo] <= p < spre[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (spre[mid] <= p) lo = mid; else hi = mid;
            }
            xi = lo;
        }
        for (int b = pw0; b < pw1; b += 64 * L1Z_U) {
            int xs[L1Z_U], ts[L1Z_U], es[L1Z_U];
            double ce[L1Z_U], dt[L1Z_U];
#pragma unroll
            for (int q = 0; q < L1Z_U; ++q) {
                const int p = b + 64 * q + lane;
                int e = 0, t = z;
                if (p < pw1) {
                    while (spre[xi + 1] <= p) ++xi;
                    e = sox[xi] + (p - spre[xi]);
                    t = a.nbr[e];
                }
                xs[q] = xi;
                es[q] = e;
                ts[q] = t;
                ce[q] = p < pw1 ? cxe[e] : 0.0;
                if (PCG_L1Z_DTE) dt[q] = p < pw1 ? dte[e] : 0.0;
            }
            if (!PCG_L1Z_DTE) {
#pragma unroll
                for (int q = 0; q < L1Z_U; ++q) dt[q] = ts[q] != z ? a.diag[ts[q]] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < L1Z_U; ++q) {
                const int t = ts[q];
                const int xi = xs[q], x = sx[xi];
                const bool adj_tz = (az[t >> 6] >> (t & 63)) & 1ull;
                int dec = 2;
                if (PCG_L1Z_FLAT) {
                    // branch-free common path: every item is evaluated (t = z and the items past P
                    // too, on defined values) and only a live test that is not certainly dependent
                    // leaves it; decide<MODE_DECIDE>'s steps as selects (a NaN c_xx|z fails den > 0)
                    const bool live = t != z && !(t < x && adj_tz);   // memo: (t, x | z) on t's side
                    tests += live;
                    const double cxx = scxx[xi];
                    const double v = cz[t] * ri;
                    const double cxt = ce[q] - su[xi] * v;
                    const double ctt = dt[q] - v * v;
                    const double den = cxx * ctt, num = cxt * cxt;
                    const bool ok = den > 0.0 && den - num > kg;
                    dec = !ok ? 2 : num < a.lo2 * den ? 1 : num > a.hi2 * den ? 0 : 2;
                    if (!live || dec == 0) continue;
                } else {
                    if (t == z) continue;              // (also the items past P)
                    if (t < x && adj_tz) continue;     // memo: node t's side holds (t, x | z)
                    ++tests;
                    const double cxx = scxx[xi];
                    if (cxx == cxx) {
                        double pv = 0.0;
                        const double u = su[xi];
                        const double v = cz[t] * ri;
                        const double cxt = ce[q] - u * v;
                        const double ctt = dt[q] - v * v;
                        dec = decide<MODE_DECIDE>(a, cxt, cxx, ctt, kg, &pv);
                    }
                }
                if (dec == 2) {
                    push_deferred(a, x, t, sg, 1);
                } else if (dec == 1) {
                    ++indep;
                    if (PCG_L1Z_ABL == 2) continue;
                    a.rm[(int64_t)x * n + t] = 1;
                    a.rm[(int64_t)t * n + x] = 1;
                    unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + (int64_t)es[q] * W);
                    atomicOr(&row[z >> 6], 1ull << (z & 63));
                    if (PCG_L1Z_ABL != 1 && adj_tz && t > x) {   // S in adj(t): also t's side of the pair
                        // its row (x's position in nbr(t)) is searched at the block's end, one lane per
                        // entry, so the search's dependent loads do not stall the sweep (inline past
                        // L1Z_MCAP entries)
                        const unsigned long long act = __ballot(1);
                        const int leader = __ffsll((long long)act) - 1;
                        const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(act >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((unsigned)act, 0u));
                        unsigned base = 0;
                        if (lane == leader) base = atomicAdd(&s_mn, (unsigned)__popcll(act));
                        base = __shfl(base, leader);
                        const unsigned slot = base + rank;
                        if (slot < (unsigned)L1Z_MCAP) {
                            s_ml[slot] = make_int2(t, x);
                        } else {
                            const int r = find_in_sorted(a.nbr + a.off[t], a.deg[t], x);
                            unsigned long long *rowt = reinterpret_cast<unsigned long long *>(a.ug + ((int64_t)a.off[t] + r) * W);
                            atomicOr(&rowt[z >> 6], 1ull << (z & 63));
                        }
                    }
                }
            }
        }
    }
    __syncthreads();
    const int nm = (int)min(s_mn, (unsigned)L1Z_MCAP);
    for (int i = tid; i < nm; i += blockDim.x) {
        const int t = s_ml[i].x, x = s_ml[i].y;
        const int r = find_in_sorted(a.nbr + a.off[t], a.deg[t], x);
        unsigned long long *rowt = reinterpret_cast<unsigned long long *>(a.ug + ((int64_t)a.off[t] + r) * W);
        atomicOr(&rowt[z >> 6], 1ull << (z & 63));
    }
    block_flush_counts(a.ctr, tests, indep);
}

// The exact path of one test (numpy.linalg.inv-order LU of the m x m matrix A in LDS, the
// reference p expression): 0 ok, 1 singular, 2 math domain. Not inlined: its polynomial
// constants would otherwise be hoisted into registers across the callers' hot loops.
__device__ __attribute__((noinline)) int exact_lu_pvalue(double *A, int m, double *B0, double *B1, double sqrt_dof,
                                                         double *pv) {
    int piv[PCG_MAX_LEVEL_DEPTH + 2];
    double i00, i01, i11;
    if (pcg_lu_inv01(A, m, piv, B0, B1, &i00, &i01, &i11)) return 1;
    const double prod = i00 * i11;
    if (prod < 0.0) return 2;
    int err = 0;
    *pv = pcg_pvalue_from_r(-i01 / sqrt(prod), sqrt_dof, &err);
    return err;
}

// k_level_lds beyond PCG_MAX_DEPTH (no deferred list): the band tests a wave's lanes collected in
// their per-lane masks (bit t: the test (x, nbr t | S) of the lane's set S), decided one at a time
// by the whole wave in its LDS slot — gather the (d + 2)^2 submatrix of C, LU and the reference p
// on lane 0 (exact_lu_pvalue), as k_level_wave does. Every lane of the wave must call it.
__device__ void deep_band_exact(const LevelArgs &a, double *slot, int D, int d, int x, const int32_t *nxs,
                                const unsigned long long *lmask, unsigned long long *uself,
                                unsigned long long *uprop, int tx, unsigned long long Smask,
                                unsigned long long band, unsigned long long &indep) {
    const int lane = threadIdx.x & 63;
    unsigned long long need = __ballot(band != 0ull);
    const int mm = d + 2;
    double *A = slot, *B0 = slot + mm * mm, *B1 = B0 + mm;
    int *var = reinterpret_cast<int *>(B1 + mm);
    while (need) {
        const int L = __builtin_ctzll(need);
        need &= need - 1;
        const unsigned long long sm = readlane_u64(Smask, L);
        unsigned long long bm = readlane_u64(band, L);
        while (bm) {
            const int t = __builtin_ctzll(bm);
            bm &= bm - 1;
            const int yg = nxs[t];
            wave_sync();
            if (lane < D && ((sm >> lane) & 1ull)) var[2 + __popcll(sm & ((1ull << lane) - 1ull))] = nxs[lane];
            if (lane == 0) {
                var[0] = x < yg ? x : yg;
                var[1] = x < yg ? yg : x;
            }
            wave_sync();
            for (int k = lane; k < mm * mm; k += 64) {
                const int r = k / mm, c = k - r * mm;
                A[k] = a.C[(int64_t)var[r] * a.ldc + var[c]];
            }
            wave_sync();
            if (lane == 0) {
                double pv = __builtin_nan("");
                const int err = exact_lu_pvalue(A, mm, B0, B1, a.sqrt_dof, &pv);
                atomicAdd(&a.ctr->exact, 1ull);
                if (err) {
                    flag_error(a, err);
                } else {
                    if (fabs(pv - a.alpha) < 1e-9) atomicAdd(&a.ctr->near_alpha, 1ull);
                    if (pv > a.alpha) {
                        ++indep;
                        atomicOr(&uself[t], sm);
                        if (((lmask[t] & sm) == sm) && t >= tx) atomicOr(&uprop[t], sm);
                    }
                }
            }
        }
    }
    wave_sync();
}

// Element ii (0-based, from the top) of a colex unrank with remaining rank rr < C(hi, ii + 1): the
// largest c in [ii, hi - 1] with C(c, ii + 1) <= rr. Closed forms for the two lowest positions
// (every T-group task decodes them): C(c, 1) = c gives c = rr; C(c, 2) = c (c - 1) / 2 gives
// c = floor((1 + sqrt(1 + 8 rr)) / 2), fixed up by one either way (rr < C(128, 2): the fp32 root is
// within 1e-4 of the exact one). Deeper positions search the LDS table tab[c * stride + ii + 1].
#ifndef PCG_COLEX_CF
#define PCG_COLEX_CF 1   // A/B: 0 = the table search at every position
#endif
template <typename R, typename TAB>
__device__ __forceinline__ int colex_elem(int ii, R rr, int hi, const TAB *tab, int stride) {
    if (PCG_COLEX_CF && ii == 0) return (int)rr;
    if (PCG_COLEX_CF && ii == 1) {
        int c = (int)((1.0f + __builtin_sqrtf(1.0f + 8.0f * (float)rr)) * 0.5f);
        if ((R)(c * (c - 1) / 2) > rr) --c;
        else if ((R)((c + 1) * c / 2) <= rr) ++c;
        return c;
    }
    int lo_ = ii, up = hi - 1;
    while (lo_ < up) {
        const int mid = (lo_ + up + 1) >> 1;
        if (tab[mid * stride + ii + 1] <= rr) lo_ = mid; else up = mid - 1;
    }
    return lo_;
}

// ---------------------------------------------------------------------------------------
// depth d >= 1, nodes with D <= 64 neighbours: the node's whole local correlation block
// M[t][k] = C[nbr t, nbr k] (D x D), C[x, nbr t], C[nbr t, nbr t] and the local adjacency
// masks lmask[t] (bit k <=> nbr k in adj(nbr t)) are staged in LDS once per block; the
// y sweep then runs barrier-free: skip = bit t of the lane's S mask, subset test
// (S in adj(y)) = (lmask[t] & Smask) == Smask, memo ownership (y < x) = t < tx. Each lane
// walks `spl` S ranks (stride = block size) so the staging is amortised over
// spl * 256 * (D - d) tests. Sepset unions and removal flags accumulate in LDS (local bits)
// and are flushed once per block.
// 1/sqrt(x) in fp64 from the fp32 hardware estimate plus one Newton step (relative
// error ~1e-14 for normal fp32-range x; x <= 0 or out of fp32 range gives inf / NaN, which the
// callers' checks reject)
__device__ __forceinline__ double rsq_nr(double x) {
    const double r0 = (double)__builtin_amdgcn_rsqf((float)x);
    return r0 * fma(-0.5 * x * r0, r0, 1.5);
}

#ifndef PCG_LDS_EXACT_DM
#define PCG_LDS_EXACT_DM 1   // depths 5-12 (threshold / full-p): one k_level_lds instantiation per depth
#endif
#ifndef PCG_LDS_COLSOLVE
#define PCG_LDS_COLSOLVE 1   // k_level_lds beyond PCG_MAX_DEPTH: column-order forward solve (n = 1000 unlimited
                             // depth: depths 13-16 5 % faster; at depth 9 it cost 30 %, so only there)
#endif
#ifndef PCG_LDS_RSQ
#define PCG_LDS_RSQ 0        // k_level_lds beyond PCG_MAX_DEPTH: pivot reciprocals by rsq_nr (fewer VALU, but
                             // measured slower: n = 1000 900 vs 850 ms — the allocation of depths 19-20 spills more)
#endif
#ifndef PCG_LDS_COLCHOL
#define PCG_LDS_COLCHOL 0    // ... and the right-looking Cholesky there (same products, same order per entry;
                             // measured slower: n = 1000 900 vs 850 ms, its upfront block load spills at d >= 18)
#endif
#ifndef PCG_LDS_DEEP_TOP
#define PCG_LDS_DEEP_TOP 20   // k_level_lds instantiations beyond PCG_MAX_DEPTH (threshold mode), <= 20
#endif
#ifndef PCG_LDS_SPILL_MIN
#define PCG_LDS_SPILL_MIN 1e7 // depths 17..20 (instantiations that spill to scratch) take the per-lane kernel
                              // only for levels of at least this many tests (else the wave kernels)
#endif
static_assert(PCG_LDS_DEEP_TOP >= 12 && PCG_LDS_DEEP_TOP <= 20, "PCG_LDS_DEEP_TOP");
template <int DM, int MODE>
__global__ __launch_bounds__(256) void k_level_lds(LevelArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int bs = blockDim.x;
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int x = lo;
    const int D = a.deg[x];
    const int d = (DM <= 4 || (MODE != MODE_EXACT && PCG_LDS_EXACT_DM)) ? DM : a.d;
    const int32_t *nxg = a.nbr + a.off[x];

    double *M = reinterpret_cast<double *>(smem);                 // D * D
    double *Mx = M + D * D;                                       // D
    double *Md = Mx + D;                                          // D
    unsigned long long *lmask = reinterpret_cast<unsigned long long *>(Md + D);   // D
    unsigned long long *uself = lmask + D;                        // D
    unsigned long long *uprop = uself + D;                        // D
    int32_t *nxs = reinterpret_cast<int32_t *>(uprop + D);       // D
    int *s_tx = nxs + D;                                          // 1 (no static LDS: G17)

    for (int i = tid; i < D; i += bs) nxs[i] = nxg[i];
    __syncthreads();
    for (int e = tid; e < D * D; e += bs) {
        const int t = e / D, k = e - t * D;
        M[e] = a.C[(int64_t)nxs[t] * a.ldc + nxs[k]];
    }
    // local adjacency masks: one wave per row t, the wave's ballot over lanes k (D <= 64)
    for (int t = tid >> 6; t < D; t += bs >> 6) {
        const int k = tid & 63;
        const uint64_t *ar = a.adj + (int64_t)nxs[t] * a.W;
        const bool bit = k < D && ((ar[nxs[k] >> 6] >> (nxs[k] & 63)) & 1ull);
        const unsigned long long m = __ballot(bit);
        if (k == 0) lmask[t] = m;
    }
    for (int t = tid; t < D; t += bs) {
        const int yg = nxs[t];
        Mx[t] = a.C[(int64_t)x * a.ldc + yg];
        Md[t] = a.diag[yg];
        uself[t] = 0;
        uprop[t] = 0;
    }
    if (tid < 64) {                   // #neighbours below x (nxs ascends; D <= 64 here)
        const int c = __popcll(__ballot(tid < D && nxs[tid] < x));
        if (tid == 0) *s_tx = c;
    }
    __syncthreads();
    const int tx = *s_tx;
    const double Cxx = a.diag[x];
    const uint64_t nS = pcg_binom(a.binom, D, d);
    const uint64_t spl = (uint64_t)a.spl;
    const uint64_t r0 = (uint64_t)(chunk - a.cpre[x]) * (uint64_t)bs * spl;
    const uint64_t r1 = min(nS, r0 + (uint64_t)bs * spl);
    unsigned long long tests = 0, indep = 0;

    if constexpr (MODE == MODE_DECIDE && DM <= 4) {
        // Lanes take consecutive colex ranks (stride = block size): within a wave the S sets
        // share their high elements, so the per-y operand reads M[t][k_i] are broadcast or
        // consecutive (bank-conflict-light). Unranking uses an LDS copy of C(c, i), c <= D.
        unsigned long long *btab = reinterpret_cast<unsigned long long *>(smem + a.lds_btab_off);
        for (int e = tid; e < (D + 1) * (DM + 1); e += bs) {
            const int c = e / (DM + 1), i = e - c * (DM + 1);
            btab[e] = pcg_binom(a.binom, c, i);
        }
        __syncthreads();
        for (uint64_t rank = r0 + tid; rank < r1; rank += bs) {
            int k[DM];
            {
                uint64_t rr = rank;
                int hi_ = D;
#pragma unroll
                for (int ii = DM - 1; ii >= 0; --ii) {
                    const int lo_ = colex_elem(ii, rr, hi_, btab, DM + 1);
                    k[ii] = lo_;
                    rr -= btab[lo_ * (DM + 1) + ii + 1];
                    hi_ = lo_;
                }
            }
            unsigned long long Smask = 0;
#pragma unroll
            for (int i = 0; i < DM; ++i) Smask |= 1ull << k[i];
            // L = chol(M_SS); Li = L^-1 (lower); u = Li M_Sx; w = Li^T u (so u.v = w.b)
            double L[DM][DM], Li[DM][DM], u[DM], w[DM], b[DM];
            bool ok = true;
            double gmin = 1.0;
#pragma unroll
            for (int j = 0; j < DM; ++j) {
                double sdiag = M[k[j] * D + k[j]];
#pragma unroll
                for (int q = 0; q < j; ++q) sdiag -= L[j][q] * L[j][q];
                ok = ok && (sdiag > 0.0);
                gmin = fmin(gmin, sdiag);
                L[j][j] = sqrt(sdiag);
                const double r = 1.0 / L[j][j];
#pragma unroll
                for (int i = j + 1; i < DM; ++i) {
                    double t = M[k[i] * D + k[j]];
#pragma unroll
                    for (int q = 0; q < j; ++q) t -= L[i][q] * L[j][q];
                    L[i][j] = t * r;
                }
                Li[j][j] = r;
            }
#pragma unroll
            for (int i = 1; i < DM; ++i)
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    double t = 0.0;
#pragma unroll
                    for (int q = j; q < i; ++q) t += L[i][q] * Li[q][j];
                    Li[i][j] = -t * Li[i][i];
                }
            double uu = 0.0;
#pragma unroll
            for (int i = 0; i < DM; ++i) b[i] = Mx[k[i]];
#pragma unroll
            for (int i = 0; i < DM; ++i) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j <= i; ++j) t += Li[i][j] * b[j];
                u[i] = t;
                uu += t * t;
            }
#pragma unroll
            for (int j = 0; j < DM; ++j) {
                double t = 0.0;
#pragma unroll
                for (int i = j; i < DM; ++i) t += Li[i][j] * u[i];
                w[j] = t;
            }
            const double cxx = Cxx - uu;
            ok = ok && (cxx > 0.0);
            const double hc = a.hi2 * cxx, lc = a.lo2 * cxx, kg = a.tau / gmin;
            for (int t = 0; t < D; ++t) {
                const double *Mt = M + t * D;
#pragma unroll
                for (int i = 0; i < DM; ++i) b[i] = Mt[k[i]];
                double vv = 0.0, wb = 0.0;
#pragma unroll
                for (int i = 0; i < DM; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j <= i; ++j) v += Li[i][j] * b[j];
                    vv += v * v;
                    wb += w[i] * b[i];
                }
                const double cxy = Mx[t] - wb;
                const double cyy = Md[t] - vv;
                const double num = cxy * cxy;
                const double cond = fma(cxx, cyy, -num);   // c_xx c_yy (1 - r^2): guard, see decide
                const bool dep = (num > hc * cyy) && (cond > kg);
                const unsigned long long lm = lmask[t];
                const bool in_y = (lm & Smask) == Smask;
                const bool live = !((Smask >> t) & 1ull) && !(t < tx && in_y);
                tests += live;
                const bool rare = live && !(ok && dep);
                if (__ballot(rare)) {
                    if (rare) {
                        const bool ind = ok && (num < lc * cyy) && (cyy > 0.0) && (cond > kg);
                        if (ind) {
                            ++indep;
                            atomicOr(&uself[t], Smask);
                            if (in_y && t >= tx) atomicOr(&uprop[t], Smask);
                        } else {
                            int sg[DM];
#pragma unroll
                            for (int i = 0; i < DM; ++i) sg[i] = nxs[k[i]];
                            push_deferred(a, x, nxs[t], sg, d);
                        }
                    }
                }
            }
        }
    } else {
        // DM > PCG_MAX_DEPTH (threshold mode, depths 13..PCG_LDS_DEEP_MAX): no deferred list; a lane
        // marks its band tests in `band` and the wave decides them after the lane's sweep
        // (deep_band_exact), so the rank loop runs a wave-uniform trip count there
        constexpr bool DEEP = DM > PCG_MAX_DEPTH;
        static_assert(!DEEP || MODE == MODE_DECIDE, "k_level_lds beyond PCG_MAX_DEPTH: threshold mode only");
        double *dslot = DEEP ? reinterpret_cast<double *>(smem + a.lds_btab_off) + (size_t)(tid >> 6) * WAVE_SLOT_DOUBLES(DM)
                             : nullptr;
        for (uint64_t rank0 = r0 + (DEEP ? (uint64_t)(tid & ~63) : (uint64_t)tid); rank0 < r1; rank0 += bs) {
            const uint64_t rank = DEEP ? rank0 + (uint64_t)(tid & 63) : rank0;
            const bool act = !DEEP || rank < r1;
            int k[DM];
    #pragma unroll
            for (int i = 0; i < DM; ++i) k[i] = 0;
            pcg_unrank_colex<DM>(act ? rank : rank0, d, D, a.binom, k);
            unsigned long long Smask = 0;
    #pragma unroll
            for (int i = 0; i < DM; ++i)
                if (i < d) Smask |= 1ull << k[i];
            // Cholesky of M_SS, u = L^-1 M_Sx
            double L[DM][DM], rinv[DM], u[DM];
            bool ok = true;
            double gmin = 1.0;
            double uu = 0.0;
            if constexpr (PCG_LDS_COLSOLVE && DM > PCG_MAX_DEPTH && PCG_LDS_COLCHOL) {
                // right-looking (column) order, as the forward solve below: step j finishes column j
                // and updates the trailing entries and u's partial sums — independent updates, and
                // every entry subtracts the same products in the same (ascending) order as the
                // left-looking form: identical results
                double tu[DM];
    #pragma unroll
                for (int i = 0; i < DM; ++i) {
                    tu[i] = Mx[k[i]];
    #pragma unroll
                    for (int m = 0; m <= i; ++m) L[i][m] = M[k[i] * D + k[m]];
                }
    #pragma unroll
                for (int j = 0; j < DM; ++j) {
                    const double sj = L[j][j];
                    ok = ok && (sj > 0.0);
                    gmin = fmin(gmin, sj);
                    const double ljj = sqrt(sj);
                    rinv[j] = 1.0 / ljj;
                    L[j][j] = ljj;
                    u[j] = tu[j] * rinv[j];
                    uu += u[j] * u[j];
    #pragma unroll
                    for (int i = j + 1; i < DM; ++i) L[i][j] = L[i][j] * rinv[j];
    #pragma unroll
                    for (int i = j + 1; i < DM; ++i) {
                        tu[i] -= L[i][j] * u[j];
    #pragma unroll
                        for (int m = j + 1; m <= i; ++m) L[i][m] -= L[i][j] * L[m][j];
                    }
                }
            } else {
    #pragma unroll
            for (int j = 0; j < DM; ++j) {
                if (j < d) {
                    double s = M[k[j] * D + k[j]];
    #pragma unroll
                    for (int q = 0; q < DM; ++q)
                        if (q < j) s -= L[j][q] * L[j][q];
                    ok = ok && (s > 0.0);
                    gmin = fmin(gmin, s);
                    if constexpr (DM > PCG_MAX_DEPTH && PCG_LDS_RSQ) {
                        // threshold mode only: 1 / sqrt by the fp32 estimate + one Newton step
                        // (1e-14 relative, far inside the +-1e-6 band) instead of an IEEE sqrt and
                        // divide; a pivot below 1e-30 is clamped, and its tiny gmin keeps every
                        // test of the set off the decision (guard tau / gmin), so it goes exact
                        rinv[j] = rsq_nr(fmax(s, 1e-30));
                    } else {
                        const double ljj = sqrt(s);
                        rinv[j] = 1.0 / ljj;
                        L[j][j] = ljj;
                    }
    #pragma unroll
                    for (int i = 0; i < DM; ++i) {
                        if (i > j && i < d) {
                            double t = M[k[i] * D + k[j]];
    #pragma unroll
                            for (int q = 0; q < DM; ++q)
                                if (q < j) t -= L[i][q] * L[j][q];
                            L[i][j] = t * rinv[j];
                        }
                    }
                }
            }
    #pragma unroll
            for (int i = 0; i < DM; ++i) {
                if (i < d) {
                    double t = Mx[k[i]];
    #pragma unroll
                    for (int q = 0; q < DM; ++q)
                        if (q < i) t -= L[i][q] * u[q];
                    u[i] = t * rinv[i];
                    uu += u[i] * u[i];
                }
            }
            }
            const double cxx = Cxx - uu;
            ok = ok && (cxx == cxx);

            unsigned long long band = 0;
            for (int t = 0; t < D; ++t) {
                if (!act || ((Smask >> t) & 1ull)) continue;
                const unsigned long long lm = lmask[t];
                const bool in_y = (lm & Smask) == Smask;
                if (t < tx && in_y) continue;          // node nbr[t] < x owns this test (memo)
                ++tests;
                int dec = 2;
                double p = 0.0;
                if (ok) {
                    const double *Mt = M + t * D;
                    double vv = 0.0, uv = 0.0;
                    if constexpr (PCG_LDS_COLSOLVE && DM > PCG_MAX_DEPTH) {
                        // the forward solve column by column: step q finishes v_q and updates every
                        // later row's partial sum, so the d - q - 1 updates of a step are
                        // independent (the row-by-row form gave the scheduler one dependent fp64
                        // chain at the one wave per SIMD of the deep instantiations). Each row's
                        // sum subtracts the same products in the same order: identical results.
                        double tt[DM];
    #pragma unroll
                        for (int i = 0; i < DM; ++i) tt[i] = i < d ? Mt[k[i]] : 0.0;
    #pragma unroll
                        for (int q = 0; q < DM; ++q) {
                            if (q < d) {
                                const double vq = tt[q] * rinv[q];
                                vv += vq * vq;
                                uv += u[q] * vq;
    #pragma unroll
                                for (int i = q + 1; i < DM; ++i)
                                    if (i < d) tt[i] -= L[i][q] * vq;
                            }
                        }
                    } else {
                        double v[DM];
    #pragma unroll
                        for (int i = 0; i < DM; ++i) {
                            if (i < d) {
                                double tt = Mt[k[i]];
    #pragma unroll
                                for (int q = 0; q < DM; ++q)
                                    if (q < i) tt -= L[i][q] * v[q];
                                v[i] = tt * rinv[i];
                                vv += v[i] * v[i];
                                uv += u[i] * v[i];
                            }
                        }
                    }
                    dec = decide<MODE>(a, Mx[t] - uv, cxx, Md[t] - vv, a.tau / gmin, &p);
                }
                if constexpr (DEEP) {
                    if (dec == 2) {
                        band |= 1ull << t;
                        continue;
                    }
                } else if (dec == 2 || (MODE == MODE_FULLP && (a.record || fabs(p - a.alpha) < 1e-9))) {
                    int sg[DM];
    #pragma unroll
                    for (int i = 0; i < DM; ++i) sg[i] = i < d ? nxs[k[i]] : 0;
                    const int yg = nxs[t];
                    if (dec == 2) {
                        push_deferred(a, x, yg, sg, d);
                        continue;
                    }
                    const int lo_ = x < yg ? x : yg, hi_ = x < yg ? yg : x;
                    if (rec_on(a, lo_, hi_)) push_record(a.records, a.rec_cap, &a.ctr->records, lo_, hi_, d, sg, p);
                    if (fabs(p - a.alpha) < 1e-9)
                        push_record(a.nearl, a.near_cap, &a.ctr->near_alpha, lo_, hi_, d, sg, p);
                }
                if (dec == 1) {
                    ++indep;
                    atomicOr(&uself[t], Smask);
                    if (in_y && t >= tx) atomicOr(&uprop[t], Smask);
                }
            }
            if constexpr (DEEP) deep_band_exact(a, dslot, D, d, x, nxs, lmask, uself, uprop, tx, Smask, band, indep);
        }
    }
    __syncthreads();
    // flush unions (local bits -> global node bits) and removal flags
    for (int t = tid; t < D; t += bs) {
        const unsigned long long us = uself[t], up = uprop[t];
        if (!(us | up)) continue;
        const int yg = nxs[t];
        a.rm[(int64_t)x * a.n + yg] = 1;
        a.rm[(int64_t)yg * a.n + x] = 1;
        if (us) {
            unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + ((int64_t)a.off[x] + t) * a.W);
            unsigned long long m = us;
            while (m) {
                const int b = __ffsll((long long)m) - 1;
                const int g = nxs[b];
                atomicOr(&row[g >> 6], 1ull << (g & 63));
                m &= m - 1;
            }
        }
        if (up) {
            const int slot = a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x);
            unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + (int64_t)slot * a.W);
            unsigned long long m = up;
            while (m) {
                const int b = __ffsll((long long)m) - 1;
                const int g = nxs[b];
                atomicOr(&row[g >> 6], 1ull << (g & 63));
                m &= m - 1;
            }
        }
    }
    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// depth 2..4, D <= 64, threshold decision: "T-group" form of the LDS-resident kernel.
// A lane owns a (d-1)-subset T of adj(x) and a group of TG consecutive candidates c with
// c < min(T) (S = {c} + T, ascending). Factoring T first and c last, per y it forms
//   v_T = L_T^-1 M[T][y],  byy = M_yy - |v_T|^2,  bxy = M_xy - u_T.v_T     (once per y)
// and per c only the last row of the triangular solve:
//   v_c = (M[c][y] - l_c.v_T) / lambda_c,  c_yy = byy - v_c^2,  c_xy = bxy - u_c v_c
// — the same partial correlation, ~9 fp64 ops per test instead of ~26. Tasks (g, T): group
// g covers c in [g*TG, g*TG+TG), T ranges over (d-1)-subsets of [g*TG+1, D) in colex order.
// blocks per CU each depth's T-group kernel is register-sized for: 4 (128 VGPRs) at depths 2-3,
// 3 (168 VGPRs) for depth 4's groups of 6
#ifndef PCG_MB2
#define PCG_MB2 4
#endif
#ifndef PCG_MB3
#define PCG_MB3 4
#endif
#ifndef PCG_MB4
#define PCG_MB4 3
#endif
__host__ __device__ constexpr int tg_minblocks(int DM) { return DM == 2 ? PCG_MB2 : (DM == 3 ? PCG_MB3 : PCG_MB4); }
// WIDE: nodes with 64 < D <= WIDE_DEG (128) — the same kernel with 128-bit local masks (the
// few high-degree nodes of depths 2-3 that the staged generic kernel used to take)
template <bool WIDE>
using LMask = std::conditional_t<WIDE, unsigned __int128, unsigned long long>;

template <bool WIDE>
__device__ __forceinline__ void lmask_atomic_or(LMask<WIDE> *p, LMask<WIDE> v) {
    if constexpr (WIDE) {
        unsigned long long *q = reinterpret_cast<unsigned long long *>(p);
        const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
        if (lo) atomicOr(q, lo);
        if (hi) atomicOr(q + 1, hi);
    } else {
        atomicOr(p, v);
    }
}

// The T-group lane tasks' (g, t0) pair table of a node of degree D, built by the whole block:
// pairs g-major, t0 = g TG + 1 .. D - DT ascending; a pair holds C(D - 1 - t0, DT - 1) tasks, so
// (hockey stick) a group's tasks from t0 on number C(D - t0, DT) and
//   ppre(g, t0) = sum_{g' < g} C(D - g' TG - 1, DT) + C(D - g TG - 1, DT) - C(D - t0, DT).
// Every entry is independent (the serial thread-0 loop it replaces took ~D^2 / TG dependent LDS
// round trips, 9-12 us per block at depths 3-4). s_tx = #neighbours below x (ballots).
template <int DM, int TG>
__device__ __forceinline__ void tgroup_pairs(int D, int x, const int32_t *nxs, const unsigned *btab, unsigned *ppre,
                                             unsigned short *pinfo, int *s_tx, int *s_np) {
    constexpr int DT = DM - 1;
    const int tid = threadIdx.x, bs = blockDim.x;
    const int ng = (D - DM) / TG + 1;
    int np = 0;
    for (int g = 0; g < ng; ++g) np += D - DT - g * TG;
    for (int q = tid; q < np; q += bs) {
        int g = 0, base = 0;
        while (base + (D - DT - g * TG) <= q) {
            base += D - DT - g * TG;
            ++g;
        }
        const int t0 = g * TG + 1 + (q - base);
        unsigned pre = btab[(D - g * TG - 1) * (DM + 1) + DT] - btab[(D - t0) * (DM + 1) + DT];
        for (int h = 0; h < g; ++h) pre += btab[(D - h * TG - 1) * (DM + 1) + DT];
        ppre[q] = pre;
        pinfo[q] = (unsigned short)((g << 8) | t0);
    }
    if (tid < 64) {
        int c = 0;
        for (int k0 = 0; k0 < D; k0 += 64) {
            const int k = k0 + tid;
            c += __popcll(__ballot(k < D && nxs[k] < x));
        }
        if (tid == 0) {
            unsigned tot = 0;
            for (int g = 0; g < ng; ++g) tot += btab[(D - g * TG - 1) * (DM + 1) + DT];
            ppre[np] = tot;
            *s_np = np;
            *s_tx = c;
        }
    }
}

// The (g, t0) pair of T-group task `task`: the last q < np with ppre[q] <= task (ppre ascends,
// ppre[np] = the task count > task). A lane's tasks ascend (stride = block size), so the search
// gallops forward from the previous task's pair (ppre[from] <= task): one or two probes per task
// instead of a log2(np) binary search of dependent LDS reads. PCG_TG_GALLOP: the kernels (bit 0
// the fp64 k_level_lds_t, bit 1 the fp32 k_level_lds_f) that gallop; measured at config 5: depth 4
// 1.93 vs 1.98 ms, depth 2 (fp64) 0.22 vs 0.21 ms, so the fp32 sweep only
#ifndef PCG_TG_GALLOP
#define PCG_TG_GALLOP 2
#endif
template <bool GALLOP>
__device__ __forceinline__ int tg_pair_search(const unsigned *ppre, int np, unsigned task, int from) {
    int lq = GALLOP ? from : 0, hq = np;
    if (GALLOP) {
        int step = 1;
        hq = min(np, lq + 1);
        while (hq < np && ppre[hq] <= task) {
            lq = hq;
            step <<= 1;
            hq = min(np, lq + step);
        }
    }
    while (hq - lq > 1) {
        const int mid = (lq + hq) >> 1;
        if (ppre[mid] <= task) lq = mid; else hq = mid;
    }
    return lq;
}

#ifndef PCG_TGT_BATCH
#define PCG_TGT_BATCH 1   // k_level_lds_t stages M and the local masks row-batched (0: per element, A/B)
#endif
template <int DM, bool WIDE>
__global__ __launch_bounds__(256, WIDE ? 1 : tg_minblocks(DM)) void k_level_lds_t(LevelArgs a) {
    using Mask = LMask<WIDE>;
    constexpr int DT = DM - 1;
    constexpr int TG = tg_of_depth(DM);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int bs = blockDim.x;
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int x = lo;
    const int D = a.deg[x];
    const int32_t *nxg = a.nbr + a.off[x];

    const int DS = (D + 3) & ~3;                                  // row stride: 32-B aligned rows
    double *M = reinterpret_cast<double *>(smem);                 // D * DS (columns >= D zero)
    double *Mx = M + D * DS;                                      // D
    double *Md = Mx + D;                                          // D
    Mask *lmask = reinterpret_cast<Mask *>(Md + D);              // D (16-B aligned: DS % 4 == 0)
    Mask *uself = lmask + D;                                      // D
    Mask *uprop = uself + D;                                      // D
    int32_t *nxs = reinterpret_cast<int32_t *>(uprop + D);       // D
    int *s_tx = nxs + D;                                          // 1
    unsigned *btab = reinterpret_cast<unsigned *>(smem + a.lds_btab_off);   // C(c, i), c <= D, i <= DM
    unsigned *ppre = btab + (D + 1) * (DM + 1);                   // task prefix per (g, t0) pair
    unsigned short *pinfo = reinterpret_cast<unsigned short *>(ppre + tg_pairs(D, DM) + 1);  // g << 8 | t0
    int *s_np = s_tx + 1;

    for (int i = tid; i < D; i += bs) nxs[i] = nxg[i];
    for (int e = tid; e < (D + 1) * (DM + 1); e += bs) {
        const int c = e / (DM + 1), i = e - c * (DM + 1);
        btab[e] = (unsigned)pcg_binom(a.binom, c, i);             // <= C(64, 4): fits 32 bits
    }
    __syncthreads();
    if (PCG_TGT_BATCH) {
        // rows of M and of the local adjacency masks: a wave takes SR rows at a time, lane k column
        // k (+ 64: WIDE), so SR x H x (C entry, adjacency word) loads are in flight per lane before
        // the first is used (the per-element loop below waits out one gather round trip per ~8
        // entries of a thread: ~20 dependent round trips per block at D = 45, ~64 at D = 128)
        constexpr int H = WIDE ? 2 : 1, SR = WIDE ? 2 : 4;
        const int lane = tid & 63, wv = tid >> 6, nwv = bs >> 6;
        int kg[H];
#pragma unroll
        for (int hh = 0; hh < H; ++hh) kg[hh] = lane + 64 * hh < D ? nxs[lane + 64 * hh] : -1;
        for (int t0 = wv * SR; t0 < D; t0 += nwv * SR) {
            double v[SR][H];
            uint64_t w[SR][H];
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                const int rg = nxs[min(t0 + r, D - 1)];
#pragma unroll
                for (int hh = 0; hh < H; ++hh) {
                    const int k = kg[hh] < 0 ? 0 : kg[hh];
                    v[r][hh] = a.C[(int64_t)rg * a.ldc + k];
                    w[r][hh] = a.adj[(int64_t)rg * a.W + (k >> 6)];
                }
            }
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                const int t = t0 + r;
                if (t >= D) break;                   // wave-uniform
                Mask m = 0;
#pragma unroll
                for (int hh = 0; hh < H; ++hh) {
                    const int k = lane + 64 * hh;
                    if (k < DS) M[t * DS + k] = kg[hh] >= 0 ? v[r][hh] : 0.0;
                    const bool bit = kg[hh] >= 0 && ((w[r][hh] >> (kg[hh] & 63)) & 1ull);
                    m |= (Mask)__ballot(bit) << (64 * hh);
                }
                if (lane == 0) lmask[t] = m;
            }
        }
    } else {
        for (int e = tid; e < D * DS; e += bs) {
            const int t = e / DS, k = e - t * DS;
            M[e] = k < D ? a.C[(int64_t)nxs[t] * a.ldc + nxs[k]] : 0.0;
        }
        // local adjacency masks: one wave per row t, lane k reads the bit adj(nxs[t], nxs[k]) and the
        // wave's ballot is the row's 64-bit word (64 independent loads in flight per row)
        for (int t = tid >> 6; t < D; t += bs >> 6) {
            const uint64_t *ar = a.adj + (int64_t)nxs[t] * a.W;
            Mask m = 0;
            for (int k0 = 0; k0 < D; k0 += 64) {
                const int k = k0 + (tid & 63);
                const bool bit = k < D && ((ar[nxs[k] >> 6] >> (nxs[k] & 63)) & 1ull);
                m |= (Mask)__ballot(bit) << k0;
            }
            if ((tid & 63) == 0) lmask[t] = m;
        }
    }
    for (int t = tid; t < D; t += bs) {
        const int yg = nxs[t];
        Mx[t] = a.C[(int64_t)x * a.ldc + yg];
        Md[t] = a.diag[yg];
        uself[t] = 0;
        uprop[t] = 0;
    }
    tgroup_pairs<DM, TG>(D, x, nxs, btab, ppre, pinfo, s_tx, s_np);
    // full-p mode with records (PCG_FLAG_RECORD): the recorded pairs (x, y) of this node, bit t.
    // Every live test of such a y goes to the exact path, which decides it with the reference's
    // own arithmetic and records its p (k_exact); the others are decided as in threshold mode
    __shared__ Mask s_recm;
    if (tid < 64) {
        Mask rm_ = 0;
        if (a.record)
            for (int k0 = 0; k0 < D; k0 += 64) {
                const int t = k0 + tid;
                const int yg = t < D ? nxs[t] : 0;
                rm_ |= (Mask)__ballot(t < D && rec_on(a, min(x, yg), max(x, yg))) << k0;
            }
        if (tid == 0) s_recm = rm_;
    }
    __syncthreads();
    const int tx = *s_tx;
    const int np = *s_np;
    const Mask recm = s_recm;
    const double Cxx = a.diag[x];
    const uint64_t ntask = ppre[np];
    const uint64_t spl = (uint64_t)a.spl;
    const uint64_t r0 = (uint64_t)(chunk - a.cpre[x]) * (uint64_t)bs * spl;
    const uint64_t r1 = min(ntask, r0 + (uint64_t)bs * spl);
    unsigned long long tests = 0, indep = 0;
    unsigned tcount = 0;

    int lq_prev = 0;
    for (uint64_t task = r0 + tid; task < r1; task += bs) {
        // (g, t0) pair of this task: the last pair whose prefix is <= task
        int lq = tg_pair_search<(PCG_TG_GALLOP & 1) != 0>(ppre, np, (unsigned)task, lq_prev);
        lq_prev = lq;
        const int info = pinfo[lq];
        const int cbase = (info >> 8) * TG;
        int T[DT];
        T[0] = info & 255;
        {   // colex unrank of T \ {t0}, a (d-2)-subset of (t0, D)
            unsigned rr = (unsigned)(task - ppre[lq]);
            int hi_ = D - T[0] - 1;
#pragma unroll
            for (int ii = DT - 2; ii >= 0; --ii) {
                const int lo_ = colex_elem(ii, rr, hi_, btab, DM + 1);
                T[ii + 1] = lo_;
                rr -= btab[lo_ * (DM + 1) + ii + 1];
                hi_ = lo_;
            }
#pragma unroll
            for (int ii = 1; ii < DT; ++ii) T[ii] += T[0] + 1;
        }
        // candidates c in [cbase, min(t0, cbase + TG)): lanes of a wave share t0 except at pair
        // boundaries, so the wave's largest candidate count bounds the sweep uniformly
        const int nval = min(T[0] - cbase, TG);
        int nmax_ = 1;
#pragma unroll
        for (int k = 2; k <= TG; ++k) nmax_ += (__ballot(nval >= k) != 0);
        const int nmax = __builtin_amdgcn_readfirstlane(nmax_);
        Mask Tmask = 0;
#pragma unroll
        for (int i = 0; i < DT; ++i) Tmask |= (Mask)1 << T[i];
        // T-info: L_T, Li_T = L_T^-1, u_T = Li_T M_Tx
        double L[DT][DT], Li[DT][DT], uT[DT];
        bool okT = true;
        double gmin = 1.0;   // smallest pivot^2 over T and the group's valid candidates (guard)
#pragma unroll
        for (int j = 0; j < DT; ++j) {
            double s = M[T[j] * DS + T[j]];
#pragma unroll
            for (int q = 0; q < j; ++q) s -= L[j][q] * L[j][q];
            okT = okT && (s > 0.0);
            gmin = fmin(gmin, s);
            L[j][j] = sqrt(s);
            const double r = 1.0 / L[j][j];
#pragma unroll
            for (int i = j + 1; i < DT; ++i) {
                double t = M[T[i] * DS + T[j]];
#pragma unroll
                for (int q = 0; q < j; ++q) t -= L[i][q] * L[j][q];
                L[i][j] = t * r;
            }
            Li[j][j] = r;
        }
#pragma unroll
        for (int i = 1; i < DT; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double t = 0.0;
#pragma unroll
                for (int q = j; q < i; ++q) t += L[i][q] * Li[q][j];
                Li[i][j] = -t * Li[i][i];
            }
        double uuT = 0.0;
#pragma unroll
        for (int i = 0; i < DT; ++i) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j <= i; ++j) t += Li[i][j] * Mx[T[j]];
            uT[i] = t;
            uuT += t * t;
        }
        // c-data for the group
        double lc[TG][DT], rl[TG], uc[TG], hc[TG];
        bool okc[TG];
#pragma unroll
        for (int jj = 0; jj < TG; ++jj) {
            rl[jj] = uc[jj] = hc[jj] = 0.0;
            okc[jj] = false;
#pragma unroll
            for (int i = 0; i < DT; ++i) lc[jj][i] = 0.0;
            if (jj >= nmax) continue;                 // wave-uniform
            const int c = cbase + jj;
            const bool valid = c < T[0];
            const int cc = valid ? c : 0;
            double ll = 0.0;
#pragma unroll
            for (int i = 0; i < DT; ++i) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j <= i; ++j) t += Li[i][j] * M[T[j] * DS + cc];
                lc[jj][i] = t;
                ll += t * t;
            }
            const double lam2 = M[cc * DS + cc] - ll;
            const double r = 1.0 / sqrt(lam2);
            double lu = 0.0;
#pragma unroll
            for (int i = 0; i < DT; ++i) lu += lc[jj][i] * uT[i];
            const double u = (Mx[cc] - lu) * r;
            const double cxx = Cxx - uuT - u * u;
            rl[jj] = r;
            uc[jj] = u;
            hc[jj] = a.hi2 * cxx;
            okc[jj] = valid && okT && (lam2 > 0.0) && (cxx > 0.0);
            if (valid) gmin = fmin(gmin, lam2);
        }
#if PCG_TG_WC
        // w_c = L_T^-T l_c = C_TT^-1 M[T][c]: then l_c . v_T = w_c . M[T][y], so each candidate's
        // chain starts from the row loads instead of waiting for v_T (same count of FMAs)
#pragma unroll
        for (int jj = 0; jj < TG; ++jj) {
            double w[DT];
#pragma unroll
            for (int i = 0; i < DT; ++i) {
                double t = 0.0;
#pragma unroll
                for (int k = i; k < DT; ++k) t += Li[k][i] * lc[jj][k];
                w[i] = t;
            }
#pragma unroll
            for (int i = 0; i < DT; ++i) lc[jj][i] = w[i];
        }
#endif
        // conditioning guard (see decide): c_xx c_yy - c_xy^2 > tau / g, with c_xx c_yy
        // recovered from the threshold product th = hi2 c_xx c_yy the sweep forms anyway
        const double inv_hi2 = 1.0 / a.hi2;
        const double kg = a.tau / gmin;
        const int cend = min(T[0], cbase + TG);      // valid candidates: c in [cbase, cend), >= 1 of them
        unsigned okm = 0;                            // candidates usable on the fast path
#pragma unroll
        for (int jj = 0; jj < TG; ++jj) okm |= (unsigned)okc[jj] << jj;
        const unsigned vmask = (1u << (cend - cbase)) - 1u;
        constexpr bool SG = ((WIDE ? PCG_TG_SGPR_WIDE : PCG_TG_SGPR) >> DM) & 1;
        // lane-mask form of the sweep's bookkeeping. Tests per task are counted in closed form:
        // every valid candidate meets every y outside T except itself, minus the dedup skips of
        // "own" y (counted in the rare path below). okv[jj]: lanes whose candidate jj is valid
        // and fast-path usable; notok: lanes with a valid candidate that is not (every y of such
        // a lane takes the rare path); uni: the wave's lanes share one candidate window, so the
        // y equal to a candidate is masked by a scalar index instead of the rare path.
        unsigned long long okv[TG], notok = 0ull, lanebit = 0ull;
        int cb0 = 0;
        bool uni = false;
        if constexpr (SG) {
            tcount += (unsigned)(nval * (D - DT - 1));     // nval = cend - cbase
#pragma unroll
            for (int jj = 0; jj < TG; ++jj) okv[jj] = __builtin_amdgcn_ballot_w64(okc[jj]);
            notok = __builtin_amdgcn_ballot_w64((vmask & ~okm) != 0u);
            cb0 = __builtin_amdgcn_readfirstlane(cbase);
            uni = __builtin_amdgcn_ballot_w64(cbase != cb0) == 0ull;
            lanebit = 1ull << (tid & 63);
        }

        // the y sweep, specialised on the wave-uniform candidate count so the NC chains stay
        // branch-free and interleaved (candidates beyond the count are not evaluated at all)
        auto sweep = [&](auto nc_tag) {
            constexpr int NC = decltype(nc_tag)::value;
            if constexpr (SG) {
            auto ystep = [&](int t, auto ym_tag) {
                constexpr int YM = decltype(ym_tag)::value;
                const Mask lm = lmask[t];
                const double *Mt = M + t * DS;
                double sc[TG];
#pragma unroll
                for (int q = 0; q < (NC + 1) / 2; ++q) {
                    const double2 m = *reinterpret_cast<const double2 *>(Mt + cbase + 2 * q);
                    sc[2 * q] = m.x;
                    sc[2 * q + 1] = m.y;
                }
                double vT[DT], mT[DT];
                double vv = 0.0, uv = 0.0;
#pragma unroll
                for (int j = 0; j < DT; ++j) mT[j] = Mt[T[j]];
#pragma unroll
                for (int i = 0; i < DT; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j <= i; ++j) v += Li[i][j] * mT[j];
                    vT[i] = v;
                    vv += v * v;
                    uv += uT[i] * v;
                }
                double projv[DT];
#pragma unroll
                for (int i = 0; i < DT; ++i) projv[i] = PCG_TG_WC ? mT[i] : vT[i];
                const double byy = Md[t] - vv;
                const double bxy = Mx[t] - uv;
#pragma unroll
                for (int i = 0; i < DT; ++i)
#pragma unroll
                    for (int jj = 0; jj < NC; ++jj) sc[jj] -= lc[jj][i] * projv[i];
                // lanes whose usable candidates are not all dependent at this y
                // YM 0: no candidate equals y for any lane (a shared window outside y); 1: shared
                // window holding y (candidate t - cb0 is y: masked by its scalar index); 2: lanes
                // with different windows (a lane whose window holds y takes the rare path)
                const int jdead = YM == 1 ? t - cb0 : -1;
                unsigned long long bad = 0ull;
#pragma unroll
                for (int jj = 0; jj < NC; ++jj) {
                    const double vc = sc[jj] * rl[jj];
                    const double cyy = byy - vc * vc;
                    const double cxy = bxy - uc[jj] * vc;
                    const double num = cxy * cxy;
                    const double th = hc[jj] * cyy;
                    const unsigned long long keep = jj == jdead ? 0ull : okv[jj];
                    // one ballot per compare: each is the compare's own lane mask (no VGPR round trip)
                    bad |= keep & ~(__builtin_amdgcn_ballot_w64(num > th) &
                                    __builtin_amdgcn_ballot_w64(fma(th, inv_hi2, -kg) > num));
                }
                const unsigned long long inT = __builtin_amdgcn_ballot_w64((bool)((Tmask >> t) & 1u));
                const bool recy = (bool)((recm >> t) & 1u);     // wave-uniform
                unsigned long long rarel = (bad | notok) & ~inT;
                if (YM == 2) rarel |= __builtin_amdgcn_ballot_w64((unsigned)(t - cbase) < (unsigned)nval);
                if (t < tx) rarel |= __builtin_amdgcn_ballot_w64((lm & Tmask) == Tmask) & ~inT;
                if (recy) rarel = __builtin_amdgcn_read_exec() & ~inT;
                if (!rarel) return;
                if (!(rarel & lanebit)) return;
                // rare path (this lane): the exact live set, the dedup skips, then the per-lane
                // decision bits from the wave masks
                const bool own = (t < tx) && ((lm & Tmask) == Tmask);
                const unsigned tb = ((unsigned)(t - cbase) < (unsigned)TG) ? (1u << (t - cbase)) : 0u;
                const unsigned skip = own ? (unsigned)(lm >> cbase) : 0u;
                if ((Tmask >> t) & 1u) return;
                const unsigned live = vmask & ~tb & ~skip;
                tcount -= __popc(vmask & ~tb & skip);
                if (recy) {                                   // recorded pair: every live test to the exact path
#pragma unroll
                    for (int jj = 0; jj < TG; ++jj) {
                        if (!((live >> jj) & 1u)) continue;
                        int sg[DM];
                        sg[0] = nxs[cbase + jj];
#pragma unroll
                        for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
                        push_deferred(a, x, nxs[t], sg, DM);
                    }
                    return;
                }
#pragma unroll
                for (int jj = 0; jj < TG; ++jj) {
                    if (!((live >> jj) & 1u)) continue;
                    const int c = cbase + jj;
                    double s_ = Mt[c];
#pragma unroll
                    for (int i = 0; i < DT; ++i) s_ -= lc[jj][i] * projv[i];
                    const double vc = s_ * rl[jj];
                    const double cyy = byy - vc * vc;
                    const double cxy = bxy - uc[jj] * vc;
                    {   // the fast path's decision, recomputed in the same operation order
                        const double num = cxy * cxy;
                        const double th = hc[jj] * cyy;
                        if (okc[jj] && (num > th) && (fma(th, inv_hi2, -kg) > num)) continue;
                    }
                    const double cxx = hc[jj] / a.hi2;
                    const bool ind = okc[jj] && (cxy * cxy < a.lo2 * cxx * cyy) && (cyy > 0.0) &&
                                     (cxx * cyy - cxy * cxy > kg);
                    const Mask Smask = Tmask | ((Mask)1 << c);
                    if (ind) {
                        ++indep;
                        lmask_atomic_or<WIDE>(&uself[t], Smask);
                        if (((lm & Smask) == Smask) && t >= tx) lmask_atomic_or<WIDE>(&uprop[t], Smask);
                    } else {
                        int sg[DM];
                        sg[0] = nxs[c];
#pragma unroll
                        for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
                        push_deferred(a, x, nxs[t], sg, DM);
                    }
                }
            };
            using Y0 = std::integral_constant<int, 0>;
            using Y1 = std::integral_constant<int, 1>;
            using Y2 = std::integral_constant<int, 2>;
            if (PCG_TG_SPLIT && uni) {
                const int w0 = min(cb0, D), w1 = min(cb0 + TG, D);
                for (int t = 0; t < w0; ++t) ystep(t, Y0{});
                for (int t = w0; t < w1; ++t) ystep(t, Y1{});
                for (int t = w1; t < D; ++t) ystep(t, Y0{});
            } else if (uni) {
                for (int t = 0; t < D; ++t) ystep(t, Y1{});
            } else {
                for (int t = 0; t < D; ++t) ystep(t, Y2{});
            }
            return;
            }
            // YU consecutive y per iteration: their chains are independent, so the in-order issue of
            // one wave has twice the fp64 work in flight (PCG_TG_Y2)
            constexpr int YU = ((PCG_TG_Y2 >> DM) & 1) ? 2 : 1;
            for (int t0y = 0; t0y < D; t0y += YU) {
                int tt[YU];
                Mask lmv[YU];
                double byy[YU], bxy[YU], projv[YU][DT];
                unsigned live[YU], dep[YU];
#pragma unroll
                for (int k = 0; k < YU; ++k) {
                    const int t = min(t0y + k, D - 1);
                    tt[k] = t;
                    // t in T: the lane idles through this y (branch-free: no exec-mask split)
                    const bool inTset = (bool)((Tmask >> t) & 1u) || (t0y + k >= D);
                    const Mask lm = lmask[t];
                    lmv[k] = lm;
                    const bool own = (t < tx) && ((lm & Tmask) == Tmask);
                    const double *Mt = M + t * DS;
                    // the TG candidate operands M[t][cbase .. cbase+TG) are contiguous and 32-B aligned
                    // (DS % 4 == 0, cbase % TG == 0): NC/2 16-B LDS reads, broadcast across the lanes
                    // of the wave that share the group
                    double sc[TG];
#pragma unroll
                    for (int q = 0; q < (NC + 1) / 2; ++q) {
                        const double2 m = *reinterpret_cast<const double2 *>(Mt + cbase + 2 * q);
                        sc[2 * q] = m.x;
                        sc[2 * q + 1] = m.y;
                    }
                    double vT[DT], mT[DT];
                    double vv = 0.0, uv = 0.0;
#pragma unroll
                    for (int j = 0; j < DT; ++j) mT[j] = Mt[T[j]];
#pragma unroll
                    for (int i = 0; i < DT; ++i) {
                        double v = 0.0;
#pragma unroll
                        for (int j = 0; j <= i; ++j) v += Li[i][j] * mT[j];
                        vT[i] = v;
                        vv += v * v;
                        uv += uT[i] * v;
                    }
#pragma unroll
                    for (int i = 0; i < DT; ++i) projv[k][i] = PCG_TG_WC ? mT[i] : vT[i];   // w_c.M[T][y] or l_c.v_T
                    byy[k] = Md[t] - vv;
                    bxy[k] = Mx[t] - uv;
                    // live candidates: valid, c != y, and not deduplicated onto y (S in adj(y), y < x)
                    const unsigned tb = ((unsigned)(t - cbase) < (unsigned)TG) ? (1u << (t - cbase)) : 0u;
                    const unsigned skip = own ? (unsigned)(lm >> cbase) : 0u;
                    live[k] = inTset ? 0u : (vmask & ~tb & ~skip);
                    // TG independent chains, interleaved
#pragma unroll
                    for (int i = 0; i < DT; ++i)
#pragma unroll
                        for (int jj = 0; jj < NC; ++jj) sc[jj] -= lc[jj][i] * projv[k][i];
                    unsigned dp = 0;
#pragma unroll
                    for (int jj = 0; jj < NC; ++jj) {
                        const double vc = sc[jj] * rl[jj];
                        const double cyy = byy[k] - vc * vc;
                        const double cxy = bxy[k] - uc[jj] * vc;
                        const double num = cxy * cxy;
                        const double th = hc[jj] * cyy;
                        dp |= (unsigned)((num > th) & (fma(th, inv_hi2, -kg) > num)) << jj;
                    }
                    dep[k] = dp;
                }
#pragma unroll
                for (int k = 0; k < YU; ++k) {
                    const int t = tt[k];
                    tcount += __popc(live[k]);
                    const bool recy = (bool)((recm >> t) & 1u);   // recorded pair: every live test to the exact path
                    const unsigned rare = recy ? live[k] : (live[k] & ~(dep[k] & okm));
                    if (__ballot(rare != 0u)) {
                        if (rare) {
                            const double *Mt = M + t * DS;
                            const Mask lm = lmv[k];
#pragma unroll
                            for (int jj = 0; jj < TG; ++jj) {
                                if (!((rare >> jj) & 1u)) continue;
                                const int c = cbase + jj;
                                if (recy) {
                                    int sg[DM];
                                    sg[0] = nxs[c];
#pragma unroll
                                    for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
                                    push_deferred(a, x, nxs[t], sg, DM);
                                    continue;
                                }
                                // recompute the decision pieces for this c (rare path)
                                double s = Mt[c];
#pragma unroll
                                for (int i = 0; i < DT; ++i) s -= lc[jj][i] * projv[k][i];
                                const double vc = s * rl[jj];
                                const double cyy = byy[k] - vc * vc;
                                const double cxy = bxy[k] - uc[jj] * vc;
                                const double cxx = hc[jj] / a.hi2;
                                const bool ind = okc[jj] && (cxy * cxy < a.lo2 * cxx * cyy) && (cyy > 0.0) &&
                                                 (cxx * cyy - cxy * cxy > kg);
                                const Mask Smask = Tmask | ((Mask)1 << c);
                                if (ind) {
                                    ++indep;
                                    lmask_atomic_or<WIDE>(&uself[t], Smask);
                                    if (((lm & Smask) == Smask) && t >= tx) lmask_atomic_or<WIDE>(&uprop[t], Smask);
                                } else {
                                    int sg[DM];
                                    sg[0] = nxs[c];
#pragma unroll
                                    for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
                                    push_deferred(a, x, nxs[t], sg, DM);
                                }
                            }
                        }
                    }
                }
            }
        };
        if constexpr (TG == 4) {
        if (nmax >= 4) sweep(std::integral_constant<int, 4>{});
        else if (nmax == 3) sweep(std::integral_constant<int, 3>{});
        else if (nmax == 2) sweep(std::integral_constant<int, 2>{});
        else sweep(std::integral_constant<int, 1>{});
        } else if constexpr (TG == 6) {   // even counts: slots past a lane's candidates are not `live`
        if (nmax > 4) sweep(std::integral_constant<int, 6>{});
        else if (nmax > 2) sweep(std::integral_constant<int, 4>{});
        else sweep(std::integral_constant<int, 2>{});
        } else {
        if (nmax > 6) sweep(std::integral_constant<int, 8>{});
        else if (nmax > 4) sweep(std::integral_constant<int, 6>{});
        else if (nmax > 2) sweep(std::integral_constant<int, 4>{});
        else sweep(std::integral_constant<int, 2>{});
        }
        tests += tcount;
        tcount = 0;
    }
    __syncthreads();
    // flush unions (local bits -> global node bits) and removal flags
    for (int t = tid; t < D; t += bs) {
        const Mask us = uself[t], up = uprop[t];
        if (!(us | up)) continue;
        const int yg = nxs[t];
        a.rm[(int64_t)x * a.n + yg] = 1;
        a.rm[(int64_t)yg * a.n + x] = 1;
        for (int side = 0; side < 2; ++side) {
            const Mask bits = side ? up : us;
            if (!bits) continue;
            const int64_t slot = side ? (int64_t)a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x)
                                      : (int64_t)a.off[x] + t;
            unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + slot * a.W);
            for (int half = 0; half < (WIDE ? 2 : 1); ++half) {
                unsigned long long m = (unsigned long long)(bits >> (64 * half));
                while (m) {
                    const int b = 64 * half + __ffsll((long long)m) - 1;
                    const int gid = nxs[b];
                    atomicOr(&row[gid >> 6], 1ull << (gid & 63));
                    m &= m - 1;
                }
            }
        }
    }
    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// fp32-screened T-group sweep (threshold mode; the default form of k_level_lds_t).
//
// The block stages A~ = fp32(C) restricted to adj(x) (half the LDS of the fp64 form). Per
// lane task the setup (L_T, L_T^-1, u_T, l_c, 1/lambda_c, u_c, c_xx) runs in fp64 on A~ and
// is rounded to fp32 once; the y sweep runs in packed fp32 (v_pk_fma_f32: two candidates per
// instruction). A test is decided "dependent" in fp32 only when that is certain for the
// fp64 C: with nu_c = ||L_S^-1||_F (S = T + {c}),
//     E_c = KE * u32 * (1 + nu_c)^2,   u32 = 2^-24,
// bounds |c^ - c| for each of c_xx, c_yy, c_xy (the sweep's rounding plus the input rounding
// C -> A~ propagated through the Schur complement, whose regression weights are bounded by
// nu_c; tools/f32_screen_study.py measures max|err| / E_c ~ 2e-3 on config 5 with KE = 64).
// Certain dependence needs (|c_xy^| - E)^2 > hi2 (c_xx^ + E)(c_yy^ + E) and the fp64 paths'
// conditioning guard c_xx c_yy - c_xy^2 > tau / g on the true values; with 2E|c_xy| <=
// E (c_xy^2 / s + s) (s = a.s_amgm ~ |c_xy| at the threshold) both become linear in c_yy^:
//     alpha c_yy^ + beta  <  c_xy^2  <  gamma c_yy^ - kappa
// (per-candidate constants, every rounding of the fp32 evaluation folded in as a margin),
// evaluated as one compare |c_xy^2 - k1 - m c_yy^| < hh c_yy^ - k2. Every other test (the
// independent ones, the band around the threshold, unusable candidates: 6e-5 of depth 4's
// tests on config 5) takes the rare path, which evaluates it in fp64 from the C in HBM and
// decides it like the fp64 kernels (band -> exact path). Decisions are therefore the fp64
// kernels' decisions; only where the fp32 sweep is certain does it decide.
typedef float f2v __attribute__((ext_vector_type(2)));
#ifndef PCG_NODE_IMG
#define PCG_NODE_IMG 1    // compact node blocks as fp32 LDS images of k_level_lds_f (DMA-staged), else fp64 rows
#endif
// k_level_lds_f's staged region of a node of degree D: M (D rows of DS floats, columns >= D zero),
// the DS y records (2 mb bytes each) and nxs (DS ints). Narrow (mb = 8): rounded to 1 KB, the unit a
// wave's LDS-DMA instruction writes (64 lanes x 16 B), so a node image is copied whole
__host__ __device__ constexpr int tgf_image_bytes(int D, int mb) {
    return mb == 8 ? (4 * D * ((D + 3) & ~3) + (2 * mb + 4) * ((D + 3) & ~3) + 1023) & ~1023
                   : (4 * D * ((D + 3) & ~3) + (2 * mb + 4) * ((D + 3) & ~3) + 15) & ~15;
}
struct alignas(16) YRecN {       // k_level_lds_f (narrow): a y's {A~_yy, A~_xy} and local adjacency mask
    f2v md;
    unsigned long long lm;
};
constexpr double F32_U = 5.9604644775390625e-08;   // 2^-24
#ifndef PCG_F32_KE
#define PCG_F32_KE 32.0   // E = 2 KE u32 (1 + nu^2) >= KE u32 (1 + nu)^2, 1.75x DESIGN §4.1's 18 u32 (1 + nu)^2
#endif
#ifndef PCG_FORK_LATE
#define PCG_FORK_LATE 1   // the aux stream's fork wait after the main stream's first class launch (0: before it)
#endif
#ifndef PCG_TG_F32
#define PCG_TG_F32 0x18   // depths (bit 1 << d) whose T-group sweep is fp32-screened by default
#endif
#ifndef PCG_TGF_SGPR
#define PCG_TGF_SGPR 0x18 // k_level_lds_f depths (bit 1 << d) whose per-y bookkeeping is in wave lane masks
                          // (depth 3 joined in round 6 once the memo skips were counted per node: 0.52 -> 0.49 ms)
#endif
#ifndef PCG_KBRACKET
#define PCG_KBRACKET 0       // skeleton_once's depth / kernel brackets: 1 timing events (each one a ~6 us marker
                             // on the device's critical path), 0 device wall-clock stamps in kernels already queued
#endif
#ifndef PCG_LAST_XINL
#define PCG_LAST_XINL 1      // the last depth of a max_depth-bounded run exports on the handle's stream
#endif
#ifndef PCG_NBLK_T
#define PCG_NBLK_T 1         // compact node blocks built transposed (k_node_blocks_t) when C's row fits in LDS
#endif
#ifndef PCG_TGF_Y3FAST
#define PCG_TGF_Y3FAST 1     // per-lane y loop (YM 3): skip the dependence-bit packing when no lane needs it
#endif
#ifndef PCG_TGF_PREFETCH
#define PCG_TGF_PREFETCH 0  // k_level_lds_f depths (bit 1 << d) whose per-lane y loop prefetches row t + 1
                             // (depth 3: 0.703 vs 0.698 ms without it; measured no gain, off)
#endif
#ifndef PCG_TGF_ABL
#define PCG_TGF_ABL 0     // k_level_lds_f ablation builds for timing (tools/build_variant.sh): 1 = tasks without their
                          // sweeps, 2 = no tasks (staging and block overhead only); results are wrong
#endif
#ifndef PCG_TGF_ABL_D
#define PCG_TGF_ABL_D 4   // the depth the ablation applies to (the narrow class only)
#endif
#ifndef PCG_TGF_PROF
#define PCG_TGF_PROF 0    // diagnostic builds only: per-phase shader-clock cycles of k_level_lds_f at depth
                          // PCG_TGF_PROF (narrow class) summed into g_tgf_prof, printed per level to stderr
#endif
#ifndef PCG_TGF_BLKT
#define PCG_TGF_BLKT 0    // diagnostic builds only: per-block wall-clock (start, end, D, tasks) of k_level_lds_f at
                          // depth PCG_TGF_BLKT (narrow class: g_blkt, wide: g_blkw), summarised per level on stderr
#endif
#if PCG_TGF_BLKT
constexpr int BLKT_MAX = 32768;
__device__ unsigned long long g_blkt[BLKT_MAX][4];
__device__ unsigned long long g_blkw[4096][4];
#endif
#if PCG_TGF_PROF
__device__ unsigned long long g_tgf_prof[8];   // block, staging, setup, sweep cycles (per wave); tasks; y iters; waves
#endif
#ifndef PCG_TGF_PKV
#define PCG_TGF_PKV 1     // k_level_lds_f: v_T = L_T^-1 m_T with two of its rows as one packed chain (A/B: 0)
#endif
#ifndef PCG_TGF_SPLIT
#define PCG_TGF_SPLIT 1   // k_level_lds_f, one candidate window per wave: y outside the window without the
                          // dead-candidate selects (depth 4: 2.24 -> 2.09 ms once the rare-path values were opaque)
#endif
#ifndef PCG_TGF_SR
#define PCG_TGF_SR 4      // k_level_lds_f, narrow class gathering A~ from C: rows per wave with loads in flight
#endif
#ifndef PCG_NB3_TARGET
#define PCG_NB3_TARGET 4096   // narrow-class block target at depth 3 (level_begin_impl)
#endif
#ifndef PCG_NB4_TARGET
#define PCG_NB4_TARGET 16384  // ... at depth 4
#endif
#ifndef PCG_SCREEN_EXACT
#define PCG_SCREEN_EXACT 1   // the fp32 sweep's level end: screen + exact path in one launch (k_screen_exact)
#endif
#ifndef PCG_TGF_LPT
#define PCG_TGF_LPT 0x10  // depths (bit 1 << d) whose k_level_lds_f narrow class is dispatched largest degree first
                          // (LevelArgs::nord; config 5 depth 4: kernel 1.715-1.74 -> 1.69-1.70 ms A/B; depth 3
                          // measured 0.68-0.69 -> 0.69-0.72: its largest-degree blocks staged together first)
#endif
#ifndef PCG_TGF_NSKIP
#define PCG_TGF_NSKIP 1   // lane-mask sweep: the node's memo skips counted once in closed form, so a lane that
                          // owns y no longer takes the rare path just to subtract its skips
#endif
#ifndef PCG_TGF_PRIO
#define PCG_TGF_PRIO 0    // k_level_lds_f depths (bit 1 << d) whose staging runs at raised wave priority (s_setprio)
#endif
#ifndef PCG_MBF2
#define PCG_MBF2 4
#endif
#ifndef PCG_WIDE_MB
#define PCG_WIDE_MB 2     // k_level_lds_f, wide class: blocks per CU of the launch bounds
#endif
#ifndef PCG_MBF3
#define PCG_MBF3 4
#endif
#ifndef PCG_MBF4
#define PCG_MBF4 4
#endif
__host__ __device__ constexpr int tgf_minblocks(int DM) { return DM == 2 ? PCG_MBF2 : (DM == 3 ? PCG_MBF3 : PCG_MBF4); }


// (x, y | S) in fp64 from the C in HBM (Cholesky of C_SS, the fp64 kernels' guard and band):
// 0 dependent, 1 independent, 2 exact path
template <int DM>
__device__ int eval_test_global(const LevelArgs &a, int x, int y, const int *Sg) {
    // every entry is gathered before the factorisation uses any of them (one round of load
    // latency per test instead of one per Cholesky step)
    double Cs[DM][DM], Cx[DM], Cy[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) {
        Cs[j][j] = a.diag[Sg[j]];
#pragma unroll
        for (int i = j + 1; i < DM; ++i) Cs[i][j] = a.C[(int64_t)Sg[i] * a.ldc + Sg[j]];
        Cx[j] = a.C[(int64_t)Sg[j] * a.ldc + x];
        Cy[j] = a.C[(int64_t)Sg[j] * a.ldc + y];
    }
    const double cxy0 = a.C[(int64_t)x * a.ldc + y], dx = a.diag[x], dy = a.diag[y];
    double L[DM][DM], rinv[DM], u[DM], v[DM];
    double gmin = 1.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < DM; ++j) {
        double s = Cs[j][j];
#pragma unroll
        for (int q = 0; q < j; ++q) s -= L[j][q] * L[j][q];
        ok = ok && (s > 0.0);
        gmin = fmin(gmin, s);
        L[j][j] = sqrt(s);
        rinv[j] = 1.0 / L[j][j];
#pragma unroll
        for (int i = j + 1; i < DM; ++i) {
            double t = Cs[i][j];
#pragma unroll
            for (int q = 0; q < j; ++q) t -= L[i][q] * L[j][q];
            L[i][j] = t * rinv[j];
        }
    }
    double uu = 0.0, vv = 0.0, uv = 0.0;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        double tu = Cx[i], tv = Cy[i];
#pragma unroll
        for (int q = 0; q < i; ++q) {
            tu -= L[i][q] * u[q];
            tv -= L[i][q] * v[q];
        }
        u[i] = tu * rinv[i];
        v[i] = tv * rinv[i];
        uu += u[i] * u[i];
        vv += v[i] * v[i];
        uv += u[i] * v[i];
    }
    if (!ok) return 2;
    return decide<MODE_DECIDE>(a, cxy0 - uv, dx - uu, dy - vv, a.tau / gmin, nullptr);
}

template <int DM, bool WIDE, bool REC = false>
__global__ __launch_bounds__(256, WIDE ? PCG_WIDE_MB : tgf_minblocks(DM)) void k_level_lds_f(LevelArgs a) {
    using Mask = LMask<WIDE>;
    constexpr int DT = DM - 1;
    constexpr int TG = tg_of_depth(DM);
    constexpr int NP = TG / 2;                                    // candidate pairs
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int bs = blockDim.x;
    int64_t chunk;
    int x;
    if (!WIDE && a.nord) {   // largest degree first: block b -> (node position i, its chunk b - nps[i])
        const int b = (int)blockIdx.x;
        if (b >= a.nps[a.nm]) return;
        const int i = chunk_node32(a.nps, a.nm, b);
        x = a.nord[i];
        chunk = a.cpre[x] + (b - a.nps[i]);
    } else {
        chunk = a.chunk_lo + blockIdx.x;
        if (chunk >= a.cpre[a.n]) return;   // (defensive: launches are sized by the exact prefix)
        x = chunk_node(a.cpre, a.n, chunk);
    }
    const int D = a.deg[x];
    const int32_t *nxg = a.nbr + a.off[x];

#if PCG_TGF_BLKT
    const unsigned long long blkt0 = wall_clock64();
#endif
#if PCG_TGF_PROF
    constexpr bool PROF = !WIDE && !REC && DM == PCG_TGF_PROF;
    const unsigned long long prof_t0 = PROF ? clock64() : 0ull;
    unsigned long long prof_setup = 0, prof_sweep = 0, prof_tasks = 0, prof_y = 0, prof_stage = 0;
#endif
    const int DS = (D + 3) & ~3;                                  // padded length / row stride
    // the staged region first (a node image, tgf_image_bytes: one DMA copy when k_node_blocks_t
    // built it), then the union masks and two ints
    float *M = reinterpret_cast<float *>(smem);                   // D * DS (columns >= D zero)
    // one 16-byte (wide: 32-byte) record per y: {A~_yy, A~_xy, [pad,] local adjacency mask}, so the
    // sweep reads a y's wave-uniform operands with one LDS instruction
    constexpr int YS = WIDE ? 8 : 4;                              // floats per record
    float *Yr = M + D * DS;                                       // DS records, 16-B aligned
    int32_t *nxs = reinterpret_cast<int32_t *>(Yr + YS * DS);    // DS
    const int img_b = tgf_image_bytes(D, (int)sizeof(Mask));
    Mask *uself = reinterpret_cast<Mask *>(smem + img_b);         // DS
    Mask *uprop = uself + DS;                                     // DS
    int *s_tx = reinterpret_cast<int *>(uprop + DS);              // 1
    int *s_np = s_tx + 1;                                         // 1
    unsigned *btab = reinterpret_cast<unsigned *>(smem + a.lds_btab_off);   // C(c, i), c <= D, i <= DM
    unsigned *ppre = btab + (D + 1) * (DM + 1);                   // task prefix per (g, t0) pair
    unsigned short *pinfo = reinterpret_cast<unsigned short *>(ppre + tg_pairs(D, DM) + 1);  // g << 8 | t0

    constexpr bool PRIO = (PCG_TGF_PRIO >> DM) & 1;
    if (PRIO) __builtin_amdgcn_s_setprio(3);
    const bool img = !WIDE && a.img;
    if (img) {
        // the node's image (M, the y records, nxs) by LDS-DMA, 1 KB per wave instruction, every
        // piece in flight at once (no VGPR round trip, one memory latency); the binomial table's
        // loads below overlap it
        const unsigned char *src = reinterpret_cast<const unsigned char *>(a.cblk + a.bo[x]);
        const int lane = tid & 63, wv = tid >> 6, nwv = bs >> 6;
        for (int off = wv * 1024; off < img_b; off += nwv * 1024)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + off + lane * 16),
                                             (__attribute__((address_space(3))) void *)(smem + off), 16, 0, 0);
    } else {
        for (int i = tid; i < D; i += bs) nxs[i] = nxg[i];
    }
    for (int e = tid; e < (D + 1) * (DM + 1); e += bs) {
        const int c = e / (DM + 1), i = e - c * (DM + 1);
        btab[e] = (unsigned)pcg_binom(a.binom, c, i);
    }
    if (img) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's image pieces landed
    __syncthreads();
    if (img) {
    } else if (!WIDE && a.cblk) {   // this depth's compact node block (k_node_blocks): coalesced rows
        // a wave loads SR rows before storing any (SR loads in flight per lane, not one dependent
        // round trip per row; SR = 8 spilled 4 more VGPRs in the sweep); the masks a lane each
        constexpr int SR = 4;
        const double *cb = a.cblk + a.bo[x];
        const uint64_t *lk = a.lmk + a.off[x];
        const int L = D + 1;
        const int lane = tid & 63, wv = tid >> 6, nwv = bs >> 6;
        for (int t0 = wv * SR; t0 < D; t0 += nwv * SR) {
            double v[SR];
#pragma unroll
            for (int r = 0; r < SR; ++r) v[r] = lane < D ? cb[min(t0 + r, D - 1) * L + lane] : 0.0;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                const int t = t0 + r;
                if (t >= D) break;                   // wave-uniform
                if (lane < DS) M[t * DS + lane] = (float)v[r];
            }
        }
        for (int t = tid; t < D; t += bs) *reinterpret_cast<Mask *>(Yr + YS * t + (WIDE ? 4 : 2)) = (Mask)lk[t];
    } else if constexpr (WIDE) {   // (the row-batched form below measured slower for the 128-wide blocks)
        for (int e = tid; e < D * DS; e += bs) {
            const int t = e / DS, k = e - t * DS;
            M[e] = k < D ? (float)a.C[(int64_t)nxs[t] * a.ldc + nxs[k]] : 0.0f;
        }
        for (int t = tid >> 6; t < D; t += bs >> 6) {
            const uint64_t *ar = a.adj + (int64_t)nxs[t] * a.W;
            Mask m = 0;
            for (int k0 = 0; k0 < D; k0 += 64) {
                const int k = k0 + (tid & 63);
                const bool bit = k < D && ((ar[nxs[k] >> 6] >> (nxs[k] & 63)) & 1ull);
                m |= (Mask)__ballot(bit) << k0;
            }
            if ((tid & 63) == 0) *reinterpret_cast<Mask *>(Yr + YS * t + (WIDE ? 4 : 2)) = m;
        }
    } else {   // rows of A~ and of the local adjacency masks: a wave takes SR rows at a time, lane k
        // column k (its global id hoisted), so SR x (C entry, adjacency word) loads are in flight
        // per lane before the first is used; no index division
        constexpr int H = 1, SR = PCG_TGF_SR;
        const int lane = tid & 63, wv = tid >> 6, nwv = bs >> 6;
        int kg[H];
#pragma unroll
        for (int hh = 0; hh < H; ++hh) kg[hh] = lane + 64 * hh < D ? nxs[lane + 64 * hh] : -1;
        for (int t0 = wv * SR; t0 < D; t0 += nwv * SR) {
            float v[SR][H];
            uint64_t w[SR][H];
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                const int t = min(t0 + r, D - 1);
                const int rg = nxs[t];
#pragma unroll
                for (int hh = 0; hh < H; ++hh) {
                    const int k = kg[hh] < 0 ? 0 : kg[hh];
                    v[r][hh] = (float)a.C[(int64_t)rg * a.ldc + k];
                    w[r][hh] = a.adj[(int64_t)rg * a.W + (k >> 6)];
                }
            }
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                const int t = t0 + r;
                if (t >= D) break;                   // wave-uniform
                Mask m = 0;
#pragma unroll
                for (int hh = 0; hh < H; ++hh) {
                    const int k = lane + 64 * hh;
                    if (k < DS) M[t * DS + k] = kg[hh] >= 0 ? v[r][hh] : 0.0f;
                    const bool bit = kg[hh] >= 0 && ((w[r][hh] >> (kg[hh] & 63)) & 1ull);
                    m |= (Mask)__ballot(bit) << (64 * hh);
                }
                if (lane == 0) *reinterpret_cast<Mask *>(Yr + YS * t + (WIDE ? 4 : 2)) = m;
            }
        }
    }
    for (int t = tid; t < D; t += bs) {
        if (!img) {
            const int yg = nxs[t];
            Yr[YS * t] = (float)a.diag[yg];
            Yr[YS * t + 1] = (float)a.C[(int64_t)x * a.ldc + yg];
        }
        uself[t] = 0;
        uprop[t] = 0;
    }
    tgroup_pairs<DM, TG>(D, x, nxs, btab, ppre, pinfo, s_tx, s_np);
    // records (PCG_FLAG_RECORD): the recorded pairs (x, y) of this node, bit t; every live test of
    // such a y goes to the exact path (decided and recorded there, as in k_level_lds_t)
    __shared__ Mask s_recm;
    __shared__ ScreenEntry s_scr[PCG_SCREEN_BUF];   // this block's screen list entries (flush_screen_blk)
    __shared__ unsigned s_scr_n;
    __shared__ unsigned long long s_scr_base;
    if (tid == 0) s_scr_n = 0;
    if (tid < 64) {
        Mask rm_ = 0;
        if (REC && a.record)
            for (int k0 = 0; k0 < D; k0 += 64) {
                const int t = k0 + tid;
                const int yg = t < D ? nxs[t] : 0;
                rm_ |= (Mask)__ballot(t < D && rec_on(a, min(x, yg), max(x, yg))) << k0;
            }
        if (tid == 0) s_recm = rm_;
    }
    __syncthreads();
    const int tx = *s_tx;
    const int np = *s_np;
    const Mask recm = REC ? s_recm : (Mask)0;   // (threshold-mode builds: no record code in the sweep)
    if (PRIO) __builtin_amdgcn_s_setprio(0);
#if PCG_TGF_PROF
    if (PROF) prof_stage = clock64() - prof_t0;
#endif
    const double Cxx = (double)(float)a.diag[x];                  // A~_xx
    const uint64_t ntask = ppre[np];
    const uint64_t spl = (uint64_t)a.spl;
    const uint64_t r0 = (uint64_t)(chunk - a.cpre[x]) * (uint64_t)bs * spl;
    constexpr int ABL = (DM == PCG_TGF_ABL_D && !WIDE) ? PCG_TGF_ABL : 0;
    const uint64_t r1 = (ABL & 2) ? r0 : min(ntask, r0 + (uint64_t)bs * spl);   // (ablation: no tasks)
    unsigned long long tests = 0, indep = 0;
    constexpr bool SGK = (PCG_TGF_SGPR >> DM) & 1;
    if (SGK && PCG_TGF_NSKIP && chunk == a.cpre[x]) {
        // the lane-mask sweep counts every (y, S) of its tasks; the node's first chunk takes back
        // the memo skips in closed form: (x, y, S) with y < x (t < tx) and S within adj(y) is y's
        // test (SkeletonDiscovery.py's cache hit), C(|adj(x) & adj(y)|, d) of them per such y
        for (int t = tid; t < tx; t += bs) {
            const Mask lm = *reinterpret_cast<const Mask *>(Yr + YS * t + (WIDE ? 4 : 2));
            int c;
            if constexpr (WIDE) c = __popcll((unsigned long long)lm) + __popcll((unsigned long long)(lm >> 64));
            else c = __popcll(lm);
            tests -= btab[c * (DM + 1) + DM];
        }
    }
    unsigned tcount = 0;
    const unsigned long long lanebit = 1ull << (tid & 63);
    const float inv_sf = (float)a.inv_s;                          // rounding covered by the check's margins
    const float lo2f = (float)(a.lo2 * (1.0 - 4.0 * F32_U));     // <= lo2
    const float hi2f = (float)(a.hi2 * (1.0 + 4.0 * F32_U));     // >= hi2
    const f2v s2 = {(float)(a.s_amgm * (1.0 + 4.0 * F32_U)), (float)(a.s_amgm * (1.0 + 4.0 * F32_U))};   // >= s
    // constant factors of the candidate setup's bounds (each rounded in its safe direction)
    constexpr double RUd = 1.0 + 16.0 * F32_U;
    const f2v ke2 = {(float)(2.0 * PCG_F32_KE * F32_U * RUd), (float)(2.0 * PCG_F32_KE * F32_U * RUd)};
    const f2v ke2u = {(float)((2.0 * PCG_F32_KE + 1.0) * F32_U * RUd), (float)((2.0 * PCG_F32_KE + 1.0) * F32_U * RUd)};
    const f2v inv_su = {(float)(a.inv_s * RUd), (float)(a.inv_s * RUd)};
    const f2v tauu = {(float)(a.tau * RUd * RUd), (float)(a.tau * RUd * RUd)};
    const f2v two_u = {(float)(2.0 * (1.0 + 8.0 * F32_U) * RUd), (float)(2.0 * (1.0 + 8.0 * F32_U) * RUd)};
    const f2v one_u = {(float)((1.0 + 8.0 * F32_U) * RUd), (float)((1.0 + 8.0 * F32_U) * RUd)};
    const f2v s2u = s2 + (float)F32_U;

    int lq_prev = 0;
    for (uint64_t task = r0 + tid; task < r1; task += bs) {
#if PCG_TGF_PROF
        const unsigned long long prof_a = PROF ? clock64() : 0ull;
        if (PROF) { ++prof_tasks; prof_y += D; }
#endif
        int lq = tg_pair_search<(PCG_TG_GALLOP & 2) != 0>(ppre, np, (unsigned)task, lq_prev);
        lq_prev = lq;
        const int info = pinfo[lq];
        const int cbase = (info >> 8) * TG;
        int T[DT];
        T[0] = info & 255;
        {
            unsigned rr = (unsigned)(task - ppre[lq]);
            int hi_ = D - T[0] - 1;
#pragma unroll
            for (int ii = DT - 2; ii >= 0; --ii) {
                const int lo_ = colex_elem(ii, rr, hi_, btab, DM + 1);
                T[ii + 1] = lo_;
                rr -= btab[lo_ * (DM + 1) + ii + 1];
                hi_ = lo_;
            }
#pragma unroll
            for (int ii = 1; ii < DT; ++ii) T[ii] += T[0] + 1;
        }
        const int nval = min(T[0] - cbase, TG);
        int nmax_ = 1;
#pragma unroll
        for (int k = 2; k <= TG; ++k) nmax_ += (__ballot(nval >= k) != 0);
        const int nmax = __builtin_amdgcn_readfirstlane(nmax_);
        Mask Tmask = 0;
#pragma unroll
        for (int i = 0; i < DT; ++i) Tmask |= (Mask)1 << T[i];
        // T setup in fp64 on A~ (reciprocal square roots: fp32 estimate + one Newton step,
        // relative error ~1e-14, far inside the E bound)
        double L[DT][DT], Li[DT][DT], uT[DT];
        bool okT = true;
        double gT = 1.0;
#pragma unroll
        for (int j = 0; j < DT; ++j) {
            double s = M[T[j] * DS + T[j]];
#pragma unroll
            for (int q = 0; q < j; ++q) s -= L[j][q] * L[j][q];
            okT = okT && (s > 0.0);
            gT = fmin(gT, s);
            const double r = rsq_nr(s);
#pragma unroll
            for (int i = j + 1; i < DT; ++i) {
                double t = M[T[i] * DS + T[j]];
#pragma unroll
                for (int q = 0; q < j; ++q) t -= L[i][q] * L[j][q];
                L[i][j] = t * r;
            }
            Li[j][j] = r;
        }
#pragma unroll
        for (int i = 1; i < DT; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double t = 0.0;
#pragma unroll
                for (int q = j; q < i; ++q) t += L[i][q] * Li[q][j];
                Li[i][j] = -t * Li[i][i];
            }
        double uuT = 0.0, liF = 0.0;
#pragma unroll
        for (int i = 0; i < DT; ++i) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                t += Li[i][j] * (double)Yr[YS * T[j] + 1];
                liF += Li[i][j] * Li[i][j];
            }
            uT[i] = t;
            uuT += t * t;
        }
        const double cx0 = Cxx - uuT;
        float Lif[DT][DT], uTf[DT];
#pragma unroll
        for (int i = 0; i < DT; ++i) {
            uTf[i] = (float)uT[i];
#pragma unroll
            for (int j = 0; j <= i; ++j) Lif[i][j] = (float)Li[i][j];
        }
        // candidate constants, two candidates per packed register. The candidate's Cholesky row
        // (l_c, 1/lambda, u_c, c_xx) is fp64; the decision constants are bounds built from it in
        // packed fp32, every rounding covered by a (1 +- 16 u32) factor in the safe direction
        f2v lcp[NP][DT], rlp[NP], ucp[NP], mp[NP], hhp[NP], k1p[NP], k2p[NP];
        bool okc[TG];
        const float liFf = (float)liF;
        const float gTf = (float)gT * (1.0f - (float)(4.0 * F32_U));
        // phase 1: every candidate's Cholesky row in fp64, rounded to fp32 as soon as it is formed
        // (the fp64 T state dies here). Phase 2 below builds the decision bounds from the fp32
        // values only. The scheduling barriers keep the compiler from interleaving the phases
        // (which held the fp64 state and all the candidate constants live at once: 173 VGPRs,
        // spilled at the 128 of four waves per SIMD).
        f2v cxp[NP], l2p[NP], r2p[NP], llp[NP];
        bool vldc[TG];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int jj = 2 * q + h;
#pragma unroll
                for (int i = 0; i < DT; ++i) lcp[q][i][h] = 0.0f;
                rlp[q][h] = 0.0f;
                ucp[q][h] = 0.0f;
                cxp[q][h] = l2p[q][h] = r2p[q][h] = llp[q][h] = 0.0f;
                vldc[jj] = false;
                if (jj < nmax) {                      // wave-uniform
                    const int c = cbase + jj;
                    const bool valid = c < T[0];
                    const int cc = valid ? c : 0;
                    double lc[DT], ll = 0.0, lu = 0.0;
#pragma unroll
                    for (int i = 0; i < DT; ++i) {
                        double t = 0.0;
#pragma unroll
                        for (int j = 0; j <= i; ++j) t += Li[i][j] * (double)M[T[j] * DS + cc];
                        lc[i] = t;
                        ll += t * t;
                        lu += t * uT[i];
                    }
                    const double lam2 = (double)M[cc * DS + cc] - ll;
                    const double r = rsq_nr(lam2);
                    const double u = ((double)Yr[YS * cc + 1] - lu) * r;
                    const double cxx = cx0 - u * u;
#pragma unroll
                    for (int i = 0; i < DT; ++i) lcp[q][i][h] = (float)lc[i];
                    rlp[q][h] = (float)r;
                    ucp[q][h] = (float)u;
                    cxp[q][h] = (float)cxx;
                    l2p[q][h] = (float)lam2;
                    r2p[q][h] = (float)(r * r);
                    llp[q][h] = (float)ll;
                    vldc[jj] = valid && okT && (lam2 > 0.0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // phase 2: the decision bounds, two candidates per packed register
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const f2v cxf = cxp[q], l2f = l2p[q], r2f = r2p[q], llf = llp[q];
            // E >= KE u32 (1 + nu)^2 + |fp32(c_xx) - c_xx|, nu^2 <= liF + (liF |l_c|^2 + 1) r^2.
            // Each bound below has fewer than 16 roundings between its inputs (themselves bounds
            // in the right direction) and its single RU / RD factor.
            constexpr float U = (float)F32_U;
            constexpr float RU = 1.0f + 16.0f * U, RD = 1.0f - 16.0f * U, U8 = 8.0f * U;
            const f2v one = {1.0f, 1.0f};
            const f2v liF2 = {liFf, liFf};
            const f2v nu2 = __builtin_elementwise_fma(__builtin_elementwise_fma(liF2, llf, one), r2f, liF2);
            const f2v E = __builtin_elementwise_fma(nu2, ke2, ke2u);  // (KE2 (1 + nu^2) + u) RU
            const f2v te = E * inv_su;                                // >= E / s
            const f2v gT2 = {gTf, gTf};
            const f2v g = (__builtin_elementwise_min(gT2, l2f) - (E + 2.0f * U)) * RD;   // <= smallest pivot^2 of C_SS
            const f2v cmE = (cxf - E) * RD;                           // <= c_xx - E
            const f2v rg = {__builtin_amdgcn_rcpf(g[0]), __builtin_amdgcn_rcpf(g[1])};
            const f2v kg = tauu * rg;                                 // >= tau / g
            const f2v hx = hi2f * (cxf + E);                          // hi2 (c_xx + E), RU in f1
            const f2v f1 = __builtin_elementwise_fma(te, two_u, one_u);   // (1 + 2 te)(1 + u8) RU
            const f2v al = hx * f1;
            const f2v be = E * (hx + s2) * f1;
            const f2v ga = (cmE - cmE * te) * ((1.0f - U8) * RD);
            const f2v ka = __builtin_elementwise_fma(E, cxf + s2u, kg) * ((1.0f + U8) * RU);  // E (c_xx + s) + kg
            const f2v mm = 0.5f * (al + ga);
            const f2v hw = __builtin_elementwise_fma(-2.0f * U8 * one, ga, 0.5f * (ga - al));
            const f2v kk1 = 0.5f * (be - ka);
            const f2v kk2 = (be + ka) * (0.5f * (1.0f + U8));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const bool ok = vldc[2 * q + h] && (te[h] <= 0.5f) && (cmE[h] > 0.0f) && (g[h] > 0.0f) && (ga[h] > al[h]);
                okc[2 * q + h] = ok;
                // an unusable candidate always passes the sweep's compare (|c_xy^2| < 3e38): its
                // lanes take the rare path through `notok`, whose per-candidate check reads okc
                mp[q][h] = ok ? mm[h] : 0.0f;
                hhp[q][h] = ok ? hw[h] : 0.0f;
                k1p[q][h] = ok ? kk1[h] : 0.0f;
                k2p[q][h] = ok ? kk2[h] : -3.0e38f;
            }
            // opaque: the rare path must read these registers, not keep (spill) the unselected values
            asm volatile("" : "+v"(mp[q]), "+v"(hhp[q]), "+v"(k1p[q]), "+v"(k2p[q]));
        }
        const int cend = min(T[0], cbase + TG);
        unsigned okm = 0;
#pragma unroll
        for (int jj = 0; jj < TG; ++jj) okm |= (unsigned)okc[jj] << jj;
        const unsigned vmask = (1u << (cend - cbase)) - 1u;
        // lane-mask sweep (closed-form test count) at the depths whose bit is set, else per-lane bits
        constexpr bool SG = (PCG_TGF_SGPR >> DM) & 1;
        unsigned long long okv[TG];
        if (SG) tcount += (unsigned)(nval * (D - DT - 1));
#pragma unroll
        for (int jj = 0; jj < TG; ++jj) okv[jj] = __builtin_amdgcn_ballot_w64(okc[jj]);
        const unsigned long long notok = __builtin_amdgcn_ballot_w64((vmask & ~okm) != 0u);
        // LDS byte offsets of the lane's candidate window and T columns within a row of A~
        const unsigned cofs = (unsigned)cbase * 4u;
        unsigned tofs[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) tofs[j] = (unsigned)T[j] * 4u;
        const int cb0 = __builtin_amdgcn_readfirstlane(cbase);
        const bool uni = __builtin_amdgcn_ballot_w64(cbase != cb0) == 0ull;
#if PCG_TGF_PROF
        const unsigned long long prof_b = PROF ? clock64() : 0ull;
        if (PROF) prof_setup += prof_b - prof_a;
#endif

        // a live test of candidate jj at y = t that the sweep's check did not make certain:
        // certain independence in fp32 (recomputed) or the fp64 screen list
        auto rare_cand = [&](int jj, int t, const float *Mt, const float *vT, float byy, float bxy, Mask lm) {
            const int q = jj >> 1, h = jj & 1;
            int c = cbase + jj;
            asm volatile("" : "+v"(c));      // no per-candidate masks / ids hoisted into the hot loop
            if (okc[jj]) {   // the sweep's check for this candidate, recomputed
                float s_ = Mt[c];
#pragma unroll
                for (int i = 0; i < DT; ++i) s_ = fmaf(-lcp[q][i][h], vT[i], s_);
                const float vc = s_ * rlp[q][h];
                const float cyy = fmaf(-vc, vc, byy);
                const float cxy = fmaf(-ucp[q][h], vc, bxy);
                const float w = fmaf(-mp[q][h], cyy, fmaf(cxy, cxy, -k1p[q][h]));
                if (__builtin_fabsf(w) < fmaf(hhp[q][h], cyy, -k2p[q][h])) return;
                // certain independence, with bounds recovered from the candidate's constants:
                // m + hh <= c_xx - E, (k1 + k2) / s >= E, k2 - k1 >= kappa >= tau / g (see the
                // setup); each fp32 rounding below is covered by a (1 +- 8 u32) factor:
                //   (|c_xy^| + E)^2 < lo2 (c_xx^ - E)(c_yy^ - E)            (r^2 < lo2)
                //   (c_xx^ - E)(c_yy^ - E) - (|c_xy^| + E)^2 > tau / g       (the guard)
                // (the opaque copies keep the compiler from hoisting these per-candidate values
                // out of the y loop, where they would only be spilled)
                constexpr float U8 = (float)(8.0 * F32_U);
                float m_ = mp[q][h], hh_ = hhp[q][h], k1_ = k1p[q][h], k2_ = k2p[q][h];
                asm volatile("" : "+v"(m_), "+v"(hh_), "+v"(k1_), "+v"(k2_));
                const float Alb = (m_ + hh_) * (1.0f - U8);
                const float Eub = (k1_ + k2_) * inv_sf * (1.0f + U8);
                const float kgub = (k2_ - k1_) * (1.0f + U8);
                const float ay = (cyy - Eub) * (1.0f - U8);
                const float ax = (__builtin_fabsf(cxy) + Eub) * (1.0f + U8);
                if (ay > 0.0f && ax * ax * (1.0f + U8) < lo2f * Alb * ay &&
                    fmaf(ax, ax, kgub) * (1.0f + U8) < Alb * ay) {
                    const Mask Smask = Tmask | ((Mask)1 << c);
                    ++indep;
                    lmask_atomic_or<WIDE>(&uself[t], Smask);
                    if (((lm & Smask) == Smask) && t >= tx) lmask_atomic_or<WIDE>(&uprop[t], Smask);
                    return;
                }
            }
            int sg[DM];
            sg[0] = nxs[c];
#pragma unroll
            for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
            push_screen_blk(a, s_scr, &s_scr_n, x, nxs[t], sg, DM);
        };
        // a recorded pair's live test: to the exact path
        auto push_rec = [&](int jj, int t) {
            int sg[DM];
            sg[0] = nxs[cbase + jj];
#pragma unroll
            for (int i = 0; i < DT; ++i) sg[i + 1] = nxs[T[i]];
            push_deferred(a, x, nxs[t], sg, DM);
        };
        auto sweep = [&](auto nc_tag) {
            constexpr int NC = decltype(nc_tag)::value;
            constexpr int NQ = NC / 2;
            // YM 1: one candidate window per wave (lane masks, y = candidate masked by index);
            // 2: windows differ (lane masks, such lanes to the rare path); 3: per-lane live and
            // dependence bits (the depths where dedup skips are common: a lane that owns y is
            // not sent down the rare path just to count its skips)
            // the LDS operands of one y (row t of A~): the candidates' entries, the T entries, the
            // {A~_yy, A~_xy} pair and the local adjacency mask. Loaded apart from their use so the
            // y loop can issue row t + 1's reads before row t's arithmetic (PCG_TGF_PREFETCH)
            struct YPre {
                f2v sc[NQ];
                float mT[DT];
                f2v md;
                Mask lm;
            };
            auto yload = [&](int t) {
                YPre p;
                // byte addresses: the row's (wave-uniform) base plus each lane's hoisted column
                // offsets (one v_add per operand instead of a shift-and-add of the column index)
                const char *Mb = reinterpret_cast<const char *>(M) + (unsigned)(t * DS) * 4u;
#pragma unroll
                for (int q = 0; q < NQ; ++q) p.sc[q] = *reinterpret_cast<const f2v *>(Mb + cofs + 8u * q);
#pragma unroll
                for (int j = 0; j < DT; ++j) p.mT[j] = *reinterpret_cast<const float *>(Mb + tofs[j]);
                if constexpr (!WIDE) {   // the y record in one 16-byte read
                    const YRecN r = *reinterpret_cast<const YRecN *>(Yr + 4 * t);
                    p.md = r.md;
                    p.lm = r.lm;
                } else {
                    p.md = *reinterpret_cast<const f2v *>(Yr + YS * t);
                    p.lm = *reinterpret_cast<const Mask *>(Yr + YS * t + 4);
                }
                return p;
            };
            auto ystep = [&](int t, auto ym_tag, const YPre &pre) {
                constexpr int YM = decltype(ym_tag)::value;
                const float *Mt = M + t * DS;
                f2v sc[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) sc[q] = pre.sc[q];
                float vT[DT], mT[DT];
#pragma unroll
                for (int j = 0; j < DT; ++j) mT[j] = pre.mT[j];
                // (|v_T|^2, u_T.v_T) accumulated as one packed pair (vu[i] = {v_i, u_i}) onto
                // -{A~_yy, A~_xy}: acc = -{b_yy, b_xy} with no separate subtraction (three roundings
                // of partial sums <= 2 in magnitude instead of k <= 1 plus one: the b_yy / b_xy error
                // terms grow by 2u, inside DESIGN §4.1's 14 u (1 + nu)^2 and 9 u (1 + nu)^2)
                f2v acc = -pre.md;
                if constexpr (PCG_TGF_PKV && DT == 3) {
                    // v_1 and v_2 as one packed chain (the same roundings in the same order as the
                    // scalar chains: L_i0 m_0, + L_i1 m_1, + L_i2 m_2)
                    const f2v l0 = {Lif[1][0], Lif[2][0]}, l1 = {Lif[1][1], Lif[2][1]};
                    const f2v m0 = {mT[0], mT[0]}, m1 = {mT[1], mT[1]};
                    const f2v p = __builtin_elementwise_fma(l1, m1, l0 * m0);
                    vT[0] = Lif[0][0] * mT[0];
                    vT[1] = p[0];
                    vT[2] = fmaf(Lif[2][2], mT[2], p[1]);
                } else if constexpr (PCG_TGF_PKV && DT == 2) {
                    const f2v l0 = {Lif[0][0], Lif[1][0]}, m0 = {mT[0], mT[0]};
                    const f2v p = l0 * m0;
                    vT[0] = p[0];
                    vT[1] = fmaf(Lif[1][1], mT[1], p[1]);
                } else {
#pragma unroll
                    for (int i = 0; i < DT; ++i) {
                        float v = 0.0f;
#pragma unroll
                        for (int j = 0; j <= i; ++j) v = fmaf(Lif[i][j], mT[j], v);
                        vT[i] = v;
                    }
                }
#pragma unroll
                for (int i = 0; i < DT; ++i) {
                    const f2v vu = {vT[i], uTf[i]}, vb = {vT[i], vT[i]};
                    acc = __builtin_elementwise_fma(vu, vb, acc);
                }
                const float byy = -acc[0];
                const float bxy = -acc[1];
#pragma unroll
                for (int i = 0; i < DT; ++i) {
                    const f2v vb = {vT[i], vT[i]};
#pragma unroll
                    for (int q = 0; q < NQ; ++q) sc[q] = __builtin_elementwise_fma(-lcp[q][i], vb, sc[q]);
                }
                const f2v byy2 = {byy, byy}, bxy2 = {bxy, bxy};
                const Mask lm = pre.lm;
                if constexpr (YM == 3) {
                    // dall: lanes whose every candidate is certainly dependent (lane masks, combined
                    // on the scalar unit); the per-lane dependence bits are only built when some
                    // lane has a candidate that is not, or an unusable one (notok)
                    f2v wq[NQ], hq[NQ];
                    unsigned long long dall = ~0ull;
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const f2v vc = sc[q] * rlp[q];
                        const f2v cyy = __builtin_elementwise_fma(-vc, vc, byy2);
                        const f2v cxy = __builtin_elementwise_fma(-ucp[q], vc, bxy2);
                        const f2v nm = __builtin_elementwise_fma(cxy, cxy, -k1p[q]);
                        wq[q] = __builtin_elementwise_fma(-mp[q], cyy, nm);
                        hq[q] = __builtin_elementwise_fma(hhp[q], cyy, -k2p[q]);
                        if (PCG_TGF_Y3FAST)
                            dall &= __builtin_amdgcn_ballot_w64(__builtin_fabsf(wq[q][0]) < hq[q][0]) &
                                    __builtin_amdgcn_ballot_w64(__builtin_fabsf(wq[q][1]) < hq[q][1]);
                    }
                    const bool inTset = (bool)((Tmask >> t) & 1u);
                    const bool own = (t < tx) && ((lm & Tmask) == Tmask);
                    const unsigned tb = ((unsigned)(t - cbase) < (unsigned)TG) ? (1u << (t - cbase)) : 0u;
                    const unsigned skip = own ? (unsigned)(lm >> cbase) : 0u;
                    const unsigned live = inTset ? 0u : (vmask & ~tb & ~skip);
                    tcount += __popc(live);
                    const bool recy = REC && (bool)((recm >> t) & 1u);     // wave-uniform
                    // a lane in dall with every valid candidate usable has rare = 0 (dp & okm covers
                    // every live bit): the wave skips the bit packing when no lane is outside that
                    if (PCG_TGF_Y3FAST && !recy && !((~dall | notok) & __builtin_amdgcn_read_exec())) return;
                    unsigned dp = 0;
#pragma unroll
                    for (int q = 0; q < NQ; ++q)
                        dp |= ((unsigned)(__builtin_fabsf(wq[q][0]) < hq[q][0]) << (2 * q)) |
                              ((unsigned)(__builtin_fabsf(wq[q][1]) < hq[q][1]) << (2 * q + 1));
                    const unsigned rare = recy ? live : (live & ~(dp & okm));
                    if (__builtin_amdgcn_ballot_w64(rare != 0u)) {
                        if (rare) {
#pragma unroll
                            for (int jj = 0; jj < TG; ++jj)
                                if ((rare >> jj) & 1u) {
                                    if (recy) push_rec(jj, t);
                                    else rare_cand(jj, t, Mt, vT, byy, bxy, lm);
                                }
                        }
                    }
                    return;
                } else {
                // dall = lanes where every candidate is certainly dependent (unusable ones always
                // pass, see the setup; YM 1 skips the candidate that is y)
                const int jdead = YM == 1 ? t - cb0 : -1;
                unsigned long long dall = ~0ull;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const f2v vc = sc[q] * rlp[q];
                    const f2v cyy = __builtin_elementwise_fma(-vc, vc, byy2);
                    const f2v cxy = __builtin_elementwise_fma(-ucp[q], vc, bxy2);
                    const f2v nm = __builtin_elementwise_fma(cxy, cxy, -k1p[q]);
                    const f2v w = __builtin_elementwise_fma(-mp[q], cyy, nm);
                    const f2v hh = __builtin_elementwise_fma(hhp[q], cyy, -k2p[q]);
                    const unsigned long long d0 = __builtin_amdgcn_ballot_w64(__builtin_fabsf(w[0]) < hh[0]);
                    const unsigned long long d1 = __builtin_amdgcn_ballot_w64(__builtin_fabsf(w[1]) < hh[1]);
                    if (YM == 1) {
                        dall &= 2 * q == jdead ? ~0ull : d0;
                        dall &= 2 * q + 1 == jdead ? ~0ull : d1;
                    } else {
                        dall &= d0 & d1;
                    }
                }
                const unsigned long long inT = __builtin_amdgcn_ballot_w64((bool)((Tmask >> t) & 1u));
                const bool recy = REC && (bool)((recm >> t) & 1u);     // wave-uniform
                unsigned long long rarel = ((~dall & __builtin_amdgcn_read_exec()) | notok) & ~inT;
                if (YM == 2) rarel |= __builtin_amdgcn_ballot_w64((unsigned)(t - cbase) < (unsigned)nval);
                if (!PCG_TGF_NSKIP && t < tx) rarel |= __builtin_amdgcn_ballot_w64((lm & Tmask) == Tmask) & ~inT;
                if (recy) rarel = __builtin_amdgcn_read_exec() & ~inT;
                if (!rarel) return;
                if (!(rarel & lanebit)) return;
                // rare path (this lane): live set and dedup skips as in k_level_lds_t
                const bool own = (t < tx) && ((lm & Tmask) == Tmask);
                const unsigned tb = ((unsigned)(t - cbase) < (unsigned)TG) ? (1u << (t - cbase)) : 0u;
                const unsigned skip = own ? (unsigned)(lm >> cbase) : 0u;
                if ((Tmask >> t) & 1u) return;
                const unsigned live = vmask & ~tb & ~skip;
                if (!PCG_TGF_NSKIP) tcount -= __popc(vmask & ~tb & skip);
#pragma unroll
                for (int jj = 0; jj < TG; ++jj)
                    if ((live >> jj) & 1u) {
                        if (recy) push_rec(jj, t);
                        else rare_cand(jj, t, Mt, vT, byy, bxy, lm);
                    }
                }
            };
            using Y0 = std::integral_constant<int, 0>;
            using Y1 = std::integral_constant<int, 1>;
            using Y2 = std::integral_constant<int, 2>;
            using Y3 = std::integral_constant<int, 3>;
            if (!SG) {
                if constexpr ((PCG_TGF_PREFETCH >> DM) & 1) {
                    // software-pipelined: row t + 1's LDS reads are in flight during row t's
                    // arithmetic (the loop was LDS-latency bound: s_waitcnt right after the reads)
                    YPre cur = yload(0);
                    for (int t = 0; t < D; ++t) {
                        const YPre nxt = yload(t + 1 < D ? t + 1 : t);
                        ystep(t, Y3{}, cur);
                        cur = nxt;
                    }
                } else {
                    for (int t = 0; t < D; ++t) ystep(t, Y3{}, yload(t));
                }
            } else if (uni && PCG_TGF_SPLIT) {
                // the window [cb0, cb0 + NC) is the only place a candidate can be y: outside it the
                // check needs no per-candidate "c == y" selects (YM 0)
                const int w0 = min(cb0, D), w1 = min(cb0 + NC, D);
                for (int t = 0; t < w0; ++t) ystep(t, Y0{}, yload(t));
                for (int t = w0; t < w1; ++t) ystep(t, Y1{}, yload(t));
                for (int t = w1; t < D; ++t) ystep(t, Y0{}, yload(t));
            } else if (uni) {
                for (int t = 0; t < D; ++t) ystep(t, Y1{}, yload(t));
            } else {
                for (int t = 0; t < D; ++t) ystep(t, Y2{}, yload(t));
            }
        };
        if constexpr (ABL & 1) {
            // ablation timing only (wrong results): the task's decode + setup without its sweep;
            // every setup output feeds one dummy so none of it is dead code
            float z = (float)okm + (float)tx + uTf[0] + Lif[DT - 1][0];
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                z += mp[q][0] + hhp[q][1] + k1p[q][0] + k2p[q][1] + rlp[q][0] + ucp[q][1];
#pragma unroll
                for (int i = 0; i < DT; ++i) z += lcp[q][i][0] + lcp[q][i][1];
            }
            tests += (z == 1234.5f) ? 1u : 0u;
            continue;
        }
        if constexpr (TG == 4) {
            if (nmax > 2) sweep(std::integral_constant<int, 4>{});
            else sweep(std::integral_constant<int, 2>{});
        } else if constexpr (TG == 6) {
            if (nmax > 4) sweep(std::integral_constant<int, 6>{});
            else if (nmax > 2) sweep(std::integral_constant<int, 4>{});
            else sweep(std::integral_constant<int, 2>{});
        } else {
            if (nmax > 6) sweep(std::integral_constant<int, 8>{});
            else if (nmax > 4) sweep(std::integral_constant<int, 6>{});
            else if (nmax > 2) sweep(std::integral_constant<int, 4>{});
            else sweep(std::integral_constant<int, 2>{});
        }
        tests += tcount;
        tcount = 0;
#if PCG_TGF_PROF
        if (PROF) prof_sweep += clock64() - prof_b;
#endif
    }
#if PCG_TGF_PROF
    if (PROF && (tid & 63) == 0) {
        atomicAdd(&g_tgf_prof[1], prof_stage);
        atomicAdd(&g_tgf_prof[2], prof_setup);
        atomicAdd(&g_tgf_prof[3], prof_sweep);
        atomicAdd(&g_tgf_prof[4], prof_tasks);
        atomicAdd(&g_tgf_prof[5], prof_y);
        atomicAdd(&g_tgf_prof[6], 1ull);
    }
#endif
    __syncthreads();
    flush_screen_blk(a, s_scr, &s_scr_n, &s_scr_base);
#if PCG_TGF_PROF
    if (PROF && tid == 0) atomicAdd(&g_tgf_prof[0], clock64() - prof_t0);
#endif
    for (int t = tid; t < D; t += bs) {
        const Mask us = uself[t], up = uprop[t];
        if (!(us | up)) continue;
        const int yg = nxs[t];
        a.rm[(int64_t)x * a.n + yg] = 1;
        a.rm[(int64_t)yg * a.n + x] = 1;
        for (int side = 0; side < 2; ++side) {
            const Mask bits = side ? up : us;
            if (!bits) continue;
            const int64_t slot = side ? (int64_t)a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x)
                                      : (int64_t)a.off[x] + t;
            unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + slot * a.W);
            for (int half = 0; half < (WIDE ? 2 : 1); ++half) {
                unsigned long long m = (unsigned long long)(bits >> (64 * half));
                while (m) {
                    const int b = 64 * half + __ffsll((long long)m) - 1;
                    const int gid = nxs[b];
                    atomicOr(&row[gid >> 6], 1ull << (gid & 63));
                    m &= m - 1;
                }
            }
        }
    }
    block_flush_counts(a.ctr, tests, indep);
#if PCG_TGF_BLKT
    if (DM == PCG_TGF_BLKT && !REC && tid == 0) {
        unsigned long long *e = WIDE ? (blockIdx.x < 4096 ? g_blkw[blockIdx.x] : nullptr)
                                     : (blockIdx.x < BLKT_MAX ? g_blkt[blockIdx.x] : nullptr);
        if (e) { e[0] = blkt0; e[1] = wall_clock64(); e[2] = (unsigned long long)D; e[3] = r1 - r0; }
    }
#endif
}

// The fp64 screen of the tests the fp32 sweep handed over (one lane per test, after the level
// kernels, before k_exact): decided like the fp64 kernels; independence writes the removal
// flags and both sides' unions as k_exact does, the band goes on to the exact path.
template <int DM, typename Band>
__device__ __forceinline__ void screen_lanes(const LevelArgs &a, int blk, int nblk, Band band) {
    const unsigned long long pushed = *(volatile const unsigned long long *)&a.ctr->screened;
    const int64_t count = (int64_t)min((unsigned long long)a.scr_cap, pushed);
    if (blk == 0 && threadIdx.x == 0 && (int64_t)pushed > a.scr_cap)
        a.rm[(int64_t)a.n * a.n] = 1;      // overflow: every rank reruns (status byte 0)
    unsigned long long nindep = 0;
    const int64_t stride = (int64_t)nblk * blockDim.x;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < count; i += stride) {
        const ScreenEntry e = a.screen[i];
        const int x = e.x, y = e.y;
        int sg[DM];
#pragma unroll
        for (int q = 0; q < DM; ++q) sg[q] = e.s[q];
        const int dec = eval_test_global<DM>(a, x, y, sg);
        if (dec == 2) {
            band(x, y, sg);
        } else if (dec == 1) {
            ++nindep;
            a.rm[(int64_t)x * a.n + y] = 1;
            a.rm[(int64_t)y * a.n + x] = 1;
            bool in_y = true;
#pragma unroll
            for (int q = 0; q < DM; ++q)
                in_y = in_y && ((a.adj[(int64_t)y * a.W + (sg[q] >> 6)] >> (sg[q] & 63)) & 1ull);
            const int sx = a.off[x] + find_in_sorted(a.nbr + a.off[x], a.deg[x], y);
#pragma unroll
            for (int q = 0; q < DM; ++q)
                atomicOr(reinterpret_cast<unsigned long long *>(&a.ug[(int64_t)sx * a.W + (sg[q] >> 6)]),
                         1ull << (sg[q] & 63));
            if (in_y && y > x) {
                const int sy = a.off[y] + find_in_sorted(a.nbr + a.off[y], a.deg[y], x);
#pragma unroll
                for (int q = 0; q < DM; ++q)
                    atomicOr(reinterpret_cast<unsigned long long *>(&a.ug[(int64_t)sy * a.W + (sg[q] >> 6)]),
                             1ull << (sg[q] & 63));
            }
        }
    }
    nindep = wave_sum(nindep);
    if ((threadIdx.x & 63) == 0 && nindep) atomicAdd(&a.ctr->indep, nindep);
}

template <int DM>
__global__ __launch_bounds__(256) void k_screen(LevelArgs a) {
    stamp_run_end(a);
    screen_lanes<DM>(a, blockIdx.x, gridDim.x, [&](int x, int y, const int *sg) { push_deferred(a, x, y, sg, DM); });
}

#ifndef PCG_NODE_BLOCKS
#define PCG_NODE_BLOCKS 0x10  // depths (bit 1 << d) whose fp32-screened narrow sweep stages compact node blocks
                              // (depth 4: kernel 2.13-2.16 -> 2.08 ms, FETCH 1.8 -> 0.18 GB; depth 3 measured no gain)
#endif
// the per-node compact blocks of the nodes with a chunk in [s_lo, s_hi): C[adj(x) + x, adj(x) + x]
// (row-major, stride D + 1, x last; each C entry read once, in C's own orientation) and the
// local adjacency masks (bit k of row t: nbr t and nbr k adjacent)
__global__ __launch_bounds__(256) void k_node_blocks(LevelArgs a, int64_t s_lo, int64_t s_hi) {
    const int x = blockIdx.x;
    if (a.cpre[x + 1] <= s_lo || a.cpre[x] >= s_hi || a.cpre[x + 1] == a.cpre[x]) return;
    const int D = a.deg[x];
    const int L = D + 1;
    __shared__ int ids[65];   // narrow nodes: D <= 64
    const int32_t *nx = a.nbr + a.off[x];
    for (int i = threadIdx.x; i < D; i += blockDim.x) ids[i] = nx[i];
    if (threadIdx.x == 0) ids[D] = x;
    __syncthreads();
    double *cb = a.cblk + a.bo[x];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    // rows: a wave per row, lane = column (D + 1 <= 65: lane 0 also takes column 64)
    for (int r = wv; r < L; r += nwv) {
        const double *row = a.C + (int64_t)ids[r] * a.ldc;
        for (int k = lane; k < L; k += 64) cb[r * L + k] = row[ids[k]];
        if (r < D) {
            const uint64_t *ar = a.adj + (int64_t)ids[r] * a.W;
            const bool bit = lane < D && ((ar[ids[lane] >> 6] >> (ids[lane] & 63)) & 1ull);
            const unsigned long long m = __ballot(bit);
            if (lane == 0) a.lmk[a.off[x] + r] = m;
        }
    }
}

// the same compact blocks, built transposed: one block per SOURCE row y stages C[y, :] and y's
// adjacency row in LDS (coalesced reads, C read once per depth), then writes row iy of the block
// of every node x whose block holds y (x in adj(y), and x = y itself for the block's last row):
// cb_x[iy][k] = C[y][ids_x[k]] from LDS, and (iy < D_x) x's local mask of y. A wave per target
// node; its rows are contiguous writes. k_node_blocks gathers the same entries from C's
// scattered columns — FETCH ~13x the block bytes at config 5's depth 4.
// IMG: the blocks are k_level_lds_f's fp32 LDS images instead (tgf_image_bytes, at bo[x] doubles):
// row iy of M = fp32(C[y][ids_x[k]]) (zero-padded to DS), y's record {fp32(C[y][y]), ., local mask},
// and from x's own row (y = x) every record's fp32(C[x][ids_x[k]]) and the id list — the values the
// kernel's own staging computes, so the sweep's results are unchanged
template <bool IMG>
__global__ __launch_bounds__(256) void k_node_blocks_t(LevelArgs a, int64_t s_lo, int64_t s_hi, int maxdeg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *row = reinterpret_cast<double *>(smem);
    uint64_t *arow = reinterpret_cast<uint64_t *>(row + a.n);
    int64_t *tbo = reinterpret_cast<int64_t *>(arow + a.W);   // per target: block offset,
    int *tx = reinterpret_cast<int *>(tbo + maxdeg + 1);       // node (-1: no block), degree, CSR offset
    int *tD = tx + maxdeg + 1, *toff = tD + maxdeg + 1;
    const int y = blockIdx.x;
    const int Dy = a.deg[y];
    const int32_t *ny = a.nbr + a.off[y];
    // the targets' descriptors in one round of loads (t = Dy: y's own block)
    bool any = false;
    for (int t = threadIdx.x; t <= Dy; t += blockDim.x) {
        const int x = t < Dy ? ny[t] : y;
        const bool hb = !(a.cpre[x + 1] <= s_lo || a.cpre[x] >= s_hi || a.cpre[x + 1] == a.cpre[x]);
        tx[t] = hb ? x : -1;
        tD[t] = a.deg[x];
        toff[t] = a.off[x];
        tbo[t] = hb ? a.bo[x] : 0;
        any = any || hb;
    }
    if (!__syncthreads_or(any)) return;
    const double *cy = a.C + (int64_t)y * a.ldc;
    for (int k = threadIdx.x; k < a.n; k += blockDim.x) row[k] = cy[k];
    const uint64_t *ay = a.adj + (int64_t)y * a.W;
    for (int k = threadIdx.x; k < a.W; k += blockDim.x) arow[k] = ay[k];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    // a target's list is one coalesced load (D <= 64: a lane per entry), issued one target ahead;
    // y's position in it is the count of smaller entries (a ballot, no dependent search)
    auto load = [&](int t) {
        const int x = tx[t], D = tD[t];
        return (x >= 0 && lane < D) ? a.nbr[toff[t] + lane] : x;
    };
    int g = wv <= Dy ? load(wv) : 0;
    for (int t = wv; t <= Dy; t += nwv) {
        const int gn = t + nwv <= Dy ? load(t + nwv) : 0;
        const int x = tx[t];
        if (IMG && x >= 0) {
            const int D = tD[t], DS = (D + 3) & ~3;
            float *img = reinterpret_cast<float *>(a.cblk + tbo[t]);
            float *Yr = img + D * DS;
            if (x == y) {
                if (lane < D) {
                    Yr[4 * lane + 1] = (float)row[g];
                    reinterpret_cast<int32_t *>(Yr + 4 * DS)[lane] = g;
                }
            } else {
                const int iy = __popcll(__ballot(lane < D && g < y));
                if (lane < DS) img[iy * DS + lane] = lane < D ? (float)row[g] : 0.0f;
                const bool bit = lane < D && ((arow[g >> 6] >> (g & 63)) & 1ull);
                const unsigned long long m = __ballot(bit);
                if (lane == 0) {
                    Yr[4 * iy] = (float)row[y];
                    *reinterpret_cast<unsigned long long *>(Yr + 4 * iy + 2) = m;
                }
            }
        } else if (x >= 0) {
            const int D = tD[t], L = D + 1;
            const int iy = x == y ? D : __popcll(__ballot(lane < D && g < y));
            double *cb = a.cblk + tbo[t] + (int64_t)iy * L;
            if (lane < L) cb[lane] = row[g];                 // lane D: column x (g = x there)
            if (L > 64 && lane == 0) cb[64] = row[x];        // D = 64: the block's last column
            if (iy < D) {
                const bool bit = lane < D && ((arow[g >> 6] >> (g & 63)) & 1ull);
                const unsigned long long m = __ballot(bit);
                if (lane == 0) a.lmk[toff[t] + iy] = m;
            }
        }
        g = gn;
    }
}

// ---------------------------------------------------------------------------------------
// depths > PCG_MAX_DEPTH (degenerate graphs, e.g. constant columns whose NaN correlations
// never separate): one thread per (x, S rank), exact LU path per test with per-thread
// scratch in global memory. Throughput is not the goal here; semantics are.
__global__ __launch_bounds__(64) void k_level_deep(LevelArgs a, double *scratch, int64_t nchunks) {
    const int d = a.d;
    const int m = d + 2;
    const int per = m * m + 2 * m + (d + 2);      // doubles: A, B0, B1, then int space
    const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double *A = scratch + gtid * per;
    double *B0 = A + m * m, *B1 = B0 + m;
    int *kk = reinterpret_cast<int *>(B1 + m);   // d ints (fits in d+2 doubles)
    int piv[PCG_MAX_LEVEL_DEPTH + 2];
    int var[PCG_MAX_LEVEL_DEPTH + 2];
    unsigned long long tests = 0, nindep = 0;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const int64_t chunk = a.chunk_lo + c;
        if (chunk >= a.cpre[a.n]) break;    // (defensive)
        int lo = chunk_node(a.cpre, a.n, chunk);
        const int x = lo;
        const int D = a.deg[x];
        const int32_t *nx = a.nbr + a.off[x];
        const uint64_t nS = pcg_binom(a.binom, D, d);
        const uint64_t rank = (uint64_t)(chunk - a.cpre[x]) * 64u + threadIdx.x;
        if (rank >= nS) continue;
        {   // colex unrank
            uint64_t rr = rank;
            int hi_ = D;
            for (int ii = d - 1; ii >= 0; --ii) {
                int lo_ = ii, up = hi_ - 1;
                while (lo_ < up) {
                    const int mid = (lo_ + up + 1) >> 1;
                    if (pcg_binom(a.binom, mid, ii + 1) <= rr) lo_ = mid; else up = mid - 1;
                }
                kk[ii] = lo_;
                rr -= pcg_binom(a.binom, lo_, ii + 1);
                hi_ = lo_;
            }
        }
        int p = 0;
        for (int t = 0; t < D; ++t) {
            if (p < d && kk[p] == t) { ++p; continue; }
            const int yg = nx[t];
            bool in_y = true;
            for (int q = 0; q < d && in_y; ++q) {
                const int s = nx[kk[q]];
                in_y = (a.adj[(int64_t)yg * a.W + (s >> 6)] >> (s & 63)) & 1ull;
            }
            if (yg < x && in_y) continue;
            ++tests;
            var[0] = x < yg ? x : yg;
            var[1] = x < yg ? yg : x;
            for (int q = 0; q < d; ++q) var[2 + q] = nx[kk[q]];
            for (int r = 0; r < m; ++r)
                for (int c = 0; c < m; ++c) A[r * m + c] = a.C[(int64_t)var[r] * a.ldc + var[c]];
            double i00, i01, i11, pv = __builtin_nan("");
            int err = 0;
            if (pcg_lu_inv01(A, m, piv, B0, B1, &i00, &i01, &i11)) err = 1;
            else {
                const double prod = i00 * i11;
                if (prod < 0.0 || a.dof_negative) err = 2;
                else pv = pcg_pvalue_from_r(-i01 / sqrt(prod), a.sqrt_dof, &err);
            }
            if (err) { flag_error(a, err); continue; }
            if (fabs(pv - a.alpha) < 1e-9) atomicAdd(&a.ctr->near_alpha, 1ull);
            if (pv > a.alpha) {
                ++nindep;
                a.rm[(int64_t)x * a.n + yg] = 1;
                a.rm[(int64_t)yg * a.n + x] = 1;
                unsigned long long *rx = reinterpret_cast<unsigned long long *>(a.ug + ((int64_t)a.off[x] + t) * a.W);
                for (int q = 0; q < d; ++q) atomicOr(&rx[var[2 + q] >> 6], 1ull << (var[2 + q] & 63));
                if (in_y && yg > x) {
                    const int sy = a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x);
                    unsigned long long *ry = reinterpret_cast<unsigned long long *>(a.ug + (int64_t)sy * a.W);
                    for (int q = 0; q < d; ++q) atomicOr(&ry[var[2 + q] >> 6], 1ull << (var[2 + q] & 63));
                }
            }
        }
    }
    if (tests) atomicAdd(&a.ctr->tests, tests);
    if (nindep) atomicAdd(&a.ctr->indep, nindep);
    if (tests) atomicAdd(&a.ctr->exact, tests);
}

// ---------------------------------------------------------------------------------------
// Deep levels (full-p mode from d = 13, threshold mode beyond the per-lane k_level_lds — see
// use_wave; PCG_WAVE_LO forces it from a given depth; the reference's unlimited-depth loop reaches
// them on sparse graphs, SkeletonDiscovery.py:72), narrow nodes (D <= WAVE_MAXD), threshold / full-p
// modes: ONE WAVE PER CONDITIONING SET S, lanes = the columns of the node block — lane t < D
// the neighbour t, lane D the node x itself. Every lane forward-solves its own column,
//   v_c = L^-1 C[S, c],   L = chol(C_SS),
// and the Cholesky factor is never formed separately: for a lane c = S_j its solve IS row j of L
// (L^-1 C_SS = L^T), so at step i the lanes read L[i][q] = v_{S_i}[q] from lane S_i (v_readlane,
// S_i is wave-uniform) and the pivot lambda_i^2 from lane S_i's own residual:
//   t_c = C[S_i][c] - sum_{q<i} L[i][q] v_c[q],   lambda_i^2 = t_{S_i},   v_c[i] = t_c / lambda_i.
// After |S| steps every lane holds |v_c|^2 and u.v_c (u = v_x, broadcast from lane D as it is
// formed), so ALL tests (x, y | S), y in adj(x) \ S, finish in parallel: c_yy = C_yy - |v_y|^2,
// c_xy = C_xy - u.v_y, c_xx = C_xx - |u|^2, decided like the other kernels (threshold band,
// conditioning guard; the rest on the exact LU path: the deferred list for |S| <= PCG_MAX_DEPTH,
// in the wave's LDS slot beyond). Per S: |S|^2 readlanes + |S|^2 / 2 fp64 FMAs per lane, for
// D - |S| tests — replaces the per-test global-scratch LU of k_level_deep (10 ms for 19 tests).
// Consecutive sets of a wave follow colex order (Gosper's next-combination on the 64-bit mask).

constexpr int WAVE_MAXD = 63;    // D + 1 lanes (the neighbours and x) per wave

// global ids of the members of a local set mask (ascending), -1 padded to PCG_MAX_DEPTH
__device__ __forceinline__ void set_members(unsigned long long mask, const int32_t *nxs, int (&sg)[PCG_MAX_DEPTH]) {
#pragma unroll
    for (int q = 0; q < PCG_MAX_DEPTH; ++q) {
        sg[q] = mask ? nxs[__builtin_ctzll(mask)] : -1;
        mask &= mask - 1;
    }
}

// The factorisation is shared between consecutive sets. A wave walks its run of colex ranks; the
// colex successor (Gosper) changes only the LOWEST elements of S, so the steps run in DESCENDING
// element order: steps 0..k-1 (the elements above the highest changed bit) and every lane's solve
// values, pivot, |v|^2 and u.v prefixes up to them stay valid, and only the steps of the changed
// low elements are redone — ~1-2 steps per set instead of |S| (round 3: the per-set
// factorisation, removed in round 5, measured slower on every deep level). The guard uses the
// smallest pivot^2 of this factorisation order.
template <int MD, int MODE>
__global__ __launch_bounds__(256) void k_level_wave(LevelArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int64_t chunk = a.chunk_lo + blockIdx.x;
    if (chunk >= a.cpre[a.n]) return;
    int lo = chunk_node(a.cpre, a.n, chunk);
    const int x = lo;
    const int D = a.deg[x];
    const int d = a.d;
    const int32_t *nxg = a.nbr + a.off[x];

    double *M = reinterpret_cast<double *>(smem);                 // D * D
    double *Mx = M + D * D;                                       // D
    double *Md = Mx + D;                                          // D
    unsigned long long *lmask = reinterpret_cast<unsigned long long *>(Md + D);   // D
    unsigned long long *uself = lmask + D;                        // D
    unsigned long long *uprop = uself + D;                        // D
    int32_t *nxs = reinterpret_cast<int32_t *>(uprop + D);       // D
    int *s_tx = nxs + D;                                          // 1
    double *slot = reinterpret_cast<double *>(smem + a.lds_btab_off) + (size_t)wv * WAVE_SLOT_DOUBLES(MD);
    // the pivots of the factorisation in registers (per wave, after the four slots)
    double *pivs = reinterpret_cast<double *>(smem + a.lds_btab_off) + 4 * (size_t)WAVE_SLOT_DOUBLES(MD) + wv * MD;

    for (int i = tid; i < D; i += blockDim.x) nxs[i] = nxg[i];
    __syncthreads();
    for (int e = tid; e < D * D; e += blockDim.x) {
        const int t = e / D, k = e - t * D;
        M[e] = a.C[(int64_t)nxs[t] * a.ldc + nxs[k]];
    }
    stage_lmask(a, nxs, D, lmask);
    for (int t = tid; t < D; t += blockDim.x) {
        const int yg = nxs[t];
        Mx[t] = a.C[(int64_t)x * a.ldc + yg];
        Md[t] = a.diag[yg];
        uself[t] = 0;
        uprop[t] = 0;
    }
    if (tid < 64) {                   // #neighbours below x (nxs ascends; D <= 64 here)
        const int c = __popcll(__ballot(tid < D && nxs[tid] < x));
        if (tid == 0) *s_tx = c;
    }
    __syncthreads();
    const int tx = *s_tx;
    const double Cxx = a.diag[x];
    const uint64_t nS = pcg_binom(a.binom, D, d);
    const uint64_t spl = (uint64_t)a.spl;
    const uint64_t r0 = (uint64_t)(chunk - a.cpre[x]) * 4u * spl + (uint64_t)wv * spl;
    const uint64_t r1 = min(nS, r0 + spl);
    unsigned long long tests = 0, indep = 0;
    if (r0 < r1) {
        unsigned long long mask = 0;      // colex unrank of r0 (wave-uniform)
        {
            uint64_t rr = r0;
            int hi_ = D;
            for (int ii = d - 1; ii >= 0; --ii) {
                int lo_ = ii, up = hi_ - 1;
                while (lo_ < up) {
                    const int mid = (lo_ + up + 1) >> 1;
                    if (pcg_binom(a.binom, mid, ii + 1) <= rr) lo_ = mid; else up = mid - 1;
                }
                mask |= 1ull << lo_;
                rr -= pcg_binom(a.binom, lo_, ii + 1);
                hi_ = lo_;
            }
        }
        const int cl = lane < D ? lane : 0;            // lane D (x) and idle lanes: a safe column
        double v[MD];                                   // this lane's solve values, step order
        unsigned long long prev = 0;                   // the mask whose steps are in registers
        for (uint64_t rank = r0; rank < r1; ++rank) {
            // steps 0..k-1 (elements above the highest bit that changed) are still valid
            int k = 0;
            if (prev) {
                const unsigned long long ch = prev ^ mask;
                const int hb = 63 - __builtin_clzll(ch);
                k = __popcll(hb == 63 ? 0ull : (mask >> (hb + 1)));
            }
            unsigned long long m = mask;              // drop the top k elements
            for (int q = 0; q < k; ++q) m &= ~(1ull << (63 - __builtin_clzll(m)));
#pragma unroll
            for (int i = 0; i < MD; ++i) {
                if (i >= k && i < d) {                 // wave-uniform
                    const int si = 63 - __builtin_clzll(m);   // the i-th largest element of S
                    m &= ~(1ull << si);
                    double t = lane < D ? M[si * D + cl] : Mx[si];
#pragma unroll
                    for (int q = 0; q < i; ++q) t -= readlane_f64(v[q], si) * v[q];   // L[i][q] = lane si's v[q]
                    const double piv = readlane_f64(t, si);
                    if (lane == 0) pivs[i] = piv;
                    v[i] = t * (1.0 / sqrt(piv));
                }
            }
            prev = mask;
            wave_sync();
            double vv = 0.0, uv = 0.0, gmin = 1.0;
            bool ok = true;
#pragma unroll
            for (int i = 0; i < MD; ++i) {
                if (i < d) {
                    const double piv = pivs[i];
                    ok = ok && (piv > 0.0);
                    gmin = fmin(gmin, piv);
                    vv += v[i] * v[i];
                    uv += readlane_f64(v[i], D) * v[i];
                }
            }
            const double cxx = Cxx - readlane_f64(vv, D);
            const double kg = a.tau / gmin;
            bool live = lane < D && !((mask >> lane) & 1ull);
            const unsigned long long lm = live ? lmask[cl] : 0ull;
            const bool in_y = (lm & mask) == mask;
            live = live && !(lane < tx && in_y);
            tests += live;
            int dec = 2;
            double p = 0.0;
            if (live && ok) dec = decide<MODE>(a, Mx[cl] - uv, cxx, Md[cl] - vv, kg, &p);
            if (live && dec == 1) {
                ++indep;
                atomicOr(&uself[cl], mask);
                if (in_y && lane >= tx) atomicOr(&uprop[cl], mask);
            }
            if (MODE == MODE_FULLP && live && dec != 2) {
                const int yg = nxs[cl];
                const int lo_ = x < yg ? x : yg, hi_ = x < yg ? yg : x;
                const bool near = fabs(p - a.alpha) < 1e-9;
                if (d <= PCG_MAX_DEPTH && (near || rec_on(a, lo_, hi_))) {
                    int sg[PCG_MAX_DEPTH];
                    set_members(mask, nxs, sg);
                    if (rec_on(a, lo_, hi_)) push_record(a.records, a.rec_cap, &a.ctr->records, lo_, hi_, d, sg, p);
                    if (near) push_record(a.nearl, a.near_cap, &a.ctr->near_alpha, lo_, hi_, d, sg, p);
                } else if (near) {
                    atomicAdd(&a.ctr->near_alpha, 1ull);
                }
            }
            if (d <= PCG_MAX_DEPTH) {
                if (live && dec == 2) {
                    int sg[PCG_MAX_DEPTH];
                    set_members(mask, nxs, sg);
                    push_deferred(a, x, nxs[cl], sg, d);
                }
            } else {
                unsigned long long need = __ballot(live && dec == 2);
                const int mm = d + 2;
                double *A = slot, *B0 = slot + mm * mm, *B1 = B0 + mm;
                int *var = reinterpret_cast<int *>(B1 + mm);
                while (need) {
                    const int L = __builtin_ctzll(need);
                    need &= need - 1;
                    const int yg = nxs[L];
                    wave_sync();
                    if (lane < D && ((mask >> lane) & 1ull))
                        var[2 + __popcll(mask & ((1ull << lane) - 1ull))] = nxs[lane];
                    if (lane == 0) {
                        var[0] = x < yg ? x : yg;
                        var[1] = x < yg ? yg : x;
                    }
                    wave_sync();
                    for (int kk = lane; kk < mm * mm; kk += 64) {
                        const int r = kk / mm, c = kk - r * mm;
                        A[kk] = a.C[(int64_t)var[r] * a.ldc + var[c]];
                    }
                    wave_sync();
                    if (lane == 0) {
                        double pv = __builtin_nan("");
                        const int err = exact_lu_pvalue(A, mm, B0, B1, a.sqrt_dof, &pv);
                        atomicAdd(&a.ctr->exact, 1ull);
                        if (err) {
                            flag_error(a, err);
                        } else {
                            if (fabs(pv - a.alpha) < 1e-9) atomicAdd(&a.ctr->near_alpha, 1ull);
                            if (pv > a.alpha) {
                                ++indep;
                                atomicOr(&uself[L], mask);
                                if (((lmask[L] & mask) == mask) && L >= tx) atomicOr(&uprop[L], mask);
                            }
                        }
                    }
                }
            }
            const unsigned long long c0 = mask & (0ull - mask);
            const unsigned long long rr = mask + c0;
            mask = (((rr ^ mask) >> 2) >> __builtin_ctzll(mask)) | rr;
        }
    }
    __syncthreads();
    for (int t = tid; t < D; t += blockDim.x) {
        const unsigned long long us = uself[t], up = uprop[t];
        if (!(us | up)) continue;
        const int yg = nxs[t];
        a.rm[(int64_t)x * a.n + yg] = 1;
        a.rm[(int64_t)yg * a.n + x] = 1;
        for (int side = 0; side < 2; ++side) {
            unsigned long long mb = side ? up : us;
            if (!mb) continue;
            const int64_t s = side ? (int64_t)a.off[yg] + find_in_sorted(a.nbr + a.off[yg], a.deg[yg], x)
                                   : (int64_t)a.off[x] + t;
            unsigned long long *row = reinterpret_cast<unsigned long long *>(a.ug + s * a.W);
            while (mb) {
                const int b = __ffsll((long long)mb) - 1;
                const int g = nxs[b];
                atomicOr(&row[g >> 6], 1ull << (g & 63));
                mb &= mb - 1;
            }
        }
    }
    block_flush_counts(a.ctr, tests, indep);
}

// ---------------------------------------------------------------------------------------
// exact path over the deferred list (LU like numpy.linalg.inv; the reference p expression)
template <int M>
__device__ __forceinline__ int lu_from_lds(const double *A, double *i00, double *i01, double *i11) {
    double R[M][M];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int c = 0; c < M; ++c) R[r][c] = A[r * M + c];
    return pcg_lu_inv01_reg<M>(R, i00, i01, i11);
}

// One wave per deferred test: the lanes gather the (d+2)^2 correlation entries in parallel
// into the wave's LDS slot (a single lane's rolled gather would wait out one HBM latency per
// entry), then lane 0 factors and decides.
// the exact path's verdict for one deferred test, after its factorisation (sing, i00, i01, i11 =
// the inverse's top-left 2 x 2 entries): numpy's errors, the reference p expression, records,
// near-alpha entries, and an independence's removal flags and per-side unions
__device__ __forceinline__ void exact_finish(const LevelArgs &a, const DeferredEntry &e, int sing, double i00, double i01,
                                             double i11, unsigned long long &nexact, unsigned long long &nindep) {
    const int d = a.d;
    const int x = e.x, y = e.y;
    const int lo_ = x < y ? x : y, hi_ = x < y ? y : x;
    double p = __builtin_nan("");
    int err = 0;
    if (sing) {
        err = 1;
    } else {
        const double prod = i00 * i11;
        if (prod < 0.0) err = 2;
        else if (a.dof_negative) err = 2;
        else {
            const double r = -i01 / sqrt(prod);
            p = pcg_pvalue_from_r(r, a.sqrt_dof, &err);
        }
    }
    ++nexact;
    if (err) { flag_error(a, err); return; }
    if (rec_on(a, lo_, hi_)) push_record(a.records, a.rec_cap, &a.ctr->records, lo_, hi_, d, e.s, p);
    if (fabs(p - a.alpha) < 1e-9) push_record(a.nearl, a.near_cap, &a.ctr->near_alpha, lo_, hi_, d, e.s, p);
    if (p > a.alpha) {
        ++nindep;
        a.rm[(int64_t)x * a.n + y] = 1;
        a.rm[(int64_t)y * a.n + x] = 1;
        if (d > 0) {
            bool in_y = true;
            for (int q = 0; q < d; ++q)
                in_y = in_y && ((a.adj[(int64_t)y * a.W + (e.s[q] >> 6)] >> (e.s[q] & 63)) & 1ull);
            const int sx = a.off[x] + find_in_sorted(a.nbr + a.off[x], a.deg[x], y);
            for (int q = 0; q < d; ++q)
                atomicOr(reinterpret_cast<unsigned long long *>(&a.ug[(int64_t)sx * a.W + (e.s[q] >> 6)]),
                         1ull << (e.s[q] & 63));
            if (in_y && y > x) {
                const int sy = a.off[y] + find_in_sorted(a.nbr + a.off[y], a.deg[y], x);
                for (int q = 0; q < d; ++q)
                    atomicOr(reinterpret_cast<unsigned long long *>(&a.ug[(int64_t)sy * a.W + (e.s[q] >> 6)]),
                             1ull << (e.s[q] & 63));
            }
        }
    }
}

// lane-per-test form for d <= 4 (m = d + 2 <= 6): each lane gathers its test's m^2 entries into
// registers (all loads issued before the first use) and factors them (numpy.linalg.inv's order,
// the same register routine the wave form's lane 0 runs: identical results). Used when the list
// is long — the full-p mode's recorded pairs put ~1e6 tests here at config 5 depth 4, where one
// wave per test left 63 of its 64 lanes idle through every factorisation
template <int M>
__device__ __forceinline__ void exact_one(const LevelArgs &a, const DeferredEntry &e, unsigned long long &nexact,
                                          unsigned long long &nindep) {
    constexpr int D = M - 2;
    {
        int var[M];
        var[0] = e.x < e.y ? e.x : e.y;
        var[1] = e.x < e.y ? e.y : e.x;
#pragma unroll
        for (int q = 0; q < D; ++q) var[2 + q] = e.s[q];
        double R[M][M];
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int c = 0; c < M; ++c) R[r][c] = a.C[(int64_t)var[r] * a.ldc + var[c]];
        double i00, i01, i11;
        const int sing = pcg_lu_inv01_reg<M>(R, &i00, &i01, &i11);
        exact_finish(a, e, sing, i00, i01, i11, nexact, nindep);
    }
}
template <int M>
__device__ __forceinline__ void exact_lanes(const LevelArgs &a, int64_t count, int blk, int nblk,
                                            unsigned long long &nexact, unsigned long long &nindep) {
    const int64_t lanes = (int64_t)nblk * blockDim.x;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < count; i += lanes) {
        const DeferredEntry e = a.deferred[i];
        exact_one<M>(a, e, nexact, nindep);
    }
}
// the exact path with a lane per test (d <= 4; launched with records, whose recorded pairs put
// every test of those pairs on the list): the overflow check of k_exact, wave-summed counters
template <int M>
__global__ __launch_bounds__(256) void k_exact_lanes(LevelArgs a) {
    stamp_run_end(a);
    const unsigned long long pushed = *(volatile const unsigned long long *)&a.ctr->deferred;
    const int64_t count = (int64_t)min((unsigned long long)a.def_cap, pushed);
    if (blockIdx.x == 0 && threadIdx.x == 0 &&
        ((int64_t)pushed > a.def_cap || (a.record && (int64_t)a.ctr->records > a.rec_cap)))
        a.rm[(int64_t)a.n * a.n] = 1;      // overflow: every rank reruns (status byte 0)
    unsigned long long nexact = 0, nindep = 0;
    exact_lanes<M>(a, count, blockIdx.x, gridDim.x, nexact, nindep);
    nexact = wave_sum(nexact);
    nindep = wave_sum(nindep);
    if ((threadIdx.x & 63) == 0 && nexact) atomicAdd(&a.ctr->exact, nexact);
    if ((threadIdx.x & 63) == 0 && nindep) atomicAdd(&a.ctr->indep, nindep);
}

__device__ __forceinline__ void exact_waves(const LevelArgs &a, unsigned char *smem, int blk, int nblk) {
    const int d = a.d;
    const int m = d + 2;
    const int per = m * m + 2 * m;
    const int lane = threadIdx.x & 63;
    double *A = reinterpret_cast<double *>(smem) + (size_t)(threadIdx.x >> 6) * per;
    double *B0 = A + m * m;
    double *B1 = B0 + m;
    int piv[PCG_MAX_DEPTH + 2];
    const unsigned long long pushed = *(volatile const unsigned long long *)&a.ctr->deferred;
    const int64_t count = (int64_t)min((unsigned long long)a.def_cap, pushed);
    if (blk == 0 && threadIdx.x == 0 &&
        ((int64_t)pushed > a.def_cap ||
         (a.record && (int64_t)*(volatile const unsigned long long *)&a.ctr->records > a.rec_cap)))
        a.rm[(int64_t)a.n * a.n] = 1;      // overflow: every rank reruns (status byte 0)
    unsigned long long nexact = 0, nindep = 0;
    const int64_t waves = (int64_t)nblk * (blockDim.x >> 6);
    for (int64_t i = (int64_t)blk * (blockDim.x >> 6) + (threadIdx.x >> 6); i < count; i += waves) {
        const DeferredEntry e = a.deferred[i];
        const int x = e.x, y = e.y;
        const int lo_ = x < y ? x : y, hi_ = x < y ? y : x;
        int var[PCG_MAX_DEPTH + 2];
        var[0] = lo_; var[1] = hi_;
        for (int q = 0; q < d; ++q) var[2 + q] = e.s[q];
        for (int k = lane; k < m * m; k += 64) {
            const int r = k / m, c = k - r * m;
            int vr = lo_, vc = lo_;
            for (int q = 0; q < m; ++q) {      // register-indexed var[] without dynamic indexing
                if (q == r) vr = var[q];
                if (q == c) vc = var[q];
            }
            A[k] = a.C[(int64_t)vr * a.ldc + vc];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane != 0) continue;
        double i00, i01, i11;
        int sing;
        switch (m) {     // depths 0..4: the factorisation in registers; deeper: in the LDS slot
        case 2: sing = lu_from_lds<2>(A, &i00, &i01, &i11); break;
        case 3: sing = lu_from_lds<3>(A, &i00, &i01, &i11); break;
        case 4: sing = lu_from_lds<4>(A, &i00, &i01, &i11); break;
        case 5: sing = lu_from_lds<5>(A, &i00, &i01, &i11); break;
        case 6: sing = lu_from_lds<6>(A, &i00, &i01, &i11); break;
        default: sing = pcg_lu_inv01(A, m, piv, B0, B1, &i00, &i01, &i11);
        }
        exact_finish(a, e, sing, i00, i01, i11, nexact, nindep);
    }
    if (nexact) atomicAdd(&a.ctr->exact, nexact);
    if (nindep) atomicAdd(&a.ctr->indep, nindep);
}

__global__ __launch_bounds__(256) void k_exact(LevelArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    stamp_run_end(a);
    exact_waves(a, smem, blockIdx.x, gridDim.x);
}

// the fp32 sweep's level end in one launch (no records, d <= 4): the level kernels' band tests
// (the deferred list, final by stream order; a handful per level at config 5) and the fp64 screen,
// whose band tests take the exact path on the spot in their lane instead of a second list. The
// exact path is the lane form's (the same register LU and verdict as k_exact); every write is an
// OR or a counter, so the order of the two parts does not matter. Replaces k_screen + k_exact
// (config 5: 8-17 us of k_exact at depths 3 and 4 for 12-14 tests)
template <int DM>
__global__ __launch_bounds__(256) void k_screen_exact(LevelArgs a) {
    stamp_run_end(a);
    const unsigned long long pushed = *(volatile const unsigned long long *)&a.ctr->deferred;
    const int64_t count = (int64_t)min((unsigned long long)a.def_cap, pushed);
    if (blockIdx.x == 0 && threadIdx.x == 0 && (int64_t)pushed > a.def_cap)
        a.rm[(int64_t)a.n * a.n] = 1;      // overflow: every rank reruns (status byte 0)
    unsigned long long nexact = 0, nindep = 0;
    exact_lanes<DM + 2>(a, count, blockIdx.x, gridDim.x, nexact, nindep);
    screen_lanes<DM>(a, blockIdx.x, gridDim.x, [&](int x, int y, const int *sg) {
        DeferredEntry e;
        e.x = x;
        e.y = y;
#pragma unroll
        for (int i = 0; i < PCG_MAX_DEPTH; ++i) e.s[i] = i < DM ? sg[i] : -1;
        exact_one<DM + 2>(a, e, nexact, nindep);
    });
    nexact = wave_sum(nexact);
    nindep = wave_sum(nindep);
    if ((threadIdx.x & 63) == 0 && nexact) atomicAdd(&a.ctr->exact, nexact);
    if ((threadIdx.x & 63) == 0 && nindep) atomicAdd(&a.ctr->indep, nindep);
}

// ---------------------------------------------------------------------------------------
// Small graphs (n <= 64: the RQ2 cases, 30-49 metrics): the WHOLE stable skeleton in one
// workgroup launch. The multi-kernel level loop costs ~90 us of launches and host round trips
// per depth whatever the work; an RQ2 case has 6-8 depths of 10^2..10^4 tests. Here C, the
// adjacency, the neighbour lists and the per-side unions live in LDS, a depth ends at a block
// barrier, and the host waits once. Same semantics as the level loop: the reference's visit
// order and memo (x evaluates (x, y, S) unless y < x and S within adj(y); an owner x < y with S
// within adj(y) also serves y's visit), the fp64 threshold decision with its band and guard, the
// exact LU path (numpy.linalg.inv order, the reference p expression) in the wave for the band,
// deferred removal, per-side unions, near-alpha records, FULL_P / RECORD / EXACT_ALL.
constexpr int SMALL_N = 64;           // nodes: one u64 adjacency word per node
constexpr int SMALL_MAXD = 16;        // deepest conditioning set here (deeper: the level loop reruns)
constexpr int SMALL_LANE_D = 6;       // depths 1..6: one lane per test (chunks of SMALL_K sets of one (x, y))
constexpr int SMALL_K = 32;
constexpr int SMALL_WAVES = 8;        // 512 threads: two waves per SIMD (256 VGPRs: the fused solves fit unspilled)
constexpr int SMALL_SLOT = (SMALL_MAXD + 2) * (SMALL_MAXD + 2) + 3 * (SMALL_MAXD + 2);   // doubles per wave
constexpr int SMALL_QCAP = 1024;      // band-queue slots per depth (PCG_TUNE_SMALL_QCAP <= this; full: the level loop reruns)
static_assert(SMALL_SLOT >= SMALL_MAXD * (SMALL_MAXD + 1), "the wave slot holds the L rows too");

struct SmallArgs {
    const double *C;
    int64_t ldc;
    int n;
    int max_depth;
    double alpha, tau;
    const uint8_t *banned;            // n x n pairs forbidden both ways, or null
    const uint64_t *binom;
    int8_t *rl;                       // n x n removal depths (-1 = kept)
    int32_t *xy;                      // exported (x, y) of removed pairs with a non-empty side union
    uint64_t *bits;                   // their union words (W = 1)
    pcg_record *nearl, *records;
    int64_t near_cap, rec_cap, rec_mod, rec_res;
    unsigned long long *ctr;          // [0] near-alpha, [1] records (cumulative over the run)
    int fullp, record, exact_all;
    int qcap;                         // band tests per depth the queue takes (<= SMALL_QCAP)
    // per depth d (device memory, 4 doubles each): the threshold band on r^2 (lo2, hi2),
    // sqrt(N - d - 3), and 1.0 when N - d - 3 < 0 (a dynamically indexed kernel-argument array
    // would be copied to scratch)
    const double *depth_cst;
    struct SmallSummary *sum;
};

struct SmallDepth {
    double lo2, hi2, sqrt_dof;
    bool dof_negative;
};

struct SmallSummary {
    int32_t levels, status;           // status: 1 singular, 2 math domain, 4 deeper than SMALL_MAXD, 8 band queue full
    int64_t xrows;                    // exported sepset rows
    int64_t tests[PCG_MAX_LEVELS], calls[PCG_MAX_LEVELS], indep[PCG_MAX_LEVELS], exact[PCG_MAX_LEVELS];
    int64_t near_alpha[PCG_MAX_LEVELS], edges_after[PCG_MAX_LEVELS];
    int32_t max_degree[PCG_MAX_LEVELS];
    uint64_t stamp[PCG_MAX_LEVELS + 1];  // wall-clock ticks (100 MHz) at the depth boundaries
    int32_t deg[PCG_MAX_LEVELS][SMALL_N];
};

// the reference p expression out of line: inlined, its erfc polynomial constants are hoisted into
// registers across the callers' loops (hundreds of VGPRs spilled)
__device__ __attribute__((noinline)) double small_pvalue(double r, double sqrt_dof, int *err) {
    return pcg_pvalue_from_r(r, sqrt_dof, err);
}

__device__ __forceinline__ int small_decide(const SmallArgs &a, const SmallDepth &k, double cxy, double cxx, double cyy,
                                            double kg, double *p) {
    if (a.exact_all) return 2;
    const double den = cxx * cyy;
    if (!(den > 0.0)) return 2;
    const double num = cxy * cxy;
    if (!(den - num > kg)) return 2;
    if (!a.fullp) {
        if (num < k.lo2 * den) return 1;
        if (num > k.hi2 * den) return 0;
        return 2;
    }
    const double r = cxy / sqrt(den);
    int err = 0;
    const double pv = small_pvalue(r, k.sqrt_dof, &err);
    if (err) return 2;
    *p = pv;
    return pv > a.alpha ? 1 : 0;
}

__device__ __forceinline__ bool small_rec_on(const SmallArgs &a, int lo, int hi) {
    return a.record && (a.rec_mod <= 1 || ((int64_t)lo * a.n + hi) % a.rec_mod == a.rec_res);
}

// the exact path of one test (lo < hi, S ascending global ids in sg) in the wave's slot: lanes
// gather the m x m matrix, lane 0 factors; returns 0 dependent, 1 independent, -1 error (flagged)
__device__ __attribute__((noinline)) int small_exact(const SmallArgs &a, const SmallDepth &kd, const double *Cf, int n,
                                                     int d, int lo, int hi,
                           unsigned long long Sg, double *slot, int *status, double *pout) {
    const int lane = threadIdx.x & 63, m = d + 2;
    double *A = slot, *B0 = slot + m * m, *B1 = B0 + m;
    int *var = reinterpret_cast<int *>(B1 + m);
    wave_sync();
    if (lane == 0) {
        var[0] = lo;
        var[1] = hi;
        unsigned long long s = Sg;
        for (int q = 0; q < d; ++q) {
            var[2 + q] = __builtin_ctzll(s);
            s &= s - 1;
        }
    }
    wave_sync();
    for (int k = lane; k < m * m; k += 64) {
        const int r = k / m, c = k - r * m;
        A[k] = Cf[var[r] * n + var[c]];
    }
    wave_sync();
    int res = 0;
    if (lane == 0) {
        // k_exact's order of checks: singular, then a negative determinant ratio or N - d - 3 < 0
        double pv = __builtin_nan("");
        int err = 0;
        int piv[PCG_MAX_LEVEL_DEPTH + 2];
        double i00, i01, i11;
        if (pcg_lu_inv01(A, m, piv, B0, B1, &i00, &i01, &i11)) {
            err = 1;
        } else {
            const double prod = i00 * i11;
            if (prod < 0.0 || kd.dof_negative) err = 2;
            else pv = small_pvalue(-i01 / sqrt(prod), kd.sqrt_dof, &err);
        }
        if (err) {
            atomicOr(status, err);
            res = -1;
        } else {
            *pout = pv;
            res = pv > a.alpha ? 1 : 0;
        }
    }
    wave_sync();
    return __shfl(res, 0);
}

__device__ __forceinline__ void small_sorted_set(unsigned long long Sg, int d, int (&sg)[PCG_MAX_DEPTH]) {
#pragma unroll
    for (int q = 0; q < PCG_MAX_DEPTH; ++q) {
        sg[q] = (q < d && Sg) ? __builtin_ctzll(Sg) : -1;
        if (q < d && Sg) Sg &= Sg - 1;
    }
}

// (x, y | S) from the correlation block in LDS, one lane: Cholesky of C_SS row by row with the
// solves for x and y fused (only L, 1/diag and the two solution vectors live); the fp64 kernels'
// guard and band. 0 dependent, 1 independent, 2 exact path
template <int DM>
__device__ __forceinline__ int small_lane_eval(const SmallArgs &a, const SmallDepth &kd, const double *Cf, int n, int d,
                                               int x, int y, const int (&sg)[DM], double *p) {
    double L[DM][DM], rinv[DM], u[DM], v[DM];
    double uu = 0.0, vv = 0.0, uv = 0.0, gmin = 1.0;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        if (i < d) {
            const double *Ci = Cf + sg[i] * n;
            double s = Ci[sg[i]];
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double t = Ci[sg[j]];
#pragma unroll
                for (int q = 0; q < j; ++q) t -= L[i][q] * L[j][q];
                L[i][j] = t * rinv[j];
                s -= L[i][j] * L[i][j];
            }
            ok = ok && (s > 0.0);
            gmin = fmin(gmin, s);
            rinv[i] = 1.0 / sqrt(s);
            double tu = Ci[x], tv = Ci[y];
#pragma unroll
            for (int q = 0; q < i; ++q) {
                tu -= L[i][q] * u[q];
                tv -= L[i][q] * v[q];
            }
            u[i] = tu * rinv[i];
            v[i] = tv * rinv[i];
            uu += u[i] * u[i];
            vv += v[i] * v[i];
            uv += u[i] * v[i];
        }
    }
    if (!ok) return 2;
    return small_decide(a, kd, Cf[x * n + y] - uv, Cf[x * n + x] - uu, Cf[y * n + y] - vv, a.tau / gmin, p);
}

// one conditioning set S (local positions `mask` within x's neighbour list, |S| = d) of node x,
// lanes = the neighbour columns (lane D = x): the k_level_wave solve, then every live y at once
template <int MD>
__device__ void small_set(const SmallArgs &a, const SmallDepth &kd, const double *Cf, const uint64_t *adjm, const uint8_t *nbx, int x,
                          int D, int d, int tx, unsigned long long mask, double *slot, uint64_t *uni, uint64_t *rmb,
                          int *status, unsigned long long &tests, unsigned long long &indep,
                          unsigned long long &exact, unsigned long long &nearc) {
    const int lane = threadIdx.x & 63, n = a.n;
    const int colg = lane < D ? nbx[lane] : x;
    double v[MD];
    double vv = 0.0, uv = 0.0, gmin = 1.0;
    bool ok = true;
    unsigned long long m = mask, Sg = 0;
    const bool member = lane < D && ((mask >> lane) & 1ull);
    const int mypos = member ? __popcll(mask & ((1ull << lane) - 1ull)) : -1;
    double *Lm = slot;
    constexpr int LS = MD + 1;
#pragma unroll
    for (int i = 0; i < MD; ++i) {
        if (i < d) {
            const int si = __builtin_ctzll(m);
            m &= m - 1;
            const int sg = nbx[si];
            Sg |= 1ull << sg;
            double t = Cf[sg * n + colg];
            const double *Li = Lm + i * LS;
#pragma unroll
            for (int q = 0; q < i; ++q) t -= Li[q] * v[q];
            const double piv = readlane_f64(t, si);
            ok = ok && (piv > 0.0);
            gmin = fmin(gmin, piv);
            v[i] = t * (1.0 / sqrt(piv));
            vv += v[i] * v[i];
            uv += readlane_f64(v[i], D) * v[i];
            if (mypos > i) Lm[mypos * LS + i] = v[i];
            wave_sync();
        }
    }
    const double cxx = Cf[x * n + x] - readlane_f64(vv, D);
    const double kg = a.tau / gmin;
    bool live = lane < D && !member;
    const bool in_y = live && ((adjm[colg] & Sg) == Sg);
    live = live && !(lane < tx && in_y);
    tests += live;
    int dec = 2;
    double p = 0.0;
    if (live && ok) dec = small_decide(a, kd, Cf[x * n + colg] - uv, cxx, Cf[colg * n + colg] - vv, kg, &p);
    const int lo_ = x < colg ? x : colg, hi_ = x < colg ? colg : x;
    if (live && dec != 2 && a.fullp) {
        if (d <= PCG_MAX_DEPTH && (small_rec_on(a, lo_, hi_) || fabs(p - a.alpha) < 1e-9)) {
            int sgl[PCG_MAX_DEPTH];
            small_sorted_set(Sg, d, sgl);
            if (small_rec_on(a, lo_, hi_)) push_record(a.records, a.rec_cap, &a.ctr[1], lo_, hi_, d, sgl, p);
            if (fabs(p - a.alpha) < 1e-9) push_record(a.nearl, a.near_cap, &a.ctr[0], lo_, hi_, d, sgl, p);
        }
        if (fabs(p - a.alpha) < 1e-9) ++nearc;
    }
    if (live && dec == 1) {
        ++indep;
        atomicOr(&uni[x * SMALL_N + colg], Sg);
        if (in_y && lane >= tx) atomicOr(&uni[colg * SMALL_N + x], Sg);
        atomicOr(&rmb[x], 1ull << colg);
        atomicOr(&rmb[colg], 1ull << x);
    }
    // the exact path of this set's remaining tests, one at a time in the wave's slot (the L rows
    // are no longer needed)
    unsigned long long need = __ballot(live && dec == 2);
    while (need) {
        const int L = __builtin_ctzll(need);
        need &= need - 1;
        const int yg = nbx[L];
        const int lo = x < yg ? x : yg, hi = x < yg ? yg : x;
        double pv = 0.0;
        const int r = small_exact(a, kd, Cf, n, d, lo, hi, Sg, slot, status, &pv);
        if (lane == 0) {
            ++exact;
            if (r >= 0) {
                int sgl[PCG_MAX_DEPTH];
                small_sorted_set(Sg, d, sgl);
                if (d <= PCG_MAX_DEPTH && small_rec_on(a, lo, hi))
                    push_record(a.records, a.rec_cap, &a.ctr[1], lo, hi, d, sgl, pv);
                if (fabs(pv - a.alpha) < 1e-9) {
                    ++nearc;
                    if (d <= PCG_MAX_DEPTH) push_record(a.nearl, a.near_cap, &a.ctr[0], lo, hi, d, sgl, pv);
                }
                if (r == 1) {
                    ++indep;
                    atomicOr(&uni[x * SMALL_N + yg], Sg);
                    if (((adjm[yg] & Sg) == Sg) && L >= tx) atomicOr(&uni[yg * SMALL_N + x], Sg);
                    atomicOr(&rmb[x], 1ull << yg);
                    atomicOr(&rmb[yg], 1ull << x);
                }
            }
        }
    }
}

__global__ __launch_bounds__(SMALL_WAVES * 64, 1) void k_pc_small(SmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = a.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double *Cf = reinterpret_cast<double *>(smem);                                  // n x n
    uint64_t *uni = reinterpret_cast<uint64_t *>(Cf + n * n);                         // 64 x 64 side unions
    uint64_t *adjm = uni + SMALL_N * SMALL_N;                                         // 64
    uint64_t *rmb = adjm + SMALL_N;                                                   // 64: this depth's removals
    uint64_t *wpre = rmb + SMALL_N;                                                   // 65: work prefix over x
    uint64_t *bin = wpre + SMALL_N + 1;                                               // C(c, k), c < 64, k <= MAXD
    uint64_t *qS = bin + SMALL_N * (SMALL_MAXD + 1);                                  // band queue: S masks
    double *slots = reinterpret_cast<double *>(qS + SMALL_QCAP);                      // waves x SMALL_SLOT
    int *deg = reinterpret_cast<int *>(slots + SMALL_WAVES * SMALL_SLOT);             // 64
    int *misc = deg + SMALL_N;                                                        // 16 ints
    uint16_t *qxy = reinterpret_cast<uint16_t *>(misc + 16);                          // band queue: x | y << 8
    int8_t *rlv = reinterpret_cast<int8_t *>(qxy + SMALL_QCAP);                       // 64 x 64
    uint8_t *nb = reinterpret_cast<uint8_t *>(rlv + SMALL_N * SMALL_N);               // 64 x 64
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(
        (reinterpret_cast<uintptr_t>(nb + SMALL_N * SMALL_N) + 7) & ~(uintptr_t)7);  // next unit, tests, indep, exact, near, xrows, queue
    SmallSummary *sum = a.sum;
    int &status = misc[0];

    for (int e = tid; e < n * n; e += blockDim.x) Cf[e] = a.C[(int64_t)(e / n) * a.ldc + e % n];
    for (int e = tid; e < SMALL_N * SMALL_N; e += blockDim.x) {
        uni[e] = 0;
        rlv[e] = -1;
    }
    // the handle's table holds rows 0..n only (build_binom(n)): rows past n are never indexed here
    // (degrees stay < n) and are zeroed, not read — reading them ran past a fresh handle's small
    // allocation (an intermittent illegal address, r06)
    for (int e = tid; e < SMALL_N * (SMALL_MAXD + 1); e += blockDim.x) {
        const int c = e / (SMALL_MAXD + 1);
        bin[e] = c <= n ? pcg_binom(a.binom, c, e % (SMALL_MAXD + 1)) : 0ull;
    }
    const unsigned long long all = n == 64 ? ~0ull : ((1ull << n) - 1ull);
    for (int x = tid; x < SMALL_N; x += blockDim.x) {
        adjm[x] = x < n ? all & ~(1ull << x) : 0ull;
        rmb[x] = 0;
        deg[x] = x < n ? n - 1 : 0;
        for (int k = 0, c = 0; k < n; ++k)
            if (k != x && x < n) nb[x * SMALL_N + c++] = (uint8_t)k;
    }
    if (tid == 0) {
        status = 0;
        for (int k = 0; k < 8; ++k) cnt[k] = 0;
        sum->xrows = 0;
    }
    // NaN nodes (a constant or non-finite column: numpy's corrcoef row is NaN throughout, its
    // diagonal included): a test with one among x, y, S is NaN in the reference — the inverse of a
    // NaN sub-matrix is NaN (no LinAlgError), so r and p are NaN and p > alpha is False: dependent.
    // The lane-per-test depths decide those directly instead of queueing every one of them for the
    // exact path (whose LU gives the same NaN), so a NaN column no longer fills the band queue.
    __shared__ unsigned long long s_nanm;
    if (tid < 64) {
        const unsigned long long m = __ballot(tid < n && Cf[tid * n + tid] != Cf[tid * n + tid]);
        if (tid == 0) s_nanm = m;
    }
    __syncthreads();
    const unsigned long long nanm = s_nanm;
    auto B = [&](int c, int k) -> uint64_t { return (c < k || c < 0) ? 0ull : bin[c * (SMALL_MAXD + 1) + k]; };
    // an independent (x, y | S): removal flags both ways, x's side union, and y's when x's visit
    // also served y's (S within adj(y), y > x)
    auto indep_effects = [&](int x, int y, unsigned long long Sg, bool in_y) {
        atomicOr(&rmb[x], 1ull << y);
        atomicOr(&rmb[y], 1ull << x);
        if (Sg) {
            atomicOr(&uni[x * SMALL_N + y], Sg);
            if (in_y && y > x) atomicOr(&uni[y * SMALL_N + x], Sg);
        }
    };
    int levels = 0;
    for (int d = 0;; ++d) {
        // the reference's loop condition (max_degree() - 1 > depth - 1), the depth cap
        int maxdeg = 0;
        for (int x = 0; x < n; ++x) maxdeg = max(maxdeg, deg[x]);
        if (!(maxdeg - 1 > d - 1) || (a.max_depth >= 0 && d > a.max_depth) || d >= PCG_MAX_LEVELS) break;
        if (d > SMALL_MAXD) {
            if (tid == 0) status |= 4;
            break;
        }
        levels = d + 1;
        const bool lanewise = d >= 1 && d <= SMALL_LANE_D;
        SmallDepth kd;
        kd.lo2 = a.depth_cst[4 * d];
        kd.hi2 = a.depth_cst[4 * d + 1];
        kd.sqrt_dof = a.depth_cst[4 * d + 2];
        kd.dof_negative = a.depth_cst[4 * d + 3] != 0.0;
        if (wv == 0) {   // work prefix over x, calls, the degree snapshot
            const int D = lane < n ? deg[lane] : 0;
            const uint64_t cd = D >= 1 ? B(D - 1, d) : 0ull;
            const uint64_t units = d == 0 ? 0ull : lanewise ? (uint64_t)D * ((cd + SMALL_K - 1) / SMALL_K) : B(D, d);
            uint64_t incl = units, csum = cd * (uint64_t)D;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
            wpre[lane + 1] = incl;
            if (lane == 0) wpre[0] = 0;
            if (lane < n) sum->deg[d][lane] = D;
            if (lane == 0) {
                sum->calls[d] = (int64_t)csum;
                sum->max_degree[d] = maxdeg;
                sum->stamp[d] = wall_clock64();
                cnt[0] = 0;
                cnt[6] = 0;
            }
        }
        __syncthreads();
        unsigned long long tests = 0, indep = 0, exact = 0, nearc = 0;
        if (d == 0 || lanewise) {
            // one lane per test: the pairs at depth 0; chunks of SMALL_K consecutive sets (colex over
            // the positions of adj(x) \ {y}) of one (x, y) at depths 1..SMALL_LANE_D. Band tests
            // queue for the exact path below.
            const uint64_t total = d == 0 ? (uint64_t)n * (n - 1) / 2 : wpre[n];
            for (uint64_t u = tid; u < total; u += blockDim.x) {
                int x = 0, y = 0;
                unsigned long long mask = 0;
                uint64_t r0 = 0, r1 = 1;
                int D = 0, yi = 0;
                if (d == 0) {
                    int r = (int)u;
                    while (r >= n - 1 - x) { r -= n - 1 - x; ++x; }
                    y = x + 1 + r;
                } else {
                    int lo = 0, hi = n;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (wpre[mid] <= u) lo = mid; else hi = mid;
                    }
                    x = lo;
                    D = deg[x];
                    const uint64_t cd = B(D - 1, d), cpy = (cd + SMALL_K - 1) / SMALL_K;
                    const uint64_t local = u - wpre[x];
                    yi = (int)(local / cpy);
                    y = nb[x * SMALL_N + yi];
                    r0 = (local % cpy) * SMALL_K;
                    r1 = min(cd, r0 + SMALL_K);
                    uint64_t rr = r0;                 // colex unrank over D - 1 positions
                    int hi_ = D - 1;
                    for (int ii = d - 1; ii >= 0; --ii) {
                        int l2 = ii, up = hi_ - 1;
                        while (l2 < up) {
                            const int mid = (l2 + up + 1) >> 1;
                            if (B(mid, ii + 1) <= rr) l2 = mid; else up = mid - 1;
                        }
                        mask |= 1ull << l2;
                        rr -= B(l2, ii + 1);
                        hi_ = l2;
                    }
                }
                for (uint64_t r = r0; r < r1; ++r) {
                    // S: positions q of adj(x) \ {y} -> neighbour index q (< yi) or q + 1
                    int sg[SMALL_LANE_D];
                    unsigned long long Sg = 0, m = mask;
#pragma unroll
                    for (int i = 0; i < SMALL_LANE_D; ++i) {
                        sg[i] = x;
                        if (i < d) {
                            const int q = __builtin_ctzll(m);
                            m &= m - 1;
                            sg[i] = nb[x * SMALL_N + (q < yi ? q : q + 1)];
                            Sg |= 1ull << sg[i];
                        }
                    }
                    const bool in_y = d > 0 && (adjm[y] & Sg) == Sg;
                    if (!(d > 0 && y < x && in_y)) {     // y's visit evaluates it otherwise
                        ++tests;
                        double p = 0.0;
                        int dec;
                        if ((Sg | (1ull << x) | (1ull << y)) & nanm) {
                            dec = 0;
                            p = __builtin_nan("");
                        } else if (d <= 2) dec = small_lane_eval<2>(a, kd, Cf, n, d, x, y, reinterpret_cast<const int(&)[2]>(sg), &p);
                        else if (d <= 4) dec = small_lane_eval<4>(a, kd, Cf, n, d, x, y, reinterpret_cast<const int(&)[4]>(sg), &p);
                        else dec = small_lane_eval<SMALL_LANE_D>(a, kd, Cf, n, d, x, y, sg, &p);
                        const int lo_ = x < y ? x : y, hi_ = x < y ? y : x;
                        if (dec == 2) {
                            const unsigned long long slot = atomicAdd(&cnt[6], 1ull);
                            if (slot < (unsigned long long)a.qcap) {
                                qxy[slot] = (uint16_t)(x | (y << 8));
                                qS[slot] = Sg;
                            } else {
                                atomicOr(&status, 8);    // more band tests than the queue holds
                            }
                        } else {
                            if (a.fullp) {
                                const bool near = fabs(p - a.alpha) < 1e-9;
                                if (small_rec_on(a, lo_, hi_) || near) {
                                    int sgl[PCG_MAX_DEPTH];
                                    small_sorted_set(Sg, d, sgl);
                                    if (small_rec_on(a, lo_, hi_))
                                        push_record(a.records, a.rec_cap, &a.ctr[1], lo_, hi_, d, sgl, p);
                                    if (near) push_record(a.nearl, a.near_cap, &a.ctr[0], lo_, hi_, d, sgl, p);
                                }
                                nearc += near;
                            }
                            if (dec == 1) {
                                ++indep;
                                indep_effects(x, y, Sg, in_y);
                            }
                        }
                    }
                    if (d > 0) {                      // next set (Gosper)
                        const unsigned long long c0 = mask & (0ull - mask);
                        const unsigned long long rr2 = mask + c0;
                        mask = (((rr2 ^ mask) >> 2) >> __builtin_ctzll(mask)) | rr2;
                    }
                }
            }
            __syncthreads();
            // the exact path of the queued band tests: one wave per test
            const int qn = (int)min(cnt[6], (unsigned long long)a.qcap);
            for (int i = wv; i < qn; i += SMALL_WAVES) {
                const int x = qxy[i] & 255, y = qxy[i] >> 8;
                const unsigned long long Sg = qS[i];
                const int lo = x < y ? x : y, hi = x < y ? y : x;
                double pv = 0.0;
                const int r = small_exact(a, kd, Cf, n, d, lo, hi, Sg, slots + wv * SMALL_SLOT, &status, &pv);
                if (lane == 0) {
                    ++exact;
                    if (r >= 0) {
                        int sgl[PCG_MAX_DEPTH];
                        small_sorted_set(Sg, d, sgl);
                        if (small_rec_on(a, lo, hi)) push_record(a.records, a.rec_cap, &a.ctr[1], lo, hi, d, sgl, pv);
                        if (fabs(pv - a.alpha) < 1e-9) {
                            ++nearc;
                            push_record(a.nearl, a.near_cap, &a.ctr[0], lo, hi, d, sgl, pv);
                        }
                        if (r == 1) {
                            ++indep;
                            indep_effects(x, y, Sg, d > 0 && (adjm[y] & Sg) == Sg);
                        }
                    }
                }
            }
        } else {
            const uint64_t total = wpre[n];
            double *slot = slots + wv * SMALL_SLOT;
            for (;;) {
                unsigned long long u = 0;
                if (lane == 0) u = atomicAdd(&cnt[0], 1ull);
                u = __shfl(u, 0);
                if (u >= total) break;
                int lo = 0, hi = n;           // wpre[lo] <= u < wpre[lo + 1]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (wpre[mid] <= u) lo = mid; else hi = mid;
                }
                const int x = lo, D = deg[x];
                uint64_t rr = u - wpre[x];
                unsigned long long mask = 0;  // colex unrank (wave-uniform)
                int hi_ = D;
                for (int ii = d - 1; ii >= 0; --ii) {
                    int lo2 = ii, up = hi_ - 1;
                    while (lo2 < up) {
                        const int mid = (lo2 + up + 1) >> 1;
                        if (B(mid, ii + 1) <= rr) lo2 = mid; else up = mid - 1;
                    }
                    mask |= 1ull << lo2;
                    rr -= B(lo2, ii + 1);
                    hi_ = lo2;
                }
                const int tx = __popcll(adjm[x] & ((1ull << x) - 1ull));
                const uint8_t *nbx = nb + x * SMALL_N;
                if (d <= 8)
                    small_set<8>(a, kd, Cf, adjm, nbx, x, D, d, tx, mask, slot, uni, rmb, &status, tests, indep, exact, nearc);
                else
                    small_set<SMALL_MAXD>(a, kd, Cf, adjm, nbx, x, D, d, tx, mask, slot, uni, rmb, &status, tests, indep,
                                          exact, nearc);
            }
        }
        // counters (lane 0 of each wave holds the exact-path counts; every lane its tests / indep)
        tests = wave_sum(tests);
        indep = wave_sum(indep);
        exact = wave_sum(exact);
        nearc = wave_sum(nearc);
        if (lane == 0) {
            atomicAdd(&cnt[1], tests);
            atomicAdd(&cnt[2], indep);
            atomicAdd(&cnt[3], exact);
            atomicAdd(&cnt[4], nearc);
        }
        __syncthreads();
        // the level barrier: forbidden pairs leave at the end of depth 0, removals applied
        // (SkeletonDiscovery.py:141-144), removed pairs' non-empty side unions exported, the next
        // depth's neighbour lists
        if (d == 0 && a.banned)
            for (int e = tid; e < n * n; e += blockDim.x) {
                const int x = e / n, y = e - x * n;
                if (x != y && a.banned[e]) atomicOr(&rmb[x], 1ull << y);
            }
        __syncthreads();
        if (tid < n) {
            const int x = tid;
            const unsigned long long gone = rmb[x] & adjm[x];
            for (unsigned long long g = gone; g; g &= g - 1) {
                const int y = __builtin_ctzll(g);
                rlv[x * SMALL_N + y] = (int8_t)d;
                const uint64_t un = uni[x * SMALL_N + y];
                if (d >= 1 && un) {
                    const unsigned long long r = atomicAdd(&cnt[5], 1ull);
                    a.xy[2 * r] = x;
                    a.xy[2 * r + 1] = y;
                    a.bits[r] = un;
                }
            }
            adjm[x] &= ~gone;
            rmb[x] = 0;
            deg[x] = __popcll(adjm[x]);
            int c = 0;
            for (unsigned long long g = adjm[x]; g; g &= g - 1) nb[x * SMALL_N + c++] = (uint8_t)__builtin_ctzll(g);
        }
        __syncthreads();              // every export read its union word before the clear
        for (int e = tid; e < SMALL_N * SMALL_N; e += blockDim.x) uni[e] = 0;
        __syncthreads();
        if (tid == 0) {
            int64_t edges = 0;
            for (int x = 0; x < n; ++x) edges += deg[x];
            sum->tests[d] = (int64_t)cnt[1];
            sum->indep[d] = (int64_t)cnt[2];
            sum->exact[d] = (int64_t)cnt[3];
            sum->near_alpha[d] = (int64_t)cnt[4];
            sum->edges_after[d] = edges / 2;
            sum->stamp[d + 1] = wall_clock64();
            for (int k = 1; k < 5; ++k) cnt[k] = 0;
        }
        __syncthreads();
        // a singular / domain error ends the run after its depth; a full band queue (status 8:
        // this depth's decisions are incomplete) ends it at once, the host reruns on the level loop.
        // (Round 4 first broke on status & 3 only: after an overflow the block went on deciding
        // depths from incomplete removals, and on dense near-threshold graphs it kept overflowing
        // every depth up to SMALL_MAXD inside one 512-thread workgroup — a 60 s hang in a parity
        // test, fixed by breaking on the overflow itself.)
        if (status & 15) break;
    }
    for (int e = tid; e < n * n; e += blockDim.x) a.rl[e] = rlv[(e / n) * SMALL_N + e % n];
    if (tid == 0) {
        sum->levels = levels;
        sum->status = status;
        sum->xrows = (int64_t)cnt[5];
    }
}

size_t small_lds_bytes(int n) {
    return sizeof(double) * (size_t)n * n +
           sizeof(uint64_t) * (SMALL_N * SMALL_N + 3 * SMALL_N + 1 + SMALL_N * (SMALL_MAXD + 1) + SMALL_QCAP) +
           sizeof(double) * SMALL_WAVES * SMALL_SLOT + sizeof(int) * (SMALL_N + 16) + sizeof(uint16_t) * SMALL_QCAP +
           2 * SMALL_N * SMALL_N + 8 + sizeof(unsigned long long) * 8;
}

// ---------------------------------------------------------------------------------------
// host helpers
uint64_t sat_add(uint64_t a, uint64_t b) { return (a > UINT64_MAX - b) ? UINT64_MAX : a + b; }

void build_binom(pcg_handle *h, int n) {
    h->binom_h.assign((size_t)(n + 1) * PCG_BK, 0);
    for (int c = 0; c <= n; ++c) {
        h->binom_h[(size_t)c * PCG_BK] = 1;
        for (int k = 1; k < PCG_BK; ++k)
            h->binom_h[(size_t)c * PCG_BK + k] =
                c == 0 ? 0 : sat_add(h->binom_h[(size_t)(c - 1) * PCG_BK + k - 1],
                                     h->binom_h[(size_t)(c - 1) * PCG_BK + k]);
    }
}

uint64_t hbinom(const pcg_handle *h, int c, int k) {
    if (c < k || c < 0) return 0;
    return h->binom_h[(size_t)c * PCG_BK + k];
}

double threshold_r2(double alpha, double N, int d) {
    // X_alpha = Phi^-1(1 - alpha/2) via Newton on the complementary error function
    double target = alpha;                        // p(X) = erfc(X/sqrt2) == alpha
    double X = 1.96;
    for (int it = 0; it < 100; ++it) {
        const double f = std::erfc(X * PCG_SQRT1_2) - target;
        const double df = -std::sqrt(2.0 / M_PI) * std::exp(-0.5 * X * X);
        const double step = f / df;
        X -= step;
        if (std::fabs(step) < 1e-15 * std::fabs(X)) break;
    }
    const double dof = N - d - 3;
    const double r = std::tanh(X / std::sqrt(dof));
    return r * r;
}

LevelArgs make_args(pcg_handle *h, int d, int mode_exact_all) {
    LevelArgs a{};
    a.C = h->C;
    a.ldc = h->ldc;
    a.diag = (const double *)h->diag.p;
    a.adj = (const uint64_t *)h->adj.p;
    a.W = h->W;
    a.n = (int)h->n;
    a.d = d;
    a.bs = h->chunk;
    a.deg = (const int32_t *)h->deg.p;
    a.off = (const int32_t *)h->off2[h->cb].p;
    a.nbr = (const int32_t *)h->nbr2[h->cb].p;
    a.cpre = (const int64_t *)h->cpre.p;
    a.binom = (const uint64_t *)h->binom.p;
    a.rm = h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p;
    a.ug = (uint64_t *)h->ug2[h->cb].p;
    a.ctr = (DevCounters *)h->ctr.p;
    a.deferred = (DeferredEntry *)h->deferred.p;
    a.def_cap = h->def_cap;
    a.screen = (ScreenEntry *)h->screenq.p;
    a.scr_cap = h->scr_cap;
    a.records = (pcg_record *)h->records.p;
    a.rec_cap = h->rec_cap;
    a.nearl = (pcg_record *)h->nearbuf.p;
    a.near_cap = h->near_cap;
    a.alpha = h->alpha;
    const double dof = (double)h->N - d - 3;
    a.dof_negative = dof < 0;
    a.sqrt_dof = dof >= 0 ? std::sqrt(dof) : 0.0;
    if (dof > 0) {
        // cached per (alpha, N, d): the Newton solve is on the host's per-depth critical path
        if (h->thr_alpha != h->alpha || h->thr_N != h->N) {
            h->thr_alpha = h->alpha;
            h->thr_N = h->N;
            for (int k = 0; k <= PCG_MAX_LEVELS; ++k) h->thr_r2[k] = -1.0;
        }
        if (h->thr_r2[d] < 0.0) h->thr_r2[d] = threshold_r2(h->alpha, (double)h->N, d);
        const double r2 = h->thr_r2[d];
        a.lo2 = r2 * (1.0 - 1e-6);
        a.hi2 = r2 * (1.0 + 1e-6);
        a.s_amgm = 0.5 * std::sqrt(r2);
        a.inv_s = 1.0 / a.s_amgm;
    } else {
        a.lo2 = -1.0;  // never decides: every test to the exact path
        a.hi2 = 1e300;
    }
    a.tau = PCG_COND_TAU;
    a.record = (h->flags & PCG_FLAG_RECORD) ? 1 : 0;
    a.rec_mod = h->rec_mod;
    a.rec_res = h->rec_res;
    a.spl = h->spl;
    if (h->nblk) {
        a.bo = (const int64_t *)h->cpre.p + h->bo_off;
        a.cblk = (double *)h->cblk.p;
        a.lmk = (uint64_t *)h->lmk.p;
        a.img = h->nimg ? 1 : 0;
    }
    (void)mode_exact_all;
    return a;
}

template <int MODE>
void launch_level_mode(pcg_handle *h, const LevelArgs &a, int64_t nchunks, size_t lds) {
    const dim3 grid((unsigned)nchunks), block((unsigned)a.bs);
    const int d = a.d;
    if (d == 1) hipLaunchKernelGGL((k_level<1, MODE>), grid, block, lds, h->stream, a);
    else if (d == 2) hipLaunchKernelGGL((k_level<2, MODE>), grid, block, lds, h->stream, a);
    else if (d == 3) hipLaunchKernelGGL((k_level<3, MODE>), grid, block, lds, h->stream, a);
    else if (d == 4) hipLaunchKernelGGL((k_level<4, MODE>), grid, block, lds, h->stream, a);
    else if (d <= 6) hipLaunchKernelGGL((k_level<6, MODE>), grid, block, lds, h->stream, a);
    else if (d <= 8) hipLaunchKernelGGL((k_level<8, MODE>), grid, block, lds, h->stream, a);
    else hipLaunchKernelGGL((k_level<12, MODE>), grid, block, lds, h->stream, a);
}

template <int MODE>
void launch_lds_mode(pcg_handle *h, const LevelArgs &a, int64_t nchunks, size_t lds) {
    const dim3 grid((unsigned)nchunks), block(256);
    const int d = a.d;
    if (d == 1) hipLaunchKernelGGL((k_level_lds<1, MODE>), grid, block, lds, h->stream, a);
    else if (d == 2) hipLaunchKernelGGL((k_level_lds<2, MODE>), grid, block, lds, h->stream, a);
    else if (d == 3) hipLaunchKernelGGL((k_level_lds<3, MODE>), grid, block, lds, h->stream, a);
    else if (d == 4) hipLaunchKernelGGL((k_level_lds<4, MODE>), grid, block, lds, h->stream, a);
    else if constexpr (MODE != MODE_EXACT && PCG_LDS_EXACT_DM) {
        // one instantiation per depth: the per-lane Cholesky arrays sized by d, not by the bucket's
        // largest depth (k_level_lds<12> took 256 VGPRs + 1 AGPR, one wave per SIMD, at d = 9)
        if (d == 5) hipLaunchKernelGGL((k_level_lds<5, MODE>), grid, block, lds, h->stream, a);
        else if (d == 6) hipLaunchKernelGGL((k_level_lds<6, MODE>), grid, block, lds, h->stream, a);
        else if (d == 7) hipLaunchKernelGGL((k_level_lds<7, MODE>), grid, block, lds, h->stream, a);
        else if (d == 8) hipLaunchKernelGGL((k_level_lds<8, MODE>), grid, block, lds, h->stream, a);
        else if (d == 9) hipLaunchKernelGGL((k_level_lds<9, MODE>), grid, block, lds, h->stream, a);
        else if (d == 10) hipLaunchKernelGGL((k_level_lds<10, MODE>), grid, block, lds, h->stream, a);
        else if (d == 11) hipLaunchKernelGGL((k_level_lds<11, MODE>), grid, block, lds, h->stream, a);
        else if constexpr (MODE == MODE_DECIDE) {
            // beyond PCG_MAX_DEPTH (up to PCG_LDS_DEEP_TOP; use_wave sends deeper levels to the
            // one-wave-per-set kernels)
            if (d == 13) hipLaunchKernelGGL((k_level_lds<13, MODE>), grid, block, lds, h->stream, a);
            else if (d == 14) hipLaunchKernelGGL((k_level_lds<14, MODE>), grid, block, lds, h->stream, a);
            else if (d == 15) hipLaunchKernelGGL((k_level_lds<15, MODE>), grid, block, lds, h->stream, a);
            else if (d == 16) hipLaunchKernelGGL((k_level_lds<16, MODE>), grid, block, lds, h->stream, a);
#if PCG_LDS_DEEP_TOP > 16
            else if (d == 17) hipLaunchKernelGGL((k_level_lds<17, MODE>), grid, block, lds, h->stream, a);
            else if (d == 18) hipLaunchKernelGGL((k_level_lds<18, MODE>), grid, block, lds, h->stream, a);
            else if (d == 19) hipLaunchKernelGGL((k_level_lds<19, MODE>), grid, block, lds, h->stream, a);
            else if (d == 20) hipLaunchKernelGGL((k_level_lds<20, MODE>), grid, block, lds, h->stream, a);
#endif
            else hipLaunchKernelGGL((k_level_lds<12, MODE>), grid, block, lds, h->stream, a);
        } else hipLaunchKernelGGL((k_level_lds<12, MODE>), grid, block, lds, h->stream, a);
    } else {
        if (d <= 6) hipLaunchKernelGGL((k_level_lds<6, MODE>), grid, block, lds, h->stream, a);
        else if (d <= 8) hipLaunchKernelGGL((k_level_lds<8, MODE>), grid, block, lds, h->stream, a);
        else hipLaunchKernelGGL((k_level_lds<12, MODE>), grid, block, lds, h->stream, a);
    }
}

constexpr int SMALL_DEG = 64;        // LDS-resident kernels handle nodes with <= 64 neighbours
constexpr int WIDE_DEG = 128;        // ... and the T-group kernel's WIDE form nodes with <= 128

// mask_bytes: 8 (64-bit local masks) or 16 (WIDE); D rounded up to 4 (the T-group row stride)
size_t lds_small_core(int D, int mask_bytes = 8) {
 return ((size_t)D * D * 8 + (size_t)D * (2 * 8 + 3 * mask_bytes + 4) + 16 + 15) & ~(size_t)15; }
size_t lds_small_bytes(int D) { return lds_small_core(D) + (size_t)(D + 1) * 5 * 8 + 24 * 8; }
// k_level_lds_t: u32 binomial table + (g, t0) pair prefix (u32) and ids (u16)
size_t lds_tgroup_bytes(int D, int DM, int mask_bytes = 8) {
    const size_t np = (size_t)tg_pairs(D, DM);
    return lds_small_core(D, mask_bytes) + (size_t)(D + 1) * (DM + 1) * 4 + (np + 1) * 4 + np * 2 + 16;
}
// k_level_lds_f (D padded to 4): three mask arrays, fp32 M, the y records, nxs, two ints; then the
// same binomial table and task prefix as k_level_lds_t
size_t lds_f32_core(int D, int mask_bytes) {
    // (the staged region, tgf_image_bytes: M, y records of 16 B per y with 8-byte masks, 32 B with
    // 16-byte ones, nxs 4 B; then two union mask arrays and two ints)
    return ((size_t)tgf_image_bytes(D, mask_bytes) + (size_t)D * 2 * mask_bytes + 8 + 15) & ~(size_t)15;
}
size_t lds_tgroup_f_bytes(int D, int DM, int mask_bytes) {
    const size_t np = (size_t)tg_pairs(D, DM);
    return lds_f32_core(D, mask_bytes) + (size_t)(D + 1) * (DM + 1) * 4 + (np + 1) * 4 + np * 2 + 16;
}
bool use_screen32(const pcg_handle *h, int d) { return (h->screen_eff >> d) & 1; }
constexpr size_t LDS_MAX = 160 * 1024;   // gfx950 LDS per workgroup

// lane tasks of k_level_lds_t for a node of degree D at depth d (see the kernel)
uint64_t tgroup_tasks(const pcg_handle *h, int D, int d) {
    uint64_t acc = 0;
    const int TG = tg_of_depth(d);
    for (int g = 0; g * TG <= D - d; ++g) {
        const int Dp = D - g * TG - 1;
        if (Dp >= d - 1) acc += hbinom(h, Dp, d - 1);
    }
    return acc;
}

// (full-p mode too: threshold decisions with the exact band, records by the exact path — the
// p-values the caller can observe; k_level_lds_t routes recorded pairs there)
bool use_tgroup(int mode, int d) { return (mode == MODE_DECIDE || mode == MODE_FULLP) && d >= 2 && d <= 4; }
// threshold mode: the deepest depth on the per-lane k_level_lds (PCG_MAX_DEPTH .. PCG_LDS_DEEP_TOP;
// PCG_TUNE_LDS_DEEP)
int lds_deep_max(const pcg_handle *h) {
    return std::min(std::max((int)h->tune[PCG_TUNE_LDS_DEEP], PCG_MAX_DEPTH), PCG_LDS_DEEP_TOP);
}
// depths whose narrow class runs k_level_wave (one wave per conditioning set); PCG_TUNE_WAVE_LO
// sets the first such depth for every mode. tests: the level's test count bound (sum over nodes
// of C(D, d) (D - d))
bool use_wave(const pcg_handle *h, int mode, int d, double tests) {
    if (!(mode == MODE_DECIDE || mode == MODE_FULLP) || d > PCG_MAX_LEVEL_DEPTH) return false;
    const int lo = (int)h->tune[PCG_TUNE_WAVE_LO];
    if (lo > 0) return d >= std::max(lo, 5);      // explicit: the wave kernels from that depth up
    // default: the wave kernels beyond the per-lane kernel's depths (PCG_MAX_DEPTH; threshold
    // mode up to lds_deep_max(), from depth 17 on only for large levels: those instantiations
    // spill to scratch at one wave per SIMD, which loses to the wave kernels on a few thousand
    // tests — n = 500's depths 17-18: 0.05 vs 0.02 ms — and wins 2.3-2.7x on 1e9;
    // PCG_TUNE_LDS_SPILL_MIN)
    if (mode != MODE_DECIDE) return d > PCG_MAX_DEPTH;
    if (d > lds_deep_max(h)) return true;
    return d > 16 && tests < (double)h->tune[PCG_TUNE_LDS_SPILL_MIN];
}
// depth 1's large class runs k_level1_pairs (pcg_level_run); its chunks split a node's
// D(D-1)/2 neighbour pairs evenly, ~L1_PAIRS_PER_CHUNK each, so a high-degree node is spread
// over many blocks instead of a D/256-chunk tail (measured: 1024 pairs 0.36 ms, 2048 0.243,
// 4096 0.192)
#ifndef PCG_L1_PAIRS
#define PCG_L1_PAIRS 4096
#endif
#ifndef PCG_TAIL_SPIN
#define PCG_TAIL_SPIN 1      // skeleton_once's last transfer: one kernel into host-coherent memory, host spin (0: blits + sync)
#endif
#ifndef PCG_TAIL_EARLY
#define PCG_TAIL_EARLY 1     // the tail kernel queued behind the depth bound's last barrier (0: after the host read it)
#endif
#ifndef PCG_MAIN_FIRST
#define PCG_MAIN_FIRST 1     // with PCG_REST_MAIN: the main-stream (longer) class launched before the forked one
#endif
#ifndef PCG_REST_MAIN
#define PCG_REST_MAIN 0x6    // depths (bit 1 << d) whose wide / large class runs on the main stream, the narrow one on aux
#endif
#ifndef PCG_CLASS_ORDER
#define PCG_CLASS_ORDER 0
#endif
constexpr int64_t L1_PAIRS_PER_CHUNK = PCG_L1_PAIRS;
int mode_of(const pcg_handle *h, int d);
bool use_l1_pairs(const pcg_handle *h, int d) { return d == 1 && mode_of(h, d) == MODE_DECIDE && h->maxdeg <= L1_MAXD; }
int64_t l1_pair_chunks(int D) { return std::max<int64_t>(1, ((int64_t)D * (D - 1) / 2 + L1_PAIRS_PER_CHUNK - 1) / L1_PAIRS_PER_CHUNK); }

// node class of a degree-D node at depth d: 0 narrow, 1 wide (T-group depths only), 2 large
int level_class(const pcg_handle *h, int D, int d, bool tg) {
    if (h->wavek) return D <= std::min(WAVE_MAXD, h->narrow_deg) ? 0 : 2;   // k_level_wave depths
    if (D <= std::min(SMALL_DEG, h->narrow_deg) &&
        (d <= PCG_MAX_DEPTH || (mode_of(h, d) == MODE_DECIDE && d <= lds_deep_max(h))))
        return 0;
    if (tg && D <= WIDE_DEG && lds_tgroup_bytes((D + 3) & ~3, d, 16) <= LDS_MAX) return 1;
    return 2;
}

int mode_of(const pcg_handle *h, int d) {
    if ((h->flags & PCG_FLAG_EXACT_ALL) || (double)h->N - d - 3 <= 0) return MODE_EXACT;
    if (h->flags & (PCG_FLAG_FULL_P | PCG_FLAG_RECORD)) return MODE_FULLP;
    return MODE_DECIDE;
}

// the summary slot of sequence number seq (a ring of two)
LevelSummary *sum_slot(const pcg_handle *h, unsigned long long seq) {
    return reinterpret_cast<LevelSummary *>(reinterpret_cast<char *>(h->summary) + (seq & 1) * h->summary_slot);
}

// the level summary (degrees, counters, status) of the current adjacency -> host-mapped memory;
// level_wait() spins until the device has written it.
int graph_launch(pcg_handle *h) {
    const int n = (int)h->n, W = h->W;
    const size_t slot = (sizeof(LevelSummary) + sizeof(int32_t) * (size_t)n + 255) & ~(size_t)255;
    if (!h->summary || h->summary_bytes < 2 * slot) {
        if (h->summary) { (void)hipStreamSynchronize(h->stream); (void)hipHostFree(h->summary); }
        h->summary = nullptr;
        h->summary_dev = nullptr;
        h->summary_bytes = 0;
        void *p = nullptr;
        if (hipHostMalloc(&p, 2 * slot, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return pcg_fail(h, PCG_ERR_OOM, "host-mapped level summary");
        h->summary = (LevelSummary *)p;
        PCG_HIP(h, hipHostGetDevicePointer(&h->summary_dev, p, 0));
        h->summary_bytes = 2 * slot;
        h->summary_slot = slot;
        sum_slot(h, 0)->seq = 0;
        sum_slot(h, 1)->seq = 0;
        h->summary_seq = 0;
    }
    const unsigned long long seq = ++h->summary_seq;
    LevelSummary *ds = reinterpret_cast<LevelSummary *>(reinterpret_cast<char *>(h->summary_dev) + (seq & 1) * h->summary_slot);
    uint8_t *status = h->depth >= 0 ? (h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p) + (int64_t)n * n : nullptr;
    // the next depth's CSR is built from the device degrees while the host waits for the
    // summary; nbr is sized by the current graph (degrees only fall), and the union rows are
    // cleared along with it when the buffer already holds the new graph's rows (the device
    // checks that against the new degree sum; at depth 0 the bound n(n - 1) would never fit)
    const int64_t bound = h->depth < 0 ? (int64_t)n * (n - 1) : h->sumdeg;
    // the new graph's CSR goes to the other buffer set; an export still reading that set (depth
    // d - 1's) is waited for on the device first
    const int t = h->depth < 0 ? 0 : 1 - h->cb;
    if (h->xpending[t]) {
        PCG_HIP(h, hipStreamWaitEvent(h->stream, h->ev_xdone[t], 0));
        h->xpending[t] = false;
    }
    // depth 0 (the complete graph) reads no neighbour lists: init builds only the summary
    const int nfill = h->depth < 0 ? 0 : (n + 3) / 4;
    if (!pcg_ensure(h, h->off2[t], sizeof(int32_t) * (n + 1)) ||
        (nfill && !pcg_ensure(h, h->nbr2[t], sizeof(int32_t) * std::max<int64_t>(bound, 1))))
        return pcg_fail(h, PCG_ERR_OOM, "neighbour lists");
    uint64_t *ug = nullptr;
    int64_t ug_rows = 0;
    if (h->depth >= 0 && h->ug2[t].p) {
        ug = (uint64_t *)h->ug2[t].p;
        ug_rows = (int64_t)(h->ug2[t].bytes / (sizeof(uint64_t) * (size_t)W));
    }
    // the new graph's degree sum is at most the current one (exact, or its bound): a buffer that
    // holds that many rows is certainly cleared by the launch below; otherwise graph_finish takes
    // the device's verdict from the summary
    h->ug_clean2[t] = ug != nullptr && nfill > 0 && ug_rows >= h->sumdeg;
    h->ug_pend_seq = (ug && !h->ug_clean2[t]) ? seq : 0;
    h->ug_pend_set = t;
    hipLaunchKernelGGL(k_summary_fill, dim3((unsigned)(nfill + 1)), dim3(256), 0, h->stream,
                       (const int32_t *)h->deg.p, n, W, (const uint64_t *)h->adj.p, (int32_t *)h->off2[t].p,
                       (int32_t *)h->nbr2[t].p, ug, ug_rows, (DevCounters *)h->ctr.p, status, ds,
                       reinterpret_cast<int32_t *>(ds + 1), seq, nfill);
    h->cb = t;
    PCG_HIP(h, hipGetLastError());
    if (h->lev_on && !h->stamps && h->lev_n < 2 * PCG_MAX_LEVELS) {   // depth boundary (skeleton_once), off the host's critical path
        hipEvent_t &e = h->lev[h->lev_n++];
        if (!e) PCG_HIP(h, hipEventCreate(&e));
        PCG_HIP(h, hipEventRecord(e, h->stream));
    }
    return PCG_OK;
}

// skeleton_once's last device -> host transfer, one launch: the near-alpha records not yet copied
// and the sepset row counter into host-coherent memory (out[1], records from out + 8), then the
// sequence number out[0] the host spins on (no blit launches, no stream-synchronize wake-up)
// (the count of new records, out[2], from the device's cumulative near-alpha counter: the kernel
// can be queued before the host has read the last summary)
__global__ void k_tail_copy(const unsigned long long *exp_ctr, const DevCounters *ctr, const pcg_record *nearl,
                            int64_t near_seen, int64_t near_cap, unsigned long long *out, unsigned long long seq) {
    constexpr int WORDS = (int)(sizeof(pcg_record) / sizeof(uint32_t));
    const int64_t cum = min((int64_t)*reinterpret_cast<const volatile unsigned long long *>(&ctr->near_alpha), near_cap);
    const int64_t nnew = max(cum - near_seen, (int64_t)0);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(nearl + near_seen);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + 8);
    for (int64_t i = threadIdx.x; i < nnew * WORDS; i += blockDim.x) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        out[1] = exp_ctr ? *reinterpret_cast<const volatile unsigned long long *>(exp_ctr) : 0ull;
        out[2] = (unsigned long long)nnew;
        __threadfence_system();
        __atomic_store_n(&out[0], seq, __ATOMIC_RELEASE);
    }
}

// chunk prefix (host-mapped, written by the decomposition) -> device, by a kernel on the
// handle's stream (no DMA-engine round trip in the level's launch burst)
__global__ void k_copy_i64(const int64_t *src, int64_t count, int64_t *dst, DevCounters *stamp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = src[i];
    if (stamp && i == 0) stamp->t_run0 = wall_clock64();   // the kernel bracket's start (h->stamps)
}

// spin until the summary with sequence number `want` is visible (a stream error or a stream that
// finished without it ends the wait with an error instead of hanging)
int level_wait(pcg_handle *h, unsigned long long want) {
    const LevelSummary *sm = sum_slot(h, want);
    unsigned spins = 0;
    while (__atomic_load_n(&sm->seq, __ATOMIC_ACQUIRE) != want) {
        if ((++spins & 1023) == 0) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e == hipSuccess) {
                if (__atomic_load_n(&sm->seq, __ATOMIC_ACQUIRE) == want) break;
                return pcg_fail(h, PCG_ERR_HIP, "level summary not written (seq %llu)", want);
            }
            if (e != hipErrorNotReady) return pcg_fail(h, PCG_ERR_HIP, "stream error: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    return PCG_OK;
}

// after the wait: host degrees (summary `seq`) and their sum / maximum
void graph_finish(pcg_handle *h, unsigned long long seq) {
    const int n = (int)h->n;
    const int32_t *dp = reinterpret_cast<const int32_t *>(sum_slot(h, seq) + 1);
    // the union rows' state counts only while no depth has used the set since (pipelined
    // loops read the summary after level_begin_buffers has taken the set)
    if (h->ug_pend_seq == seq && seq) h->ug_clean2[h->ug_pend_set] = sum_slot(h, seq)->ug_clean != 0;
    h->deg_h.assign(dp, dp + n);
    int64_t s = 0;
    int32_t mx = 0;
    for (int i = 0; i < n; ++i) {
        s += dp[i];
        mx = std::max(mx, dp[i]);
    }
    h->sumdeg = s;
    h->maxdeg = mx;
}

size_t level_lds(const pcg_handle *h, int bs) {
    const size_t D = (size_t)h->maxdeg, W = (size_t)h->W;
    const size_t E = D + W + 2;
    return ((D * 4 + 15) & ~(size_t)15) + 2 * E * 8 + (size_t)(bs / 64) * 2 * W * 8;
}

}  // namespace

// ======================================================================================
// C ABI
extern "C" int pcg_skeleton_init(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                                 double alpha, int flags, int8_t *removed_level) {
    if (!h || !C || !removed_level || n < 2 || ldc < n || !(alpha > 0 && alpha < 1))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_skeleton_init: invalid arguments (n=%lld)", (long long)n);
    if (n > INT32_MAX / 2) return pcg_fail(h, PCG_ERR_INVALID, "n too large");
    PCG_HIP(h, hipSetDevice(h->device));
    if (h->rm_ext && h->rm_ext_bytes < n * n + PCG_RM_STATUS)
        return pcg_fail(h, PCG_ERR_INVALID, "removal buffer too small (%lld < n*n + PCG_RM_STATUS = %lld)",
                        (long long)h->rm_ext_bytes, (long long)(n * n + PCG_RM_STATUS));
    h->C = C; h->n = n; h->ldc = ldc; h->N = N; h->alpha = alpha; h->flags = flags;
    h->rl = removed_level;
    h->W = (int)((n + 63) / 64);
    h->depth = -1;
    h->deg_levels.clear();
    if (h->xs) PCG_HIP(h, hipStreamSynchronize(h->xs));   // a previous run's exports are done
    h->xpending[0] = h->xpending[1] = false;
    h->xany = false;
    h->xinl = false;
    h->cb = 0;
    h->export_rows = 0;
    export_to_own(h, 0);
    h->need_cap = 0;
    h->rec_h.clear(); h->near_h.clear();
    h->rec_total = h->near_total = 0;
    h->near_seen = h->near_total_dev = 0;
    memset(&h->st, 0, sizeof(h->st));
    const int W = h->W;
    if (!pcg_ensure(h, h->adj, sizeof(uint64_t) * n * W) || !pcg_ensure(h, h->deg, sizeof(int32_t) * n) ||
        !pcg_ensure(h, h->diag, sizeof(double) * n) || !pcg_ensure(h, h->rm, (size_t)n * n + PCG_RM_STATUS) ||
        !pcg_ensure(h, h->ctr, sizeof(DevCounters)) || !pcg_ensure(h, h->exp_ctr, sizeof(unsigned long long)) ||
        !pcg_ensure(h, h->deferred, sizeof(DeferredEntry) * h->def_cap) ||
        !pcg_ensure(h, h->screenq, sizeof(ScreenEntry) * h->scr_cap) ||
        !pcg_ensure(h, h->nearbuf, sizeof(pcg_record) * h->near_cap) ||
        !pcg_ensure(h, h->records, sizeof(pcg_record) * std::max<int64_t>(h->rec_cap, 1)))
        return pcg_fail(h, PCG_ERR_OOM, "device allocation failed (n=%lld)", (long long)n);
    if (h->binom_n != (int)n) {
        build_binom(h, (int)n);
        if (!pcg_ensure(h, h->binom, sizeof(uint64_t) * h->binom_h.size())) return PCG_ERR_OOM;
        PCG_HIP(h, hipMemcpyAsync(h->binom.p, h->binom_h.data(), sizeof(uint64_t) * h->binom_h.size(),
                                  hipMemcpyHostToDevice, h->stream));
        h->binom_n = (int)n;
    }
    hipLaunchKernelGGL(k_init, dim3(1024), dim3(256), 0, h->stream, (uint64_t *)h->adj.p, (int)n, W, C, ldc,
                       (double *)h->diag.p, (int32_t *)h->deg.p, removed_level,
                       h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p, (int64_t)n * n + PCG_RM_STATUS,
                       (unsigned long long *)h->exp_ctr.p);
    PCG_HIP(h, hipGetLastError());
    // the level counters start at zero (k_summary_fill keeps the run's near-alpha count)
    PCG_HIP(h, hipMemsetAsync(h->ctr.p, 0, sizeof(DevCounters), h->stream));
    int rc = graph_launch(h);   // also clears the counters
    if (rc) return rc;
    // the complete graph's degrees are known (k_init writes n - 1 everywhere): depth 0 is
    // decided and enqueued without waiting for this summary (the next level_wait covers it)
    h->deg_h.assign((size_t)n, (int32_t)(n - 1));
    h->sumdeg = (int64_t)n * (n - 1);
    h->maxdeg = (int32_t)(n - 1);
    return PCG_OK;
}

// the level's start-of-depth statistics from the exact degrees in h->deg_h (max degree, the
// reference's ci_test call count, the degree snapshot, the level count)
void level_start_stats(pcg_handle *h, int depth) {
    const int n = (int)h->n, maxd = h->maxdeg;
    h->deg_levels.insert(h->deg_levels.end(), h->deg_h.begin(), h->deg_h.end());
    h->st.max_degree[depth] = h->maxdeg;
    h->st.levels = depth + 1;
    std::vector<int64_t> hist(maxd + 1, 0);
    for (int x = 0; x < n; ++x) ++hist[h->deg_h[x]];
    // calls-equivalent: sum_x D_x * C(D_x - 1, d) (ci_test invocations incl. cache hits)
    int64_t calls = 0;
    for (int D = std::max(depth - 1, 0); D <= maxd; ++D) {
        if (!hist[D]) continue;
        const uint64_t c = hbinom(h, D - 1, depth);
        calls += (int64_t)std::min<uint64_t>(c, (uint64_t)INT64_MAX / 4096) * D * hist[D];
    }
    h->st.calls[depth] = calls;
}

int level_begin_buffers(pcg_handle *h, int depth);

#ifndef PCG_L1Z_EARLY
#define PCG_L1Z_EARLY 1   // k_edge_c enqueued before the level's host decomposition (1) or behind the prefix copy
#endif                    // (0: depth-1 level 0.165-0.174 vs 0.157-0.163 ms, two A/B passes on one box)
// depth 1 by conditioning node (k_level1_z) over the whole level on one rank
bool l1z_use(const pcg_handle *h, int d) {
    return d == 1 && PCG_L1Z && h->tune[PCG_TUNE_L1Z] && mode_of(h, d) == MODE_DECIDE && !(h->flags & PCG_FLAG_RECORD) && h->world == 1 &&
           l1z_lds_bytes(h->n, h->W, h->maxdeg) + 8 * L1Z_MCAP + 512 <= LDS_MAX;
}

// k_level1_z's per-edge C_xt / C_tt (into the compact-block buffer, which depth 1 does not use otherwise)
int l1z_edges(pcg_handle *h) {
    const int64_t S1 = std::max<int64_t>(h->sumdeg, 1);
    if (!pcg_ensure(h, h->cblk, 2 * sizeof(double) * (size_t)S1))
        return pcg_fail(h, PCG_ERR_OOM, "depth-1 edge correlations");
    const LevelArgs a = make_args(h, 1, false);
    double *cxe = (double *)h->cblk.p;
    hipLaunchKernelGGL(k_edge_c, dim3((unsigned)((h->n + 3) / 4)), dim3(256), 0, h->stream, a.C, a.ldc, a.deg, a.off,
                       a.nbr, (int)h->n, a.diag, cxe, cxe + S1);
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

int level_begin_impl(pcg_handle *h, int depth, int64_t *total_chunks) {
    if (!h || depth != h->depth + 1) return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_begin: depth order");
    // reference loop condition: while max_degree() - 1 > depth_prev
    if (!(h->maxdeg - 1 > depth - 1)) {
        if (total_chunks) *total_chunks = 0;
        return 1;  // done
    }
    if (depth >= PCG_MAX_LEVELS || depth > PCG_MAX_LEVEL_DEPTH)
        return pcg_fail(h, PCG_ERR_INVALID, "conditioning depth %d exceeds PCG_MAX_LEVEL_DEPTH=%d", depth,
                        PCG_MAX_LEVEL_DEPTH);
    h->depth = depth;
    const int n = (int)h->n;
    h->l1z_pre = false;
    if (PCG_L1Z_EARLY && l1z_use(h, depth)) {   // depth 1's per-edge C values run while the host decomposes
        if (int rc = l1z_edges(h)) return rc;
        h->l1z_pre = true;
    }
    level_start_stats(h, depth);
    // per-degree tables: the decomposition below is O(n) lookups (it sits between two
    // device phases of the level loop, so it is on the critical path)
    const int maxd = h->maxdeg;
    std::vector<int64_t> hist(maxd + 1, 0);
    for (int x = 0; x < n; ++x) ++hist[h->deg_h[x]];
    // work decomposition: depth 0 = one chunk per row; depth >= 1 = three node classes:
    // narrow (D <= 64: LDS-resident kernels), wide (64 < D <= 128 at the T-group depths: the
    // T-group kernel with 128-bit masks), large (the rest: staged generic kernels)
    h->cpre_h.assign(3 * (size_t)(n + 1), 0);
    int64_t *cs = h->cpre_h.data(), *cw = cs + (n + 1), *cl = cw + (n + 1);
    std::vector<int64_t> bo;           // compact-block offsets (doubles, k_node_blocks)
    h->nblk = false;
    h->nimg = false;
    h->work_h.assign(n, 0);
    h->maxdeg_small = 0;
    h->maxdeg_wide = 0;
    h->total_wide = 0;
    h->spl_w = 1;
    if (depth == 0) {
        // 64 x 64 tiles of the pair triangle; node 64*bi owns the T - bi tiles of tile row bi
        h->chunk = 256;
        h->spl = 1;
        h->tgroup = false;
        h->wavek = false;
        const int T = (n + 63) / 64;
        int64_t acc = 0;
        for (int x = 0; x <= n; ++x) {
            cs[x] = acc;
            cw[x] = 0;
            cl[x] = 0;
            if (x < n && (x & 63) == 0) acc += T - (x >> 6);
        }
        for (int x = 0; x < n; ++x) h->work_h[x] = n - 1 - x;
        h->total_small = acc;
        h->total_large = 0;
    } else {
        // small class units: T-group lane tasks (threshold mode, depth 2..4) or S ranks
        const bool tg = use_tgroup(mode_of(h, depth), depth);
        h->tgroup = tg;
        double tests_bound = 0.0;            // sum over nodes of C(D, d) (D - d)
        for (int D = depth + 1; D <= maxd; ++D) {
            if (!hist[D]) continue;
            double c = 1.0;
            for (int i = 0; i < depth; ++i) c = c * (double)(D - i) / (double)(i + 1);
            tests_bound += (double)hist[D] * c * (double)(D - depth);
        }
        h->wavek = use_wave(h, mode_of(h, depth), depth, tests_bound);
        // fp32-screened depths: PCG_TUNE_SCREEN_MASK, else pcg_set_screen_precision's choice
        const int64_t tm = h->tune[PCG_TUNE_SCREEN_MASK];
        h->screen_eff = tm >= 0 ? (int)tm : (h->screen_mask < 0 ? PCG_TG_F32 : h->screen_mask);
        h->screen_eff &= 0x1c;   // the error bound (KE = 64) is derived for d = 2..4 only
        // compact node blocks (k_node_blocks) for the narrow class of the fp32-screened sweeps
        h->nblk = tg && use_screen32(h, depth) && ((h->tune[PCG_TUNE_NODE_BLOCKS] >> depth) & 1);
        // ... as fp32 LDS images when the transposed builder's row of C fits its LDS
        h->nimg = h->nblk && PCG_NODE_IMG && PCG_NBLK_T &&
                  8 * (size_t)n + 8 * (size_t)h->W + (size_t)(maxd + 1) * (sizeof(int64_t) + 3 * sizeof(int)) <= 64 * 1024;
        std::vector<uint64_t> ns_of(maxd + 1, 0), units_of(maxd + 1, 0);
        std::vector<int> cls_of(maxd + 1, 2);
        double sum_small = 0.0, sum_wide = 0.0, sum_large = 0.0;
        int cnt_large = 0;
        for (int D = depth + 1; D <= maxd; ++D) {
            const uint64_t ns = hbinom(h, D, depth);
            if (hist[D] && ns > ((uint64_t)1 << 46))
                return pcg_fail(h, PCG_ERR_INVALID, "depth %d work too large (deg %d)", depth, D);
            ns_of[D] = ns;
            cls_of[D] = level_class(h, D, depth, tg);
            units_of[D] = cls_of[D] < 2 ? (tg ? tgroup_tasks(h, D, depth) : ns) : ns;
            if (!hist[D]) continue;
            if (cls_of[D] == 0) {
                h->maxdeg_small = D;
                sum_small += (double)units_of[D] * hist[D];
            } else if (cls_of[D] == 1) {
                h->maxdeg_wide = D;
                sum_wide += (double)units_of[D] * hist[D];
            } else {
                sum_large += (double)ns * hist[D];
                cnt_large += (int)hist[D];
            }
        }
        // narrow-class block target: ~4096 LDS-resident blocks per depth and rank, 16384 at depth
        // 4, whose long per-node task lists otherwise leave a tail (measured 2.53 -> 2.40 ms; depth
        // 3 is best at 4096); each lane walks spl units. The wide class (a few nodes) aims at ~512
        // blocks so its nodes are spread over the chip. PCG_TUNE_NB / PCG_TUNE_NBW override.
        const double nb_target = h->tune[PCG_TUNE_NB] > 0 ? (double)h->tune[PCG_TUNE_NB]
                                 : (depth == 4 ? (double)PCG_NB4_TARGET : depth == 3 ? (double)PCG_NB3_TARGET : 4096.0);
        // lanes per block: 256 S ranks / T-group tasks, or 4 conditioning sets (k_level_wave: a
        // wave each, sharing the factorisation along a wave's run of sets: longer runs there)
        const double per_block = h->wavek ? 4.0 : 256.0;
        const double spl_cap = h->wavek ? 512.0 : 64.0;
        h->spl = (int)std::min(spl_cap, std::max(1.0, std::floor(sum_small / (per_block * nb_target * h->world))));
        const double nbw_target = (double)h->tune[PCG_TUNE_NBW];
        h->spl_w = (int)std::min(64.0, std::max(1.0, std::floor(sum_wide / (256.0 * nbw_target * h->world))));
        const double mean_large = cnt_large ? sum_large / cnt_large : 0.0;
        h->chunk = (depth > PCG_MAX_DEPTH || mean_large <= 64) ? 64 : (mean_large <= 128 ? 128 : 256);
        const uint64_t csz = (uint64_t)(h->wavek ? 4 : 256) * h->spl, cszw = (uint64_t)256 * h->spl_w;
        std::vector<int64_t> nch_of(maxd + 1, 0);
        const bool l1p = use_l1_pairs(h, depth);
        for (int D = depth + 1; D <= maxd; ++D) {
            const int c = cls_of[D];
            nch_of[D] = c == 0 ? (int64_t)((units_of[D] + csz - 1) / csz)
                               : c == 1 ? (int64_t)((units_of[D] + cszw - 1) / cszw)
                                        : l1p ? l1_pair_chunks(D) : (int64_t)((ns_of[D] + h->chunk - 1) / h->chunk);
        }
        int64_t ss = 0, sw = 0, sl = 0, sb = 0;
        if (h->nblk) bo.assign(n + 1, 0);
        for (int x = 0; x < n; ++x) {
            cs[x] = ss;
            cw[x] = sw;
            cl[x] = sl;
            if (h->nblk) bo[x] = sb;
            const int D = h->deg_h[x];
            if (D < depth + 1) continue;
            h->work_h[x] = (int64_t)ns_of[D] * (D - depth);
            const int c = cls_of[D];
            (c == 0 ? ss : c == 1 ? sw : sl) += nch_of[D];
            if (h->nblk && c == 0) sb += h->nimg ? tgf_image_bytes(D, 8) / 8 : (int64_t)(D + 1) * (D + 1);
        }
        if (h->nblk) bo[n] = sb;
        cs[n] = ss;
        cw[n] = sw;
        cl[n] = sl;
        h->total_small = ss;
        h->total_wide = sw;
        h->total_large = sl;
    }
    h->total_chunks = h->total_small + h->total_wide + h->total_large;
    if (total_chunks) *total_chunks = h->total_chunks;
    // k_level_lds_f's dispatch order (narrow class): the nodes with narrow chunks by degree, largest
    // first (a counting sort), and their chunk prefix in that order — a block's time grows with D,
    // so the level's tail is made of its shortest blocks (int32, packed after the other arrays)
    h->nlpt = 0;
    std::vector<int32_t> lpt;
    if (((PCG_TGF_LPT >> depth) & 1) && depth >= 1 && h->tgroup && !h->wavek && use_screen32(h, depth) && h->total_small > 0) {
        const int64_t *cs = h->cpre_h.data();
        const int maxd = h->maxdeg;
        std::vector<int32_t> st(maxd + 2, 0);
        int m = 0;
        for (int x = 0; x < n; ++x)
            if (cs[x + 1] > cs[x]) { ++st[h->deg_h[x]]; ++m; }
        for (int D = maxd, pos = 0; D >= 0; --D) {
            const int c = st[D];
            st[D] = pos;
            pos += c;
        }
        lpt.assign(2 * (size_t)m + 1, 0);
        int32_t *nps = lpt.data(), *nord = nps + m + 1;
        for (int x = 0; x < n; ++x)
            if (cs[x + 1] > cs[x]) nord[st[h->deg_h[x]]++] = x;
        for (int i = 0; i < m; ++i) nps[i + 1] = nps[i] + (int32_t)(cs[nord[i] + 1] - cs[nord[i]]);
        h->nlpt = m;
    }
    PCG_HT(h, "begin:decomposed");
    // host-mapped upload: the three class prefixes, then (k_node_blocks) the compact-block offsets,
    // then the dispatch order
    h->bo_off = 3 * (int64_t)(n + 1);
    h->lpt_off = h->bo_off + (h->nblk ? (int64_t)(n + 1) : 0);
    const int64_t cnt = h->lpt_off + ((int64_t)lpt.size() + 1) / 2;
    if (!pcg_ensure_pinned(h, h->cpre_pin, sizeof(int64_t) * cnt))
        return pcg_fail(h, PCG_ERR_OOM, "pinned chunk prefix");
    {
        int64_t *pin = (int64_t *)h->cpre_pin.p;
        memcpy(pin, h->cpre_h.data(), sizeof(int64_t) * 3 * (n + 1));
        if (h->nblk) {
            memcpy(pin + h->bo_off, bo.data(), sizeof(int64_t) * (n + 1));
            if (!pcg_ensure(h, h->cblk, sizeof(double) * std::max<int64_t>(bo[n], 1)) ||
                !pcg_ensure(h, h->lmk, sizeof(uint64_t) * std::max<int64_t>(h->sumdeg, 1)))
                return pcg_fail(h, PCG_ERR_OOM, "compact node blocks");
        }
        if (!lpt.empty()) memcpy(pin + h->lpt_off, lpt.data(), sizeof(int32_t) * lpt.size());
    }
    if (!pcg_ensure(h, h->cpre, sizeof(int64_t) * cnt)) return PCG_ERR_OOM;
    // rm, the counters and the status bytes were cleared by the previous depth's k_level_close /
    // k_summary_fill (or at init); the union rows by k_summary_fill (or here, on first use)
    {
        const void *src = h->cpre_pin.dp;
        hipLaunchKernelGGL(k_copy_i64, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, h->stream,
                           (const int64_t *)src, cnt, (int64_t *)h->cpre.p,
                           h->stamps ? (DevCounters *)h->ctr.p : nullptr);
        PCG_HIP(h, hipGetLastError());
    }
    PCG_HT(h, "begin:prefix-copy-launched");
    // (PCG_L1Z_EARLY 0) depth 1's per-edge C values right behind the prefix copy
    if (!h->l1z_pre && l1z_use(h, depth)) {
        if (int rc = l1z_edges(h)) return rc;
        h->l1z_pre = true;
    }
    return level_begin_buffers(h, depth);
}

// the depth's union rows (cleared unless k_summary_fill already did) and, once per run, the
// sepset export buffer; sized by h->sumdeg (exact, or the bound in bound mode)
int level_begin_buffers(pcg_handle *h, int depth) {
    if (depth >= 1) {
        const size_t ugb = sizeof(uint64_t) * (size_t)std::max<int64_t>(h->sumdeg, 1) * h->W;
        DevBuf &ugb_ = h->ug2[h->cb];
        void *before = ugb_.p;
        if (!pcg_ensure(h, ugb_, ugb)) return pcg_fail(h, PCG_ERR_OOM, "sepset union rows (%zu B)", ugb);
        if (ugb_.p != before || !h->ug_clean2[h->cb]) PCG_HIP(h, hipMemsetAsync(ugb_.p, 0, ugb, h->stream));
        h->ug_clean2[h->cb] = false;
        h->ug_pend_seq = 0;
        if (depth == 1 || h->export_cap == 0) {
            // every ordered pair adjacent at depth 1 is exported at most once over all depths
            // (depth-0 removals carry empty sepsets), so one allocation covers the run
            const int64_t cap = std::max<int64_t>(h->sumdeg, 1);
            h->need_cap = cap;
            if (h->usr_xy && h->usr_bits && h->usr_cap >= cap && h->world == 1 && !h->rm_ext) {
                // the caller's buffers hold every row this run can export: no copy after the call
                h->dst_xy = h->usr_xy;
                h->dst_bits = h->usr_bits;
                h->dst_cap = h->usr_cap;
                h->dst_user = true;
                h->export_cap = cap;
            } else {
                if (!pcg_ensure(h, h->exportbuf, sizeof(uint64_t) * cap * h->W) ||
                    !pcg_ensure(h, h->export_xy, sizeof(int32_t) * 2 * cap))
                    return pcg_fail(h, PCG_ERR_OOM, "sepset export buffer");
                h->export_cap = cap;
                export_to_own(h, cap);
            }
        }
    }
    return PCG_OK;
}

extern "C" int pcg_level_begin(pcg_handle *h, int depth, int64_t *total_chunks, int32_t *max_degree,
                               uint8_t **rm_dev) {
    if (h && max_degree) *max_degree = h->maxdeg;
    if (h && rm_dev) *rm_dev = h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p;
    return level_begin_impl(h, depth, total_chunks);
}

extern "C" int pcg_set_forbidden_pairs(pcg_handle *h, const uint8_t *banned_dev) {
    if (!h) return PCG_ERR_INVALID;
    h->banned = banned_dev;
    return PCG_OK;
}

extern "C" int pcg_set_narrow_degree(pcg_handle *h, int max_degree) {
    if (!h || max_degree < 1) return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_narrow_degree: %d", max_degree);
    h->narrow_deg = max_degree;
    return PCG_OK;
}

extern "C" int pcg_set_screen_precision(pcg_handle *h, int fp32) {
    if (!h) return PCG_ERR_INVALID;
    h->screen_mask = fp32 ? -1 : 0;
    return PCG_OK;
}

extern "C" int pcg_set_world_size(pcg_handle *h, int world) {
    if (!h || world < 1) return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_world_size: world %d", world);
    h->world = world;
    return PCG_OK;
}

extern "C" int pcg_set_removal_buffer(pcg_handle *h, uint8_t *rm_dev, int64_t bytes) {
    if (!h) return PCG_ERR_INVALID;
    h->rm_ext = rm_dev;
    h->rm_ext_bytes = rm_dev ? bytes : 0;
    return PCG_OK;
}

extern "C" int pcg_level_chunk_work(pcg_handle *h, int64_t *prefix_host, int64_t capacity) {
    if (!h || !prefix_host || capacity < h->total_chunks + 1)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_chunk_work: capacity");
    const int n = (int)h->n;
    int64_t acc = 0;
    prefix_host[0] = 0;
    for (int cls = 0; cls < 3; ++cls) {
        const int64_t *cp = (const int64_t *)h->cpre_pin.p + cls * (n + 1);
        const int64_t base = cls == 0 ? 0 : cls == 1 ? h->total_small : h->total_small + h->total_wide;
        const uint64_t csz = cls == 0 ? (uint64_t)256 * h->spl : cls == 1 ? (uint64_t)256 * h->spl_w
                                                                        : (uint64_t)h->chunk;
        for (int x = 0; x < n; ++x) {
            const int64_t c0 = cp[x], c1 = cp[x + 1];
            if (c1 == c0) continue;
            if (h->depth == 0) {   // tile (x/64, x/64 + c - c0): its pair count
                const int bi = x >> 6;
                const int64_t ri = std::min<int64_t>(64, n - 64 * (int64_t)bi);
                for (int64_t c = c0; c < c1; ++c) {
                    const int bj = bi + (int)(c - c0);
                    const int64_t rj = std::min<int64_t>(64, n - 64 * (int64_t)bj);
                    acc += (bj == bi ? ri * (ri - 1) / 2 : ri * rj) + 1;
                    prefix_host[base + c + 1] = acc;
                }
                continue;
            }
            const int D = h->deg_h[x];
            if (cls == 2 && use_l1_pairs(h, h->depth)) {   // k_level1_pairs: an even share of the pairs, two tests each
                const int64_t np = (int64_t)D * (D - 1) / 2, nch = c1 - c0;
                for (int64_t c = c0; c < c1; ++c) {
                    acc += 2 * (np * (c - c0 + 1) / nch - np * (c - c0) / nch) + 1;
                    prefix_host[base + c + 1] = acc;
                }
                continue;
            }
            const bool tg = (cls < 2) && h->tgroup;
            const uint64_t ns = tg ? tgroup_tasks(h, D, h->depth) : hbinom(h, D, h->depth);
            const int64_t per_unit = (int64_t)(D - h->depth) * (tg ? tg_of_depth(h->depth) : 1);
            for (int64_t c = c0; c < c1; ++c) {
                const uint64_t r0 = (uint64_t)(c - c0) * csz;
                const uint64_t r1 = std::min<uint64_t>(r0 + csz, ns);
                acc += (int64_t)(r1 - r0) * per_unit + 1;
                prefix_host[base + c + 1] = acc;
            }
        }
    }
    return PCG_OK;
}

// contiguous, work-balanced chunk range of `rank`: the first chunk whose inclusive work
// prefix reaches total*r/world (numpy searchsorted 'left' over the prefix), as
// rcaeval_amd.dist.split_by_work computes it from pcg_level_chunk_work
extern "C" int pcg_level_split(pcg_handle *h, int rank, int world, int64_t *chunk_lo, int64_t *chunk_hi) {
    if (!h || world < 1 || rank < 0 || rank >= world || !chunk_lo || !chunk_hi)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_split: rank %d world %d", rank, world);
    const int64_t total = h->total_chunks;
    std::vector<int64_t> prefix((size_t)total + 1);
    int rc = pcg_level_chunk_work(h, prefix.data(), total + 1);
    if (rc) return rc;
    if (total <= 0) { *chunk_lo = *chunk_hi = 0; return PCG_OK; }
    const double W = (double)prefix[total];
    auto cut = [&](int r) -> int64_t {
        if (r <= 0) return 0;
        if (r >= world) return total;
        const double target = W * r / world;
        return (int64_t)(std::lower_bound(prefix.begin(), prefix.end(), target,
                                          [](int64_t v, double t) { return (double)v < t; }) - prefix.begin());
    };
    const int64_t lo = std::min(cut(rank), total), hi = std::min(std::max(cut(rank + 1), lo), total);
    *chunk_lo = lo;
    *chunk_hi = hi;
    return PCG_OK;
}

extern "C" int pcg_level_run(pcg_handle *h, int64_t chunk_lo, int64_t chunk_hi) {
    if (!h || chunk_lo < 0 || chunk_hi > h->total_chunks || chunk_lo > chunk_hi)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_run: chunk range");
    const int d = h->depth;
    const int mode = mode_of(h, d);
    const bool rec = (h->flags & PCG_FLAG_RECORD) != 0;   // T-group sweeps with record routing
    PCG_HT(h, "run:start");
    {
        LevelArgs a = make_args(h, d, mode == MODE_EXACT);
        a.chunk_lo = chunk_lo;
        const int64_t nch = chunk_hi - chunk_lo;
        hipEvent_t *rv = h->rev[d];
        // kernel bracket: timing events, or (skeleton_once) the prefix copy's and the first
        // post-class kernel's wall-clock stamps
        const bool kb = !h->stamps || d > PCG_MAX_DEPTH;
        for (int k = 0; k < 2; ++k)
            if (!rv[k]) PCG_HIP(h, hipEventCreate(&rv[k]));
        if (kb) PCG_HIP(h, hipEventRecord(rv[0], h->stream));
        if (nch > 0) {
            if (d == 0) {
                const dim3 grid((unsigned)nch), block(256);
                if (mode == MODE_DECIDE) hipLaunchKernelGGL(k_level0<MODE_DECIDE>, grid, block, 0, h->stream, a);
                else if (mode == MODE_FULLP) hipLaunchKernelGGL(k_level0<MODE_FULLP>, grid, block, 0, h->stream, a);
                else hipLaunchKernelGGL(k_level0<MODE_EXACT>, grid, block, 0, h->stream, a);
                if (h->banned && chunk_lo == 0) {
                    // background knowledge (pcg_set_forbidden_pairs): pairs forbidden in both
                    // directions leave at the end of depth 0 whatever their tests said
                    // (SkeletonDiscovery.py:86-101, stable branch). Rank 0's slice carries them
                    // into the merged flags in a sharded run.
                    const int64_t nn = (int64_t)h->n * h->n;
                    hipLaunchKernelGGL(k_or_flags, dim3((unsigned)std::min<int64_t>((nn + 255) / 256, 4096)), dim3(256), 0,
                                       h->stream, h->banned, (int64_t)h->n, a.rm);
                }
            } else if (l1z_use(h, d) && chunk_lo == 0 && chunk_hi == h->total_chunks) {
                // the whole depth by conditioning node (k_level1_z)
                if (!h->l1z_pre)
                    if (int rc = l1z_edges(h)) return rc;
                const int64_t S1 = std::max<int64_t>(h->sumdeg, 1);
                const double *cxe = (const double *)h->cblk.p, *dte = cxe + S1;
                hipLaunchKernelGGL(k_level1_z, dim3((unsigned)h->n), dim3(L1Z_BS), l1z_lds_bytes(h->n, h->W, h->maxdeg), h->stream,
                                   a, cxe, dte);
            } else {
                const int64_t S = h->total_small, Wd = h->total_wide;
                const int64_t s_lo = chunk_lo, s_hi = std::min(chunk_hi, S);
                const int64_t w_lo = std::max(chunk_lo, S) - S, w_hi = std::max(std::min(chunk_hi, S + Wd) - S, w_lo);
                const int64_t l_lo = std::max(chunk_lo, S + Wd) - (S + Wd);
                const int64_t l_hi = std::max(chunk_hi - (S + Wd), l_lo);
                // narrow and (wide or large) present: the wide / large classes run on the aux
                // stream beside the narrow class, forked after everything already on the main
                // stream and joined before the exact path
                // PCG_CLASS_ORDER (A/B): 0 narrow launched first, the wide / large classes forked
                // beside it; 1 the same with the wide / large launches first; 2 / 3 no fork (one
                // stream: narrow then the rest / the rest then narrow)
                const bool fork = PCG_CLASS_ORDER <= 1 && s_hi > s_lo && (w_hi > w_lo || l_hi > l_lo);
                hipStream_t main_stream = h->stream;
                // the fork point is the kernel bracket's start event rv[0] (or ev_fork), recorded on the
                // main stream after the prefix copy. The class expected to finish first runs on the aux
                // stream (PCG_REST_MAIN: depths whose wide / large class is the longer one run it on
                // the main stream and the narrow class on aux), so the join waits on an event that has
                // usually fired already instead of one that fires a cross-stream hop late
                const bool rest_main = fork && ((PCG_REST_MAIN >> d) & 1);
                if (fork) {
                    if (!h->aux) PCG_HIP(h, hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking));
                    if (!h->ev_join) PCG_HIP(h, hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
                    if (!kb) {   // the fork point (no timing)
                        if (!h->ev_fork) PCG_HIP(h, hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
                        PCG_HIP(h, hipEventRecord(h->ev_fork, h->stream));
                    }
                }
                auto run_narrow = [&]() -> int {
                    if (s_hi > s_lo) {
                        LevelArgs as = a;
                        as.chunk_lo = s_lo;
                        as.bs = 256;
                        const int dl = h->tgroup ? (h->maxdeg_small + 3) & ~3 : h->maxdeg_small;
                        as.lds_btab_off = (int)lds_small_core(dl);
                        size_t lds = h->tgroup ? lds_tgroup_bytes(dl, d) : lds_small_bytes(dl);
                        if (!h->tgroup && d > PCG_MAX_DEPTH)   // k_level_lds's per-wave exact-path slots
                            lds = std::max(lds, lds_small_core(dl) + 4 * sizeof(double) * WAVE_SLOT_DOUBLES(PCG_LDS_DEEP_TOP));
                        if (h->wavek) {
                            const dim3 grid((unsigned)(s_hi - s_lo)), block(256);
                            const size_t core = lds_small_core(h->maxdeg_small);
                            as.lds_btab_off = (int)core;
                            if (d <= 16) {
                                const size_t ldsw = core + 4 * sizeof(double) * (WAVE_SLOT_DOUBLES(16) + 16);
                                if (mode == MODE_DECIDE) hipLaunchKernelGGL((k_level_wave<16, MODE_DECIDE>), grid, block, ldsw, h->stream, as);
                                else hipLaunchKernelGGL((k_level_wave<16, MODE_FULLP>), grid, block, ldsw, h->stream, as);
                            } else {
                                const size_t ldsw = core + 4 * sizeof(double) * (WAVE_SLOT_DOUBLES(32) + 32);
                                if (mode == MODE_DECIDE) hipLaunchKernelGGL((k_level_wave<32, MODE_DECIDE>), grid, block, ldsw, h->stream, as);
                                else hipLaunchKernelGGL((k_level_wave<32, MODE_FULLP>), grid, block, ldsw, h->stream, as);
                            }
                        } else if (h->tgroup && use_screen32(h, d)) {
                            if (h->nblk) {   // compact node blocks: the sweep stages them instead of gathering C
                                // built transposed (C's rows staged in LDS) when a row fits
                                const size_t tl = sizeof(double) * (size_t)h->n + sizeof(uint64_t) * (size_t)h->W +
                                                  (size_t)(h->maxdeg + 1) * (sizeof(int64_t) + 3 * sizeof(int));
                                if (h->nimg)
                                    hipLaunchKernelGGL(k_node_blocks_t<true>, dim3((unsigned)h->n), dim3(256), tl, h->stream, as, s_lo,
                                                       s_hi, (int)h->maxdeg);
                                else if (PCG_NBLK_T && tl <= 64 * 1024)
                                    hipLaunchKernelGGL(k_node_blocks_t<false>, dim3((unsigned)h->n), dim3(256), tl, h->stream, as, s_lo,
                                                       s_hi, (int)h->maxdeg);
                                else
                                    hipLaunchKernelGGL(k_node_blocks, dim3((unsigned)h->n), dim3(256), 0, h->stream, as, s_lo, s_hi);
                            }
                            as.lds_btab_off = (int)lds_f32_core(dl, 8);
                            const size_t ldsf = lds_tgroup_f_bytes(dl, d, 8);
                            const dim3 grid((unsigned)(s_hi - s_lo)), block(256);
                            if (h->nlpt && s_lo == 0 && s_hi == S) {   // the whole class: largest degree first
                                as.nps = reinterpret_cast<const int32_t *>((const int64_t *)h->cpre.p + h->lpt_off);
                                as.nord = as.nps + h->nlpt + 1;
                                as.nm = h->nlpt;
                            }
                            if (d == 2) { if (rec) hipLaunchKernelGGL((k_level_lds_f<2, false, true>), grid, block, ldsf, h->stream, as); else hipLaunchKernelGGL((k_level_lds_f<2, false>), grid, block, ldsf, h->stream, as); }
                            else if (d == 3) { if (rec) hipLaunchKernelGGL((k_level_lds_f<3, false, true>), grid, block, ldsf, h->stream, as); else hipLaunchKernelGGL((k_level_lds_f<3, false>), grid, block, ldsf, h->stream, as); }
                            else { if (rec) hipLaunchKernelGGL((k_level_lds_f<4, false, true>), grid, block, ldsf, h->stream, as); else hipLaunchKernelGGL((k_level_lds_f<4, false>), grid, block, ldsf, h->stream, as); }
                        } else if (h->tgroup) {
                            const dim3 grid((unsigned)(s_hi - s_lo)), block(256);
                            if (d == 2) hipLaunchKernelGGL((k_level_lds_t<2, false>), grid, block, lds, h->stream, as);
                            else if (d == 3) hipLaunchKernelGGL((k_level_lds_t<3, false>), grid, block, lds, h->stream, as);
                            else hipLaunchKernelGGL((k_level_lds_t<4, false>), grid, block, lds, h->stream, as);
                        } else if (mode == MODE_DECIDE) launch_lds_mode<MODE_DECIDE>(h, as, s_hi - s_lo, lds);
                        else if (mode == MODE_FULLP) launch_lds_mode<MODE_FULLP>(h, as, s_hi - s_lo, lds);
                        else launch_lds_mode<MODE_EXACT>(h, as, s_hi - s_lo, lds);
                    }
                    return PCG_OK;
                };
                auto run_rest = [&]() -> int {
                    if (w_hi > w_lo) {
                        LevelArgs aw = a;
                        aw.cpre = (const int64_t *)h->cpre.p + (h->n + 1);
                        aw.chunk_lo = w_lo;
                        aw.bs = 256;
                        aw.spl = h->spl_w;
                        const int dl = (h->maxdeg_wide + 3) & ~3;
                        const dim3 grid((unsigned)(w_hi - w_lo)), block(256);
                        if (use_screen32(h, d)) {
                            aw.lds_btab_off = (int)lds_f32_core(dl, 16);
                            const size_t lds = lds_tgroup_f_bytes(dl, d, 16);
                            if (d == 2) { if (rec) hipLaunchKernelGGL((k_level_lds_f<2, true, true>), grid, block, lds, h->stream, aw); else hipLaunchKernelGGL((k_level_lds_f<2, true>), grid, block, lds, h->stream, aw); }
                            else if (d == 3) { if (rec) hipLaunchKernelGGL((k_level_lds_f<3, true, true>), grid, block, lds, h->stream, aw); else hipLaunchKernelGGL((k_level_lds_f<3, true>), grid, block, lds, h->stream, aw); }
                            else { if (rec) hipLaunchKernelGGL((k_level_lds_f<4, true, true>), grid, block, lds, h->stream, aw); else hipLaunchKernelGGL((k_level_lds_f<4, true>), grid, block, lds, h->stream, aw); }
                        } else {
                            aw.lds_btab_off = (int)lds_small_core(dl, 16);
                            const size_t lds = lds_tgroup_bytes(dl, d, 16);
                            if (d == 2) hipLaunchKernelGGL((k_level_lds_t<2, true>), grid, block, lds, h->stream, aw);
                            else if (d == 3) hipLaunchKernelGGL((k_level_lds_t<3, true>), grid, block, lds, h->stream, aw);
                            else hipLaunchKernelGGL((k_level_lds_t<4, true>), grid, block, lds, h->stream, aw);
                        }
                    }
                    if (l_hi > l_lo && d > PCG_MAX_DEPTH) {
                        LevelArgs al = a;
                        al.cpre = (const int64_t *)h->cpre.p + 2 * (h->n + 1);
                        const int64_t nch_deep = l_hi - l_lo;
                        const int grid = (int)std::min<int64_t>(nch_deep, 512);
                        const int m = d + 2;
                        const size_t per = (size_t)(m * m + 2 * m + (d + 2));
                        if (!pcg_ensure(h, h->pr_scratch, sizeof(double) * per * 64 * grid))
                            return pcg_fail(h, PCG_ERR_OOM, "deep-level scratch");
                        al.chunk_lo = l_lo;
                        hipLaunchKernelGGL(k_level_deep, dim3(grid), dim3(64), 0, h->stream, al, (double *)h->pr_scratch.p,
                                           nch_deep);
                    } else if (l_hi > l_lo) {
                        LevelArgs al = a;
                        al.cpre = (const int64_t *)h->cpre.p + 2 * (h->n + 1);
                        al.chunk_lo = l_lo;
                        const size_t lds = level_lds(h, al.bs);
                        if (lds > LDS_MAX)
                            return pcg_fail(h, PCG_ERR_INVALID, "max degree %d too large for LDS staging", h->maxdeg);
                        if (mode == MODE_DECIDE && d == 1 && h->maxdeg <= L1_MAXD)
                        {
                            const bool i32 = (int64_t)h->n * std::max<int64_t>(h->ldc, h->n) < ((int64_t)1 << 31);
                            if (i32)
                                hipLaunchKernelGGL(k_level1_pairs<true>, dim3((unsigned)(l_hi - l_lo)), dim3(256),
                                                   l1_lds_bytes(h->maxdeg), h->stream, al);
                            else
                                hipLaunchKernelGGL(k_level1_pairs<false>, dim3((unsigned)(l_hi - l_lo)), dim3(256),
                                                   l1_lds_bytes(h->maxdeg), h->stream, al);
                        }
                        else if (mode == MODE_DECIDE) launch_level_mode<MODE_DECIDE>(h, al, l_hi - l_lo, lds);
                        else if (mode == MODE_FULLP) launch_level_mode<MODE_FULLP>(h, al, l_hi - l_lo, lds);
                        else launch_level_mode<MODE_EXACT>(h, al, l_hi - l_lo, lds);
                    }
                    return PCG_OK;
                };
                // a class launched on the aux stream (h->stream swapped; restored on every exit)
                auto launch = [&](bool on_aux, auto &&fn) -> int {
                    struct StreamSwap {
                        pcg_handle *h; hipStream_t main; bool on;
                        ~StreamSwap() { if (on) h->stream = main; }
                    } swap{h, main_stream, on_aux};
                    if (on_aux) h->stream = h->aux;
                    return fn();
                };
                // (the class on the main stream is launched first: it is the longer one)
                const bool rest_first = PCG_CLASS_ORDER == 1 || PCG_CLASS_ORDER == 3 || (PCG_MAIN_FIRST && rest_main);
                const bool narrow_aux = fork && rest_main, rest_aux = fork && !rest_main;
                // the aux stream's wait on the fork point is enqueued after the main stream's first
                // launch when that class runs on the main stream (PCG_FORK_LATE): the wait's host
                // cost then lands behind a kernel that is already running
                const bool late = PCG_FORK_LATE && fork && !(rest_first ? rest_aux : narrow_aux);
                if (fork && !late) PCG_HIP(h, hipStreamWaitEvent(h->aux, kb ? rv[0] : h->ev_fork, 0));
                PCG_HT(h, "run:forked");
                int rc2 = rest_first ? launch(rest_aux, run_rest) : launch(narrow_aux, run_narrow);
                PCG_HT(h, "run:first-class");
                if (late && !rc2) PCG_HIP(h, hipStreamWaitEvent(h->aux, kb ? rv[0] : h->ev_fork, 0));
                if (!rc2) rc2 = rest_first ? launch(narrow_aux, run_narrow) : launch(rest_aux, run_rest);
                if (rc2) return rc2;
                PCG_HT(h, "run:second-class");
                if (fork) {
                    PCG_HIP(h, hipEventRecord(h->ev_join, h->aux));
                    PCG_HIP(h, hipStreamWaitEvent(main_stream, h->ev_join, 0));
                }
            }
        }
        PCG_HIP(h, hipGetLastError());
        if (kb) PCG_HIP(h, hipEventRecord(rv[1], h->stream));
        h->run_timed = kb;
        PCG_HT(h, "run:launched");
        // exact path over the deferred list; the kernel reads the list length on the device
        // (no host round trip) and raises the overflow status byte if the list overflowed
        // beyond PCG_MAX_DEPTH every kernel decides its band tests itself (k_level_wave,
        // k_level_lds's wave slots, k_level_deep): nothing is deferred, no launch
        if (d > PCG_MAX_DEPTH) return PCG_OK;
        a = make_args(h, d, mode == MODE_EXACT);
        a.stamp_end = kb ? 0 : 1;     // the first kernel behind the classes closes the bracket
        if (PCG_SCREEN_EXACT && h->tgroup && use_screen32(h, d) && !(h->flags & PCG_FLAG_RECORD)) {
            // the screen and the exact path in one launch (k_screen_exact)
            if (d == 2) hipLaunchKernelGGL(k_screen_exact<2>, dim3(256), dim3(256), 0, h->stream, a);
            else if (d == 3) hipLaunchKernelGGL(k_screen_exact<3>, dim3(256), dim3(256), 0, h->stream, a);
            else hipLaunchKernelGGL(k_screen_exact<4>, dim3(256), dim3(256), 0, h->stream, a);
            PCG_HIP(h, hipGetLastError());
            return PCG_OK;
        }
        if (h->tgroup && use_screen32(h, d)) {   // the fp32 sweep's undecided tests, in fp64
            // the list length is only known on the device; a grid-stride loop over it (1024 blocks
            // measured no faster than 256: 40 vs 36 us for 1.3e5 tests)
            if (d == 2) hipLaunchKernelGGL(k_screen<2>, dim3(256), dim3(256), 0, h->stream, a);
            else if (d == 3) hipLaunchKernelGGL(k_screen<3>, dim3(256), dim3(256), 0, h->stream, a);
            else hipLaunchKernelGGL(k_screen<4>, dim3(256), dim3(256), 0, h->stream, a);
            a.stamp_end = 0;
        }
        const int m = d + 2;
        const int per = (m * m + 2 * m) * 8;      // one LDS slot per wave
        // records: every test of a recorded pair comes here (up to ~1e6 at config 5 depth 4 with a
        // 1-in-4099 pair sample), a lane each at d <= 4; otherwise the threshold mode's few band
        // tests, a wave each
        if ((h->flags & PCG_FLAG_RECORD) && m <= 6) {
            const dim3 g(1024), b(256);
            if (m == 2) hipLaunchKernelGGL(k_exact_lanes<2>, g, b, 0, h->stream, a);
            else if (m == 3) hipLaunchKernelGGL(k_exact_lanes<3>, g, b, 0, h->stream, a);
            else if (m == 4) hipLaunchKernelGGL(k_exact_lanes<4>, g, b, 0, h->stream, a);
            else if (m == 5) hipLaunchKernelGGL(k_exact_lanes<5>, g, b, 0, h->stream, a);
            else hipLaunchKernelGGL(k_exact_lanes<6>, g, b, 0, h->stream, a);
        } else {
            hipLaunchKernelGGL(k_exact, dim3(256), dim3(256), (size_t)per * 4, h->stream, a);
        }
        PCG_HIP(h, hipGetLastError());
        return PCG_OK;
    }
}

// the level barrier of the current depth, enqueued: removals applied, the next graph's summary and
// CSR (k_summary_fill), the depth's sepset export on the export stream. Returns the summary's
// sequence number in *seq (level_end_finish waits for it).
int level_end_enqueue(pcg_handle *h, unsigned long long *seq) {
    if (!h || h->depth < 0) return pcg_fail(h, PCG_ERR_INVALID, "pcg_level_end without begin");
    const int d = h->depth, n = (int)h->n, W = h->W;
    uint8_t *rmb = h->rm_ext ? h->rm_ext : (uint8_t *)h->rm.p;
    // everything below is stream-ordered; the level costs ONE host sync: export the unions of
    // removed pairs (device-side append), apply the removals (SkeletonDiscovery.py:141-144),
    // recount degrees, and fetch counters + status + degrees in one batch
    hipLaunchKernelGGL(k_level_close, dim3((unsigned)n), dim3(256), 0, h->stream, rmb, (uint64_t *)h->adj.p,
                       (int32_t *)h->deg.p, h->rl, n, W, d);
    PCG_HIP(h, hipGetLastError());
    PCG_HT(h, "end:tail-launched");
    const int xcb = h->cb;               // depth d's CSR / union buffer set (graph_launch flips cb)
    const int64_t xsum = h->sumdeg;
    // degrees + counters + status -> host-mapped summary
    int rc = graph_launch(h);
    // graphs whose CSR holds at most PCG_TUNE_EXPORT_INLINE entries export on the handle's stream
    // the last depth of a max_depth-bounded run has no next depth to overlap its export with: it
    // runs right behind the barrier on the handle's stream (no cross-stream hop before the sync)
    const bool last = PCG_LAST_XINL && h->run_max_depth >= 0 && d >= h->run_max_depth;
    if (!rc && d >= 1 && xsum > 0 && (last || xsum <= h->tune[PCG_TUNE_EXPORT_INLINE])) {
        // a small graph's export on the handle's stream, right behind the barrier: one launch
        // instead of the export stream's four calls (it runs while the host decomposes the next
        // depth, and is done before any later launch can reuse buffer set xcb)
        hipLaunchKernelGGL(k_export, dim3((unsigned)((xsum + 255) / 256)), dim3(256), 0, h->stream,
                           (const int32_t *)h->off2[xcb].p, (const int32_t *)h->nbr2[xcb].p,
                           (const int8_t *)h->rl, d, (const uint64_t *)h->ug2[xcb].p, n, W, xsum,
                           h->dst_xy, h->dst_bits, h->dst_cap, (unsigned long long *)h->exp_ctr.p);
        PCG_HIP(h, hipGetLastError());
        h->xany = true;
        h->xinl = true;
    } else if (!rc && d >= 1 && xsum > 0) {
        // depth d's sepset export on the export stream, queued behind the barrier (removed_level
        // written); it reads buffer set xcb while the next depth runs on the other set
        if (!h->xs) PCG_HIP(h, hipStreamCreateWithFlags(&h->xs, hipStreamNonBlocking));
        if (!h->ev_xready) PCG_HIP(h, hipEventCreateWithFlags(&h->ev_xready, hipEventDisableTiming));
        if (!h->ev_xdone[xcb]) PCG_HIP(h, hipEventCreateWithFlags(&h->ev_xdone[xcb], hipEventDisableTiming));
        PCG_HIP(h, hipEventRecord(h->ev_xready, h->stream));
        PCG_HIP(h, hipStreamWaitEvent(h->xs, h->ev_xready, 0));
        hipLaunchKernelGGL(k_export, dim3((unsigned)((xsum + 255) / 256)), dim3(256), 0, h->xs,
                           (const int32_t *)h->off2[xcb].p, (const int32_t *)h->nbr2[xcb].p,
                           (const int8_t *)h->rl, d, (const uint64_t *)h->ug2[xcb].p, n, W, xsum,
                           h->dst_xy, h->dst_bits, h->dst_cap, (unsigned long long *)h->exp_ctr.p);
        PCG_HIP(h, hipEventRecord(h->ev_xdone[xcb], h->xs));
        h->xpending[xcb] = true;
        h->xany = true;
    }
    PCG_HT(h, "end:summary-launched");
    if (seq) *seq = h->summary_seq;
    return rc;
}

// wait for depth d's barrier summary (sequence number seq) and take the level's counters, status
// and the degrees of the graph that follows it (into h->deg_h / sumdeg / maxdeg)
int level_end_finish(pcg_handle *h, int d, unsigned long long seq, pcg_stats *stats) {
    int rc = level_wait(h, seq);
    if (rc) return rc;
    PCG_HT(h, "end:summary-seen");
    const LevelSummary *sm = sum_slot(h, seq);
    const DevCounters c = sm->ctr;
    if (h->stamps) {
        // depth d's boundaries: the summary before it (init's at depth 0, still in the other slot of
        // the ring, which holds seq - 1 until the next launch) and this one
        if (h->lev_stamp.empty()) {
            const LevelSummary *pv = sum_slot(h, seq - 1);
            h->lev_stamp.push_back(pv->seq == seq - 1 ? pv->stamp : 0ull);
        }
        h->lev_stamp.push_back(sm->stamp);
        if (d < PCG_MAX_LEVELS && c.t_run0 && c.t_run1 > c.t_run0 && h->wall_khz > 0)
            h->st.kernel_ms[d] = (double)(c.t_run1 - c.t_run0) / h->wall_khz;
    }
    uint8_t status[8];
    for (int k = 0; k < 8; ++k) status[k] = sm->status[k];
    if (h->rev[d][1] && !h->lev_on && h->run_timed) {   // (skeleton_once reads every depth's brackets after its last depth)
        float ms = 0.f;
        hipError_t e = hipEventElapsedTime(&ms, h->rev[d][0], h->rev[d][1]);
        if (e == hipErrorNotReady) {        // the summary can land before the runtime marks the event
            PCG_HIP(h, hipEventSynchronize(h->rev[d][1]));
            e = hipEventElapsedTime(&ms, h->rev[d][0], h->rev[d][1]);
        }
        PCG_HIP(h, e);
        h->run_ms = ms;
        h->run_timed = false;
    }
    PCG_HT(h, "end:kernel-ms-read");
    // records / near-alpha to host (parity runs; before the next level reuses the buffers)
    if ((h->flags & PCG_FLAG_RECORD) && c.records && (int64_t)c.records <= h->rec_cap) {
        const size_t old = h->rec_h.size();
        h->rec_h.resize(old + c.records);
        PCG_HIP(h, hipMemcpy(h->rec_h.data() + old, h->records.p, sizeof(pcg_record) * c.records,
                             hipMemcpyDeviceToHost));
    }
    // the device's near-alpha list accumulates over the run: this depth's entries follow the
    // ones already copied
    const int64_t near_cum = std::min<int64_t>((int64_t)c.near_alpha, h->near_cap);
    h->near_pending = near_cum;
    if (!h->defer_near && near_cum > h->near_seen) {
        const size_t old = h->near_h.size();
        h->near_h.resize(old + (near_cum - h->near_seen));
        PCG_HIP(h, hipMemcpy(h->near_h.data() + old, (pcg_record *)h->nearbuf.p + h->near_seen,
                             sizeof(pcg_record) * (near_cum - h->near_seen), hipMemcpyDeviceToHost));
    }
    const int64_t near_d = (int64_t)c.near_alpha - h->near_total_dev;
    h->near_total_dev = (int64_t)c.near_alpha;
    if (!h->defer_near) h->near_seen = std::max(h->near_seen, near_cum);
    h->st.tests[d] = (int64_t)c.tests;
    h->st.indep[d] = (int64_t)c.indep;
    h->st.exact[d] = (int64_t)c.exact;
    h->st.screened[d] = (int64_t)c.screened;
    h->st.near_alpha[d] = near_d;
    if (!h->lev_on) h->st.kernel_ms[d] = h->run_ms;
#if PCG_TGF_BLKT
    if (d == PCG_TGF_BLKT) {
        static std::vector<unsigned long long> bt(BLKT_MAX * 4), bw(4096 * 4);
        (void)hipMemcpyFromSymbol(bt.data(), HIP_SYMBOL(g_blkt), bt.size() * 8, 0, hipMemcpyDeviceToHost);
        (void)hipMemcpyFromSymbol(bw.data(), HIP_SYMBOL(g_blkw), bw.size() * 8, 0, hipMemcpyDeviceToHost);
        for (int cls = 0; cls < 2; ++cls) {
            const std::vector<unsigned long long> &v = cls ? bw : bt;
            const int nb = (int)std::min<int64_t>(cls ? h->total_wide : h->total_small, cls ? 4096 : BLKT_MAX);
            if (nb <= 0) continue;
            unsigned long long t0 = ~0ull, t1 = 0;
            double dur = 0.0;
            std::vector<unsigned long long> ends;
            double dD[8] = {}, nD[8] = {};
            for (int b = 0; b < nb; ++b) {
                const unsigned long long *e = &v[4 * b];
                if (!e[1]) continue;
                t0 = std::min(t0, e[0]);
                t1 = std::max(t1, e[1]);
                dur += (double)(e[1] - e[0]);
                ends.push_back(e[1]);
                const int k = std::min(7, (int)(e[2] / 16));
                dD[k] += (double)(e[1] - e[0]);
                nD[k] += 1.0;
            }
            std::sort(ends.begin(), ends.end());
            // concurrency: a sweep over the start / end events
            std::vector<std::pair<unsigned long long, int>> ev;
            for (int b = 0; b < nb; ++b)
                if (v[4 * b + 1]) { ev.push_back({v[4 * b], 1}); ev.push_back({v[4 * b + 1], -1}); }
            std::sort(ev.begin(), ev.end());
            int cur = 0, cmax = 0;
            for (auto &e2 : ev) { cur += e2.second; cmax = std::max(cmax, cur); }
            fprintf(stderr, "[blkt d%d %s] max concurrent blocks %d\n", d, cls ? "wide" : "narrow", cmax);
            auto q = [&](double f) { return (double)(ends[(size_t)(f * (ends.size() - 1))] - t0) / 100.0; };
            fprintf(stderr, "[blkt d%d %s] blocks %d span %.1f us  ends at 50/90/99/100%%: %.1f %.1f %.1f %.1f us  "
                    "mean block %.1f us  slot-occupancy(1024) %.2f  mean us by D/16:", d, cls ? "wide" : "narrow", nb,
                    (double)(t1 - t0) / 100.0, q(0.5), q(0.9), q(0.99), q(1.0), dur / nb / 100.0,
                    dur / 100.0 / (1024.0 * (double)(t1 - t0) / 100.0));
            for (int k = 0; k < 8; ++k)
                if (nD[k] > 0) fprintf(stderr, " %d:%.1f(%d)", k, dD[k] / nD[k] / 100.0, (int)nD[k]);
            fprintf(stderr, "\n");
        }
        std::fill(bt.begin(), bt.end(), 0ull);
        std::fill(bw.begin(), bw.end(), 0ull);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_blkt), bt.data(), bt.size() * 8, 0, hipMemcpyHostToDevice);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_blkw), bw.data(), bw.size() * 8, 0, hipMemcpyHostToDevice);
    }
#endif
#if PCG_TGF_PROF
    if (d == PCG_TGF_PROF) {
        unsigned long long pr[8] = {};
        (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_tgf_prof), sizeof(pr), 0, hipMemcpyDeviceToHost);
        fprintf(stderr, "[tgf prof d%d] waves %llu  per wave: stage %.0f setup %.0f sweep %.0f cyc; tasks/lane %.2f "
                "y/task %.1f; per wave-task setup %.0f, per wave-y sweep %.1f cyc; block %.0f cyc\n", d, pr[6],
                (double)pr[1] / pr[6], (double)pr[2] / pr[6], (double)pr[3] / pr[6], (double)pr[4] / pr[6],
                (double)pr[5] / pr[4], (double)pr[2] / pr[4], (double)pr[3] / pr[5], (double)pr[0] * 4.0 / pr[6]);
        memset(pr, 0, sizeof(pr));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tgf_prof), pr, sizeof(pr), 0, hipMemcpyHostToDevice);
    }
#endif
    if (status[3]) {   // checked first: the failed rank will not rerun, so nobody may
        if (stats) *stats = h->st;
        return pcg_fail(h, PCG_ERR_PEER, "level %d: another rank failed at this depth", d);
    }
    // the record list can also overflow inside the exact path itself (full-p mode sends every test
    // of a recorded pair there), after that kernel's own check: the summary's final count decides
    // (one GPU; a sharded run keeps the device status byte, which every rank agrees on)
    const bool rec_over = h->world == 1 && !h->rm_ext && (h->flags & PCG_FLAG_RECORD) && (int64_t)c.records > h->rec_cap;
    if (status[0] || rec_over) {
        // some rank's exact-path (or record) list overflowed: the level is incomplete on every
        // rank. Enlarge and let the driver rerun the skeleton (pcg_skeleton does it itself).
        h->def_cap = std::max<int64_t>(h->def_cap * 4, (int64_t)c.deferred * 2);
        if ((int64_t)c.screened > h->scr_cap) h->scr_cap = std::max<int64_t>(h->scr_cap * 4, (int64_t)c.screened * 2);
        if (h->flags & PCG_FLAG_RECORD) h->rec_cap = std::max<int64_t>(h->rec_cap * 4, (int64_t)c.records * 2);
        if (stats) *stats = h->st;
        return pcg_fail(h, PCG_ERR_OVERFLOW, "level %d: exact-path list overflowed; capacity raised to %lld, rerun",
                        d, (long long)h->def_cap);
    }
    if (c.error || status[1] || status[2]) {
        const bool singular = (c.error & 1) || status[1];
        h->st.error = singular ? PCG_ERR_SINGULAR : PCG_ERR_DOMAIN;
        if (stats) *stats = h->st;
        return pcg_fail(h, h->st.error,
                        singular ? "Data correlation matrix is singular. Cannot run fisherz test. Please check your data."
                                 : "math domain error");
    }
    graph_finish(h, seq);
    h->st.edges_after[d] = h->sumdeg / 2;
    PCG_HT(h, "end:done");
    if (stats) *stats = h->st;
    return PCG_OK;
}

extern "C" int pcg_level_end(pcg_handle *h, pcg_stats *stats) {
    unsigned long long seq = 0;
    int rc = level_end_enqueue(h, &seq);
    if (rc) return rc;
    return level_end_finish(h, h->depth, seq, stats);
}

// the level loop's tail (PCG_TAIL_SPIN): the exports still on the export stream joined into the
// handle's stream, then k_tail_copy (queued right behind the last depth's barrier when the depth
// bound says it is the last); the host spins on its sequence number as on a level summary
static int tail_launch(pcg_handle *h) {
    const size_t need = 64 + sizeof(pcg_record) * (size_t)std::max<int64_t>(h->near_cap, 1);
    if (h->tail_bytes < need) {
        if (h->tail) { PCG_HIP(h, hipStreamSynchronize(h->stream)); (void)hipHostFree(h->tail); }
        h->tail = h->tail_dev = nullptr;
        h->tail_bytes = 0;
        void *p = nullptr;
        if (hipHostMalloc(&p, need, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return pcg_fail(h, PCG_ERR_OOM, "host-mapped tail buffer");
        h->tail = p;
        PCG_HIP(h, hipHostGetDevicePointer(&h->tail_dev, p, 0));
        h->tail_bytes = need;
        reinterpret_cast<volatile unsigned long long *>(p)[0] = 0;
        h->tail_seq = 0;
    }
    for (int i = 0; i < 2; ++i)
        if (h->xpending[i]) PCG_HIP(h, hipStreamWaitEvent(h->stream, h->ev_xdone[i], 0));
    hipLaunchKernelGGL(k_tail_copy, dim3(1), dim3(256), 0, h->stream,
                       h->xany ? (const unsigned long long *)h->exp_ctr.p : nullptr, (const DevCounters *)h->ctr.p,
                       (const pcg_record *)h->nearbuf.p, h->near_seen, h->near_cap,
                       (unsigned long long *)h->tail_dev, ++h->tail_seq);
    PCG_HIP(h, hipGetLastError());
    return PCG_OK;
}

static int tail_wait(pcg_handle *h) {
    const unsigned long long seq = h->tail_seq;
    const unsigned long long *tw = reinterpret_cast<const unsigned long long *>(h->tail);
    unsigned spins = 0;
    while (__atomic_load_n(&tw[0], __ATOMIC_ACQUIRE) != seq) {
        if ((++spins & 1023) == 0) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e == hipSuccess) {
                if (__atomic_load_n(&tw[0], __ATOMIC_ACQUIRE) == seq) break;
                return pcg_fail(h, PCG_ERR_HIP, "tail copy not written (seq %llu)", seq);
            }
            if (e != hipErrorNotReady) return pcg_fail(h, PCG_ERR_HIP, "stream error: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    const int64_t nnew = (int64_t)tw[2];
    if (nnew > 0) {
        const pcg_record *src = reinterpret_cast<const pcg_record *>(tw + 8);
        h->near_h.insert(h->near_h.end(), src, src + nnew);
    }
    h->near_seen += nnew;
    if (h->xany) {
        const unsigned long long rows = tw[1];
        h->xany = false;
        h->xinl = false;
        h->xpending[0] = h->xpending[1] = false;
        if ((int64_t)rows > h->dst_cap)
            return pcg_fail(h, PCG_ERR_OVERFLOW, "sepset export overflow (%llu rows > %lld)", rows,
                            (long long)h->dst_cap);
        h->export_rows = (int64_t)rows;
    }
    return PCG_OK;
}

// One level-loop run's host-path state, shared by the single-GPU loop (skeleton_once) and the
// native sharded driver (comm.hip sharded_once): level d's wall time from the summaries' device
// wall-clock stamps (no timing events in the loop), the near-alpha records copied once after the
// last depth (a synchronous copy per depth that had some sat on the loop's critical path), the
// depth bound's last export on the handle's stream, and the tail kernel
void level_run_begin(pcg_handle *h, int max_depth) {
    h->htrace_on = h->tune[PCG_TUNE_HOST_TRACE] != 0;
    h->htrace.clear();
    PCG_HT(h, "init:start");
    h->lev_on = true;
    h->lev_n = 0;
    h->defer_near = true;
    h->near_pending = 0;
    h->run_max_depth = max_depth;
    h->stamps = !PCG_KBRACKET;
    h->lev_stamp.clear();
    if (h->stamps && h->wall_khz <= 0) {
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device);
        h->wall_khz = khz > 0 ? khz : 100000;
    }
}

// the depth bound's last depth: the tail transfer is queued behind its barrier right away
bool level_run_tail_early(const pcg_handle *h, int depth) {
    return PCG_TAIL_SPIN && PCG_TAIL_EARLY && h->run_max_depth >= 0 && depth >= h->run_max_depth;
}

int level_run_tail_launch(pcg_handle *h) { return tail_launch(h); }

void level_run_abort(pcg_handle *h, bool tail_queued) {
    if (tail_queued) {
        // the last depth failed after its tail kernel was queued (singular / domain / overflow /
        // a peer's failure): let that kernel finish writing the tail buffer before returning, and
        // leave no export marked pending, so no later call reads a half-written tail or stale state
        const std::string err = h->err;
        (void)tail_wait(h);
        h->err = err;
        h->xany = h->xinl = false;
        h->xpending[0] = h->xpending[1] = false;
    }
    h->lev_on = false;
    h->defer_near = false;
    h->run_max_depth = -1;
    h->stamps = false;
}

// after the last depth (done depths ran): the tail (export row count, near-alpha records) and
// the per-depth wall times
int level_run_finish(pcg_handle *h, int done, bool tail_queued) {
    int rc = PCG_OK;
    h->lev_on = false;
    h->defer_near = false;
    h->run_max_depth = -1;
    const bool stamped = h->stamps;
    h->stamps = false;
    const int64_t nnew = h->near_pending - h->near_seen;
    if (PCG_TAIL_SPIN) {
        if (!tail_queued) rc = tail_launch(h);
        if (!rc) rc = tail_wait(h);
        if (rc) return rc;
    } else if (nnew > 0) {
        if (!pcg_ensure_pinned(h, h->near_pin, sizeof(pcg_record) * (size_t)nnew))
            return pcg_fail(h, PCG_ERR_OOM, "pinned near-alpha records");
        PCG_HIP(h, hipMemcpyAsync(h->near_pin.p, (pcg_record *)h->nearbuf.p + h->near_seen,
                                  sizeof(pcg_record) * (size_t)nnew, hipMemcpyDeviceToHost, h->stream));
    }
    if (!PCG_TAIL_SPIN) rc = export_sync(h);   // the last depth's export (the skeleton's sepset rows)
    if (rc) return rc;
    if (!PCG_TAIL_SPIN && nnew > 0) {
        PCG_HIP(h, hipStreamSynchronize(h->stream));
        const pcg_record *src = (const pcg_record *)h->near_pin.p;
        h->near_h.insert(h->near_h.end(), src, src + nnew);
        h->near_seen = h->near_pending;
    }
    if (stamped) {
        for (int depth = 0; depth < done && depth + 1 < (int)h->lev_stamp.size(); ++depth) {
            const unsigned long long t0 = h->lev_stamp[depth], t1 = h->lev_stamp[depth + 1];
            if (t0 && t1 > t0) h->st.level_ms[depth] = (double)(t1 - t0) / h->wall_khz;
        }
        for (int depth = PCG_MAX_DEPTH + 1; depth < done; ++depth)   // (unstamped depths: event brackets)
            if (h->rev[depth][1]) {
                float ms = 0.f;
                PCG_HIP(h, hipEventSynchronize(h->rev[depth][1]));
                PCG_HIP(h, hipEventElapsedTime(&ms, h->rev[depth][0], h->rev[depth][1]));
                h->st.kernel_ms[depth] = ms;
            }
    } else if (done && h->lev_n > done) {
        PCG_HIP(h, hipEventSynchronize(h->lev[done]));
        for (int depth = 0; depth < done; ++depth) {
            float ms = 0.f;
            PCG_HIP(h, hipEventElapsedTime(&ms, h->lev[depth], h->lev[depth + 1]));
            h->st.level_ms[depth] = ms;
            if (h->rev[depth][1]) {     // the CI-test kernel brackets, read here, off the per-depth path
                PCG_HIP(h, hipEventElapsedTime(&ms, h->rev[depth][0], h->rev[depth][1]));
                h->st.kernel_ms[depth] = ms;
            }
        }
    }
    if (h->htrace_on && !h->htrace.empty()) {
        const double t0 = h->htrace.front().second;
        double prev = t0;
        for (auto &e : h->htrace) {
            fprintf(stderr, "[pcg host] %9.1f us  +%7.1f  %s\n", e.second - t0, e.second - prev, e.first);
            prev = e.second;
        }
    }
    return PCG_OK;
}

// The single-GPU level loop. (Round 3/4 built a pipelined form that enqueued depth d before depth
// d - 1's summary was read, and a fused one-launch level barrier; both measured slower — DESIGN §9
// — and were removed in round 5.)
static int skeleton_once(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N, double alpha,
                         int max_depth, int flags, int8_t *removed_level) {
    level_run_begin(h, max_depth);
    int rc = pcg_skeleton_init(h, C, n, ldc, N, alpha, flags, removed_level);
    if (rc) { level_run_abort(h, false); return rc; }
    PCG_HT(h, "init:done");
    int done = 0;
    bool tail_queued = false;
    for (int depth = 0;; ++depth) {
        if (max_depth >= 0 && depth > max_depth) break;
        if (depth >= PCG_MAX_LEVELS) break;   // pcg_level_begin refuses deeper levels itself
        int64_t total = 0;
        PCG_HT(h, "loop:begin");
        rc = level_begin_impl(h, depth, &total);
        if (rc == 1) break;
        if (!rc) rc = pcg_level_run(h, 0, total);
        unsigned long long seq = 0;
        if (!rc) rc = level_end_enqueue(h, &seq);
        if (!rc && level_run_tail_early(h, depth)) {
            rc = tail_launch(h);
            tail_queued = true;
        }
        if (!rc) rc = level_end_finish(h, depth, seq, nullptr);
        if (rc) { level_run_abort(h, tail_queued); return rc; }
        done = depth + 1;
    }
    return level_run_finish(h, done, tail_queued);
}

namespace {
// the small-graph path is taken for n <= SMALL_N on one rank with the handle's own removal flags
// (PCG_TUNE_SMALL = 0: the level loop for every size)
bool small_ok(const pcg_handle *h, int64_t n) {
    if (n < 2 || n > SMALL_N || h->world != 1 || h->rm_ext) return false;
    return h->tune[PCG_TUNE_SMALL] != 0;
}

// returns PCG_OK, an error, or 1: deeper than SMALL_MAXD or a full band queue (the caller reruns
// on the level loop)
int skeleton_small(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N, double alpha, int max_depth,
                   int flags, int8_t *removed_level) {
    if (!h || !C || !removed_level || n < 2 || ldc < n || !(alpha > 0 && alpha < 1))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_skeleton: invalid arguments (n=%lld)", (long long)n);
    PCG_HIP(h, hipSetDevice(h->device));
    h->C = C; h->n = n; h->ldc = ldc; h->N = N; h->alpha = alpha; h->flags = flags;
    h->rl = removed_level;
    h->W = 1;
    h->depth = -1;
    h->deg_levels.clear();
    if (h->xs) PCG_HIP(h, hipStreamSynchronize(h->xs));
    h->xpending[0] = h->xpending[1] = false;
    h->xany = false;
    h->xinl = false;
    h->export_rows = 0;
    h->rec_h.clear(); h->near_h.clear();
    h->rec_total = h->near_total = 0;
    h->near_seen = h->near_total_dev = 0;
    memset(&h->st, 0, sizeof(h->st));
    const int64_t rows = n * (n - 1);
    if (!pcg_ensure(h, h->export_xy, sizeof(int32_t) * 2 * (size_t)rows) ||
        !pcg_ensure(h, h->exportbuf, sizeof(uint64_t) * (size_t)rows) ||
        !pcg_ensure(h, h->nearbuf, sizeof(pcg_record) * h->near_cap) ||
        !pcg_ensure(h, h->records, sizeof(pcg_record) * std::max<int64_t>(h->rec_cap, 1)) ||
        !pcg_ensure(h, h->small_sum, sizeof(SmallSummary) + 128 + 32 * (SMALL_MAXD + 1)) ||
        !pcg_ensure_pinned(h, h->small_pin, sizeof(SmallSummary) + 64))
        return pcg_fail(h, PCG_ERR_OOM, "small-graph skeleton buffers (n=%lld)", (long long)n);
    h->export_cap = std::max(h->export_cap, rows);
    export_to_own(h, h->export_cap);
    if (h->binom_n != (int)n) {
        build_binom(h, (int)n);
        if (!pcg_ensure(h, h->binom, sizeof(uint64_t) * h->binom_h.size())) return PCG_ERR_OOM;
        PCG_HIP(h, hipMemcpyAsync(h->binom.p, h->binom_h.data(), sizeof(uint64_t) * h->binom_h.size(),
                                  hipMemcpyHostToDevice, h->stream));
        h->binom_n = (int)n;
    }
    SmallArgs a{};
    a.C = C; a.ldc = ldc; a.n = (int)n; a.max_depth = max_depth; a.alpha = alpha; a.tau = PCG_COND_TAU;
    a.banned = h->banned;
    a.binom = (const uint64_t *)h->binom.p;
    a.rl = removed_level;
    a.xy = (int32_t *)h->export_xy.p;
    a.bits = (uint64_t *)h->exportbuf.p;
    a.nearl = (pcg_record *)h->nearbuf.p;
    a.records = (pcg_record *)h->records.p;
    a.near_cap = h->near_cap;
    a.rec_cap = h->rec_cap;
    a.rec_mod = h->rec_mod;
    a.rec_res = h->rec_res;
    // RECORD alone records every unique test with its p: full-p mode, as the level loop (mode_of)
    a.fullp = (flags & (PCG_FLAG_FULL_P | PCG_FLAG_RECORD)) ? 1 : 0;
    a.record = (flags & PCG_FLAG_RECORD) ? 1 : 0;
    a.exact_all = (flags & PCG_FLAG_EXACT_ALL) ? 1 : 0;
    a.qcap = (int)std::min<int64_t>(std::max<int64_t>(h->tune[PCG_TUNE_SMALL_QCAP], 1), SMALL_QCAP);
    a.sum = (SmallSummary *)h->small_sum.p;
    a.ctr = reinterpret_cast<unsigned long long *>((char *)h->small_sum.p + sizeof(SmallSummary) + 8 -
                                                   (sizeof(SmallSummary) % 8));
    double cst[4 * (SMALL_MAXD + 1)];
    for (int d = 0; d <= SMALL_MAXD; ++d) {     // make_args' per-depth constants
        const double dof = (double)N - d - 3;
        cst[4 * d + 3] = dof < 0 ? 1.0 : 0.0;
        cst[4 * d + 2] = dof >= 0 ? std::sqrt(dof) : 0.0;
        if (dof > 0) {
            const double r2 = threshold_r2(alpha, (double)N, d);
            cst[4 * d] = r2 * (1.0 - 1e-6);
            cst[4 * d + 1] = r2 * (1.0 + 1e-6);
        } else {
            cst[4 * d] = -1.0;
            cst[4 * d + 1] = 1e300;
        }
    }
    double *cst_dev = reinterpret_cast<double *>((char *)a.ctr + 64);
    a.depth_cst = cst_dev;
    PCG_HIP(h, hipMemcpyAsync(cst_dev, cst, sizeof(cst), hipMemcpyHostToDevice, h->stream));
    hipEvent_t *ev = h->lev;
    for (int k = 0; k < 2; ++k)
        if (!ev[k]) PCG_HIP(h, hipEventCreate(&ev[k]));
    const SmallSummary *sm = (const SmallSummary *)h->small_pin.p;
    const unsigned long long *c2 = reinterpret_cast<const unsigned long long *>(
        (const char *)h->small_pin.p + ((const char *)a.ctr - (const char *)h->small_sum.p));
    for (int attempt = 0;; ++attempt) {
        PCG_HIP(h, hipMemsetAsync(a.ctr, 0, 2 * sizeof(unsigned long long), h->stream));
        PCG_HIP(h, hipEventRecord(ev[0], h->stream));
        hipLaunchKernelGGL(k_pc_small, dim3(1), dim3(SMALL_WAVES * 64), small_lds_bytes((int)n), h->stream, a);
        PCG_HIP(h, hipGetLastError());
        PCG_HIP(h, hipEventRecord(ev[1], h->stream));
        const size_t sb = sizeof(SmallSummary) + 64;
        PCG_HIP(h, hipMemcpyAsync(h->small_pin.p, h->small_sum.p, sb, hipMemcpyDeviceToHost, h->stream));
        PCG_HIP(h, hipStreamSynchronize(h->stream));
        if (sm->status & 12) return 1;
        // the record list overflowed (the records are of the whole run: a too small
        // record_capacity, or none set): enlarge it as the level loop does and run again
        if (!(flags & PCG_FLAG_RECORD) || (int64_t)c2[1] <= h->rec_cap) break;
        if (attempt >= 2)
            return pcg_fail(h, PCG_ERR_OVERFLOW, "record buffer overflow (%llu > %lld)", c2[1], (long long)h->rec_cap);
        h->rec_cap = std::max<int64_t>(h->rec_cap * 4, (int64_t)c2[1] * 2);
        if (!pcg_ensure(h, h->records, sizeof(pcg_record) * h->rec_cap))
            return pcg_fail(h, PCG_ERR_OOM, "record buffer (%lld)", (long long)h->rec_cap);
        a.records = (pcg_record *)h->records.p;
        a.rec_cap = h->rec_cap;
    }
    int wall_khz = 100000;            // wall_clock64's rate (kHz)
    (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, h->device);
    if (wall_khz <= 0) wall_khz = 100000;
    const int L = sm->levels;
    h->st.levels = L;
    for (int d = 0; d < L; ++d) {
        h->st.tests[d] = sm->tests[d];
        h->st.calls[d] = sm->calls[d];
        h->st.indep[d] = sm->indep[d];
        h->st.exact[d] = sm->exact[d];
        h->st.near_alpha[d] = sm->near_alpha[d];
        h->st.edges_after[d] = sm->edges_after[d];
        h->st.max_degree[d] = sm->max_degree[d];
        h->st.level_ms[d] = h->st.kernel_ms[d] = (double)(sm->stamp[d + 1] - sm->stamp[d]) / wall_khz;
        h->deg_levels.insert(h->deg_levels.end(), sm->deg[d], sm->deg[d] + n);
    }
    h->export_rows = sm->xrows;
    const int64_t nn = std::min<int64_t>((int64_t)c2[0], h->near_cap);
    if (nn > 0) {
        h->near_h.resize((size_t)nn);
        PCG_HIP(h, hipMemcpy(h->near_h.data(), h->nearbuf.p, sizeof(pcg_record) * nn, hipMemcpyDeviceToHost));
    }
    if (flags & PCG_FLAG_RECORD) {
        h->rec_h.resize((size_t)c2[1]);
        if (c2[1])
            PCG_HIP(h, hipMemcpy(h->rec_h.data(), h->records.p, sizeof(pcg_record) * c2[1], hipMemcpyDeviceToHost));
    }
    if (sm->status & 3) {
        const bool singular = sm->status & 1;
        h->st.error = singular ? PCG_ERR_SINGULAR : PCG_ERR_DOMAIN;
        return pcg_fail(h, h->st.error,
                        singular ? "Data correlation matrix is singular. Cannot run fisherz test. Please check your data."
                                 : "math domain error");
    }
    return PCG_OK;
}
}  // namespace

extern "C" int pcg_skeleton(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N, double alpha,
                            int max_depth, int flags, int8_t *removed_level, pcg_stats *stats) {
    int rc = PCG_OK;
    int driver = PCG_DRIVER_LEVELS;
    if (h && small_ok(h, n)) {
        rc = skeleton_small(h, C, n, ldc, N, alpha, max_depth, flags, removed_level);
        if (rc != 1) {
            h->st.driver = PCG_DRIVER_SMALL;
            if (stats) *stats = h->st;
            return rc;
        }
        driver = PCG_DRIVER_SMALL_RERUN;
    }
    for (int attempt = 0; attempt < 6; ++attempt) {
        rc = skeleton_once(h, C, n, ldc, N, alpha, max_depth, flags, removed_level);
        if (rc != PCG_ERR_OVERFLOW) break;
    }
    if (h) h->st.driver = driver;
    if (stats && h) *stats = h->st;
    return rc;
}

extern "C" int pcg_pc_skeleton(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C,
                               int64_t ldc, double alpha, int max_depth, int flags, int8_t *removed_level,
                               pcg_stats *stats) {
    const int rc = pcg_corr_launch(h, X, N, n, ldx, C, ldc);     // stream-ordered: no host sync between
    if (rc) return rc;
    return pcg_skeleton(h, C, n, ldc, N, alpha, max_depth, flags, removed_level, stats);
}

// wait for the queued sepset exports and take their row count (the export stream's counter)
int export_sync(pcg_handle *h) {
    if (!h->xany) return PCG_OK;
    // the row counter comes back on the export stream itself: one stream sync, no device-wide copy
    if (!pcg_ensure_pinned(h, h->ctr_pin, sizeof(unsigned long long))) return pcg_fail(h, PCG_ERR_OOM, "pinned counter");
    // exports on the handle's stream (xinl) and/or on the export stream: the counter is read
    // behind all of them
    hipStream_t s = h->xs ? h->xs : h->stream;
    if (PCG_LAST_XINL && h->xs && h->xinl) {
        // the counter is read on the handle's stream, behind the export stream's pending exports
        for (int i = 0; i < 2; ++i)
            if (h->xpending[i]) PCG_HIP(h, hipStreamWaitEvent(h->stream, h->ev_xdone[i], 0));
        s = h->stream;
    } else if (h->xs && h->xinl) {
        if (!h->ev_xready) PCG_HIP(h, hipEventCreateWithFlags(&h->ev_xready, hipEventDisableTiming));
        PCG_HIP(h, hipEventRecord(h->ev_xready, h->stream));
        PCG_HIP(h, hipStreamWaitEvent(h->xs, h->ev_xready, 0));
    }
    PCG_HIP(h, hipMemcpyAsync(h->ctr_pin.p, h->exp_ctr.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    PCG_HIP(h, hipStreamSynchronize(s));
    const unsigned long long rows = *(const unsigned long long *)h->ctr_pin.p;
    h->xany = false;
    h->xinl = false;
    h->xpending[0] = h->xpending[1] = false;
    if ((int64_t)rows > h->dst_cap)
        return pcg_fail(h, PCG_ERR_OVERFLOW, "sepset export overflow (%llu rows > %lld)", rows,
                        (long long)h->dst_cap);
    h->export_rows = (int64_t)rows;
    return PCG_OK;
}

extern "C" int pcg_set_sepset_buffers(pcg_handle *h, int32_t *xy_dev, uint64_t *bits_dev, int64_t capacity) {
    if (!h || capacity < 0 || ((xy_dev == nullptr) != (bits_dev == nullptr)))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_set_sepset_buffers: invalid arguments");
    h->usr_xy = capacity > 0 ? xy_dev : nullptr;
    h->usr_bits = capacity > 0 ? bits_dev : nullptr;
    h->usr_cap = h->usr_xy ? capacity : 0;
    return PCG_OK;
}

extern "C" int pcg_sepset_target(pcg_handle *h, int32_t *in_caller, int64_t *capacity_needed) {
    if (!h) return PCG_ERR_INVALID;
    if (in_caller) *in_caller = h->dst_user ? 1 : 0;
    if (capacity_needed) *capacity_needed = h->need_cap;
    return PCG_OK;
}

extern "C" int pcg_degrees(pcg_handle *h, int32_t *deg_host, int64_t capacity) {
    if (!h || !deg_host || capacity < (int64_t)h->deg_levels.size())
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_degrees: capacity %lld < %zu", (long long)capacity,
                        h ? h->deg_levels.size() : 0);
    memcpy(deg_host, h->deg_levels.data(), sizeof(int32_t) * h->deg_levels.size());
    return PCG_OK;
}

extern "C" int pcg_sepset_count(pcg_handle *h, int64_t *count, int32_t *words_per_row) {
    if (!h) return PCG_ERR_INVALID;
    const int rc = export_sync(h);
    if (rc) return rc;
    if (count) *count = h->export_rows;
    if (words_per_row) *words_per_row = h->W;
    return PCG_OK;
}

extern "C" int pcg_sepset_export(pcg_handle *h, int32_t *xy_host, uint64_t *bits_host, int64_t count) {
    if (!h) return PCG_ERR_INVALID;
    const int rc = export_sync(h);
    if (rc) return rc;
    if (count > h->export_rows) return pcg_fail(h, PCG_ERR_INVALID, "pcg_sepset_export: count");
    if (count == 0) return PCG_OK;
    PCG_HIP(h, hipMemcpy(xy_host, h->dst_xy, sizeof(int32_t) * 2 * count, hipMemcpyDeviceToHost));
    PCG_HIP(h, hipMemcpy(bits_host, h->dst_bits, sizeof(uint64_t) * count * h->W, hipMemcpyDeviceToHost));
    return PCG_OK;
}

extern "C" int pcg_sepset_export_device(pcg_handle *h, int32_t *xy_dev, uint64_t *bits_dev, int64_t count) {
    if (!h) return PCG_ERR_INVALID;
    const int rc = export_sync(h);
    if (rc) return rc;
    if (count > h->export_rows) return pcg_fail(h, PCG_ERR_INVALID, "pcg_sepset_export_device: count");
    if (count == 0) return PCG_OK;
    if (xy_dev != h->dst_xy)
        PCG_HIP(h, hipMemcpyAsync(xy_dev, h->dst_xy, sizeof(int32_t) * 2 * count, hipMemcpyDeviceToDevice, h->stream));
    if (bits_dev != h->dst_bits)
        PCG_HIP(h, hipMemcpyAsync(bits_dev, h->dst_bits, sizeof(uint64_t) * count * h->W, hipMemcpyDeviceToDevice,
                                  h->stream));
    return PCG_OK;
}

extern "C" int pcg_record_count(pcg_handle *h, int64_t *count, int64_t *near_count) {
    if (!h) return PCG_ERR_INVALID;
    if (count) *count = (int64_t)h->rec_h.size();
    if (near_count) *near_count = (int64_t)h->near_h.size();
    return PCG_OK;
}

extern "C" int pcg_record_export(pcg_handle *h, pcg_record *rec_host, int64_t count, pcg_record *near_host,
                                 int64_t near_count) {
    if (!h || count > (int64_t)h->rec_h.size() || near_count > (int64_t)h->near_h.size())
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_record_export: count");
    if (count) memcpy(rec_host, h->rec_h.data(), sizeof(pcg_record) * count);
    if (near_count) memcpy(near_host, h->near_h.data(), sizeof(pcg_record) * near_count);
    return PCG_OK;
}
