// handle.h — engine handle shared by the HIP translation units of libpcgpu.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include <chrono>

#include "pcgpu.h"

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

struct PinBuf {                    // page-locked host staging (async per-level transfers)
    void *p = nullptr;
    void *dp = nullptr;            // its device address (hipHostMallocMapped), queried once
    size_t bytes = 0;
};

// Device-side counters of one level (zeroed by pcg_level_begin).
struct DevCounters {
    unsigned long long tests;      // unique tests evaluated
    unsigned long long indep;      // unique tests with p > alpha
    unsigned long long deferred;   // tests pushed to the exact path (may exceed capacity)
    unsigned long long exact;      // tests resolved by the exact path
    unsigned long long records;    // records written (may exceed capacity)
    unsigned long long near_alpha; // |p - alpha| < 1e-9 (may exceed capacity)
    unsigned long long exported;   // sepset rows exported this level
    unsigned long long error;      // PCG_ERR_* bits (1 singular, 2 domain)
    unsigned long long screened;   // tests the fp32 sweep handed to the fp64 screen list (may exceed capacity)
    // skeleton_once's kernel bracket in device wall-clock ticks: after the chunk-prefix copy, at the
    // start of the first kernel behind the CI-test classes (0: not stamped)
    unsigned long long t_run0, t_run1;
};

// host-mapped per-level summary (k_level_summary); n int32 degrees follow the struct
struct LevelSummary {
    DevCounters ctr;
    uint8_t status[8];
    int32_t ug_clean;              // k_summary_fill cleared every union row of the new graph
    unsigned long long stamp;      // device wall-clock ticks when the summary was written
    unsigned long long seq;        // written last, after a system-scope fence
};

struct ScreenEntry {               // one test the fp32 sweep could not decide (k_screen: fp64)
    int32_t x, y;
    int32_t s[4];                  // conditioning set (global ids, ascending), depths 2..4
};

struct DeferredEntry {             // one test routed to the exact (LU) path
    int32_t x, y;                  // visiting node x, neighbour y
    int32_t s[PCG_MAX_DEPTH];      // conditioning set (global ids)
};

inline double pcg_now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define PCG_HT(h, label) \
    do { if ((h)->htrace_on) (h)->htrace.emplace_back((label), pcg_now_us()); } while (0)

struct pcg_handle {
    int device = 0;
    int64_t tune[PCG_TUNE_COUNT] = {};   // pcg_set_tuning knobs (defaults from the environment at pcg_create)
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t lev[2 * PCG_MAX_LEVELS] = {};   // depth-boundary events (skeleton_once), read after the last depth
    bool lev_on = false;
    int lev_n = 0;

    // scratch
    DevBuf screenq;                 // fp32 sweep -> fp64 screen list (k_level_lds_f -> k_screen)
    DevBuf adj, deg, rm, cpre, binom, ctr, deferred, records, nearbuf, exportbuf, export_xy, diag, colmean,
        pr_scratch, batch_scratch, chisq_scratch;
    DevBuf k1_digits;               // K1 int8 digit / residue planes of the centred X (corr.hip)
    // the (N, n, k, b) a CRT-mode pcg_corr_shard computed h->colmean's column exponents for;
    // pcg_corr_shard_finish refuses to rebuild C from exponents of any other call
    int64_t k1_stamp[4] = {0, 0, 0, 0};
    bool k1_stamp_ok = false;
    // CSR (offsets, neighbour lists) and sepset union rows, double-buffered: depth d's sepset
    // export reads buffer set cb on the export stream while depth d + 1 runs on set 1 - cb
    DevBuf off2[2], nbr2[2], ug2[2];
    int cb = 0;                      // buffer set of the current graph
    bool ug_clean2[2] = {false, false};   // the union rows of set i's CSR are all zero
    unsigned long long ug_pend_seq = 0;   // summary whose ug_clean still applies to set ug_pend_set
    int ug_pend_set = 0;
    hipStream_t xs = nullptr;        // sepset export stream
    hipEvent_t ev_xready = nullptr, ev_xdone[2] = {nullptr, nullptr};
    bool xpending[2] = {false, false};    // an export reading set i is queued on xs
    bool xany = false;               // exports queued since the last export_sync
    bool xinl = false;               // ... some of them on the handle's stream (small graphs)
    DevBuf exp_ctr;                  // rows exported so far (device, persists across depths)
    PinBuf ctr_pin, deg_pin, off_pin, cpre_pin, status_pin;
    DevBuf small_sum;                // single-workgroup small-graph skeleton: summary + counters
    PinBuf small_pin;                // its host copy
    std::vector<uint64_t> binom_h;   // host copy of the binomial table
    uint8_t *rm_ext = nullptr;       // caller-owned removal-flag buffer (multi-GPU)
    const uint8_t *banned = nullptr; // pcg_set_forbidden_pairs: n x n pairs removed at depth 0
    int64_t rm_ext_bytes = 0;
    int64_t rec_cap = 0, def_cap = 1 << 20, near_cap = 1 << 16, scr_cap = 1 << 20;
    int64_t rec_mod = 0, rec_res = 0;  // pcg_set_record_sample (0/1 = record every test)
    int64_t export_cap = 0;          // rows
    int64_t export_rows = 0;         // rows exported so far (host mirror)
    // where this run's sepset rows go (pcg_set_sepset_buffers): the caller's device buffers when
    // they hold the run's row bound (one GPU), else the handle's own exportbuf / export_xy
    int32_t *usr_xy = nullptr;
    uint64_t *usr_bits = nullptr;
    int64_t usr_cap = 0;
    int32_t *dst_xy = nullptr;
    uint64_t *dst_bits = nullptr;
    int64_t dst_cap = 0;
    bool dst_user = false;
    int64_t need_cap = 0;            // this run's row bound (the ordered pairs entering depth 1)
    int binom_n = -1;                // binom table built for 0..binom_n

    // skeleton state (single-GPU and level-step API)
    const double *C = nullptr;
    int64_t n = 0, ldc = 0, N = 0;
    int W = 0;
    double alpha = 0.05;
    int flags = 0;
    int8_t *rl = nullptr;
    int depth = -1;                  // depth prepared by level_begin
    int64_t total_chunks = 0;        // narrow + wide + large class chunks of the current depth
    int64_t total_small = 0, total_wide = 0, total_large = 0;
    int chunk = 256;                 // block size of the staged (large-degree) kernel
    int spl = 1;                     // S ranks per lane of the LDS-resident kernel
    int world = 1;                   // ranks sharing each level's work list (pcg_set_world_size)
    int32_t maxdeg_small = 0;        // largest degree handled by the LDS-resident kernel
    int32_t maxdeg_wide = 0;         // largest degree of the wide (128-bit mask) T-group class
    int spl_w = 1;                   // tasks per lane of the wide class
    int narrow_deg = 64;             // pcg_set_narrow_degree (testing: route more nodes to the wide class)
    bool tgroup = false;             // small class runs k_level_lds_t this depth
    bool wavek = false;              // small class runs k_level_wave this depth (deep levels)
    bool nblk = false;               // small class stages per-node compact blocks (k_node_blocks) this depth
    bool l1z_pre = false;            // depth 1's per-edge C values (k_edge_c) enqueued by pcg_level_begin
    bool nimg = false;               // ... as fp32 LDS images of k_level_lds_f (k_node_blocks_t<true>)
    DevBuf cblk, lmk;                // k_node_blocks: per-node compact correlation blocks, local masks
    int64_t bo_off = 0;              // int64 offset of the compact-block offsets in cpre / cpre_pin
    int64_t lpt_off = 0;             // ... of k_level_lds_f's dispatch order (int32 nps, then nord)
    int nlpt = 0;                    // nodes in that order (0: canonical order)
    hipEvent_t rev[PCG_MAX_LEVELS][2] = {};   // per-depth CI-test kernel brackets
    int64_t near_seen = 0;           // near-alpha entries copied so far (the device list accumulates)
    int64_t near_total_dev = 0;      // the device's cumulative near-alpha count at the last level end
    int64_t near_pending = 0;        // the device list's length (capped) at the last level end
    bool defer_near = false;         // skeleton_once: near-alpha records copied once after the last depth
    PinBuf near_pin;                 // their host staging
    int run_max_depth = -1;          // skeleton_once's max_depth (-1: unbounded, or the level-step API)
    // skeleton_once's depth boundaries (the summaries' wall-clock stamps; PCG_KBRACKET = 0)
    std::vector<unsigned long long> lev_stamp;
    bool stamps = false;
    int wall_khz = 0;
    hipEvent_t ev_fork = nullptr;    // the class fork point when the kernel brackets are stamped
    // skeleton_once's last device -> host transfer (k_tail_copy): host-coherent, mapped
    void *tail = nullptr, *tail_dev = nullptr;
    size_t tail_bytes = 0;
    unsigned long long tail_seq = 0;
    size_t summary_slot = 0;         // bytes per slot of the two-slot host-mapped summary ring
    int screen_eff = 0;              // the current depth's effective mask (set by pcg_level_begin)
    int screen_mask = -1;            // depths (bit 1 << d) with the fp32-screened T-group sweep (k_level_lds_f); -1 = default
    int32_t maxdeg = 0;
    int64_t sumdeg = 0;
    LevelSummary *summary = nullptr;    // host-mapped, coherent (graph_launch / level_wait)
    void *summary_dev = nullptr;        // its device address, queried once at allocation
    size_t summary_bytes = 0;
    unsigned long long summary_seq = 0;
    // PCG_TUNE_HOST_TRACE: host timestamps of the level loop's steps, printed after each skeleton
    bool htrace_on = false;
    std::vector<std::pair<const char *, double>> htrace;
    std::vector<int32_t> deg_h;      // degrees at the start of the current depth
    std::vector<int32_t> deg_levels; // levels x n
    std::vector<int64_t> cpre_h;     // 3 x (n + 1): narrow, wide, large class chunk prefixes
    std::vector<int64_t> work_h;     // per-node tests estimate
    std::vector<pcg_record> rec_h, near_h;
    int64_t rec_total = 0, near_total = 0;
    pcg_stats st{};
    double thr_alpha = -1.0, thr_N = -1.0;   // threshold_r2 cache (make_args)
    double thr_r2[PCG_MAX_LEVELS + 1] = {};
    float run_ms = 0.f;              // CI-test kernel time of the current level
    bool run_timed = false;          // ev[2]/ev[3] bracket this level's CI-test kernels

    // second stream: a depth's large-degree class runs beside its LDS-resident class
    hipStream_t aux = nullptr;
    hipEvent_t ev_join = nullptr;

    // the native sharded driver's transport (comm.hip): an RCCL communicator (pcg_comm_init), or
    // a pcg_comm_group of handles in this process (pcg_comm_init_group); comm_ops its collectives
    void *comm = nullptr;
    const struct CommOps *comm_ops = nullptr;
    int comm_rank = 0, comm_world = 1;
    DevBuf comm_rm, comm_packed, comm_gathered, comm_small;
    DevBuf comm_status;   // agree(): one int32 all-reduced with MAX, allocated before the communicator
    // the native driver's set-up agreements (comm.hip): the (n, N, world, plan signature) of the last
    // agreed sharded K1 and the (n, world) of the last agreed skeleton set-up. A call that matches
    // and allocates nothing skips the agreement's host round trip (every rank makes the same calls,
    // so every rank skips it together); any allocation or a new tuple agrees again
    int64_t k1_agreed[4] = {-1, -1, -1, 0};
    int64_t sk_agreed[2] = {-1, -1};
    uint64_t alloc_events = 0;       // device / pinned allocations made by pcg_ensure*, ever
};

void pcg_comm_release(pcg_handle *h);      // comm.hip: destroy the communicator, free its buffers
// corr.hip: K1 queued on h->stream without the host sync of pcg_corr (pcg_pc_skeleton)
int export_sync(pcg_handle *h);   // skeleton.hip: wait for the sepset exports, take their row count
int pcg_corr_launch(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C, int64_t ldc);
int64_t k1_plan_signature(const pcg_handle *h, int64_t n, int64_t N);   // corr.hip: K1's plan, for cross-rank agreement
// corr.hip: the native sharded K1's CRT path without host syncs (see corr.hip)
int corr_shard_crt_prepare(pcg_handle *h, int64_t N, int64_t n, int world, bool *crt, int64_t *unit_bytes);
int corr_shard_crt_enqueue(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, int rank, int world,
                           double *packed);
int corr_shard_crt_finish_enqueue(pcg_handle *h, const double *gathered, int64_t N, int64_t n, double *C, int64_t ldc);
// skeleton.hip: one level-loop run's host-path state (device-clock depth stamps, near-alpha records
// once after the last depth, the depth bound's last export on the handle's stream, the tail
// kernel), shared by pcg_skeleton's loop and the native sharded driver
void level_run_begin(pcg_handle *h, int max_depth);
bool level_run_tail_early(const pcg_handle *h, int depth);   // queue the tail behind this depth's barrier?
int level_run_tail_launch(pcg_handle *h);
void level_run_abort(pcg_handle *h, bool tail_queued);
int level_run_finish(pcg_handle *h, int done, bool tail_queued);
int level_end_enqueue(pcg_handle *h, unsigned long long *seq);
int level_end_finish(pcg_handle *h, int d, unsigned long long seq, pcg_stats *stats);
void pcg_tuning_defaults(int64_t *tune);   // api.hip: the built-in values, overridden by the environment

// the run's sepset rows go to the handle's own export buffers (capacity cap rows); called again
// whenever those buffers are (re)allocated
inline void export_to_own(pcg_handle *h, int64_t cap) {
    h->dst_xy = (int32_t *)h->export_xy.p;
    h->dst_bits = (uint64_t *)h->exportbuf.p;
    h->dst_cap = cap;
    h->dst_user = false;
}

int pcg_fail(pcg_handle *h, int code, const char *fmt, ...);
bool pcg_ensure(pcg_handle *h, DevBuf &b, size_t bytes);   // grow-only allocation
bool pcg_ensure_pinned(pcg_handle *h, PinBuf &b, size_t bytes);   // grow-only, page-locked

#define PCG_HIP(h, expr)                                                                    \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return pcg_fail((h), PCG_ERR_HIP, "%s failed: %s (%s:%d)", #expr,               \
                            hipGetErrorString(_e), __FILE__, __LINE__);                     \
    } while (0)
