// comm.hip — native multi-GPU driver of libpcgpu.so: RCCL over xGMI, one process per GPU.
//
// each PC depth's work list is split by work across the ranks (the same
// pcg_level_split cut as the Python driver in rcaeval_amd/dist.py), every rank evaluates its
// owner-disjoint chunk range, and the removal flags + status are merged with ONE all-gather of
// bit-packed upper-triangle flags on the handle's stream (barrier.hip: RCCL has no bitwise OR,
// so every rank ORs the gathered copies itself) before pcg_level_end applies them identically
// everywhere. The loop runs in C: no host-language round trip between the per-depth steps.
//
// The driver's collectives go through a per-handle transport table (CommOps):
//  * RCCL (pcg_comm_init, the default): resolved at run time — first the copy the process has
//    already loaded (PyTorch ships one), else librccl.so.1 — so a process that also uses
//    torch.distributed holds one RCCL;
//  * an in-process group of handles (pcg_comm_group_create / pcg_comm_init_group): host-staged
//    collectives between handles driven from separate threads of one process. RCCL refuses two
//    ranks on one device (rccl.h ncclCommInitRank: "each rank must use a different device"), so
//    this is how the rank-dependent code of the driver (the level split, the packed all-gather
//    + merge, the stats all-reduce, the sepset gathers) runs at world 2..8 on one GPU. The group
//    also checks that every rank issues the same collective (kind, size) in the same order — the
//    mismatch RCCL would hang on — and fails all ranks with PCG_ERR_RCCL when they do not.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "handle.h"

enum CommType { COMM_I32, COMM_I64 };
enum CommOp { COMM_MAX, COMM_SUM };

// the collectives of the native driver, on the handle's stream (RCCL) or completed on return
// (group). all_gather: `bytes` per rank, rank-major into recv; all_reduce: in place.
struct CommOps {
    const char *name;
    int (*all_gather)(pcg_handle *h, const void *send, void *recv, size_t bytes);
    int (*all_reduce)(pcg_handle *h, void *buf, size_t count, CommType t, CommOp op);
    void (*release)(pcg_handle *h);
};

namespace {

struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *lib = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so"}) {
            lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);          // already in the process?
            if (lib) break;
        }
        if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!lib) lib = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!lib) {
            r.err = std::string("librccl not found: ") + dlerror();
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(lib, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(lib, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(lib, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(lib, "ncclAllReduce");
        r.all_gather = (decltype(r.all_gather))dlsym(lib, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(lib, "ncclGetErrorString");
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.all_gather &&
               r.error_string;
        if (!r.ok) r.err = "librccl lacks an expected symbol";
    });
    return r;
}

#define PCG_NCCL(h, expr)                                                                   \
    do {                                                                                    \
        ncclResult_t _r = (expr);                                                           \
        if (_r != ncclSuccess)                                                              \
            return pcg_fail((h), PCG_ERR_RCCL, "%s failed: %s", #expr, rccl().error_string(_r)); \
    } while (0)

// ---- RCCL transport -------------------------------------------------------------------
int rccl_all_gather(pcg_handle *h, const void *send, void *recv, size_t bytes) {
    PCG_NCCL(h, rccl().all_gather(send, recv, bytes, ncclUint8, (ncclComm_t)h->comm, h->stream));
    return PCG_OK;
}

int rccl_all_reduce(pcg_handle *h, void *buf, size_t count, CommType t, CommOp op) {
    PCG_NCCL(h, rccl().all_reduce(buf, buf, count, t == COMM_I32 ? ncclInt32 : ncclInt64,
                                  op == COMM_MAX ? ncclMax : ncclSum, (ncclComm_t)h->comm, h->stream));
    return PCG_OK;
}

void rccl_release(pcg_handle *h) {
    if (h->comm && rccl().ok) rccl().comm_destroy((ncclComm_t)h->comm);
}

const CommOps kRcclOps = {"rccl", rccl_all_gather, rccl_all_reduce, rccl_release};

}  // namespace

// ---- in-process group transport ---------------------------------------------------------
// One slot of host memory per rank. A collective: each rank copies its device operand into its
// slot (stream-synchronised), all ranks meet at a barrier, each rank reads every slot (gather:
// concatenates, reduce: combines in rank order) and copies the result to its device buffer, and
// all ranks meet again before any slot is reused. A barrier that waits longer than the group's
// timeout, or a rank that fails inside a collective, breaks the group: every waiting and later
// collective returns PCG_ERR_RCCL instead of hanging.
struct pcg_comm_group {
    int world = 1;
    double timeout_s = 300.0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::string why;
    std::vector<std::vector<unsigned char>> slot;
    std::vector<uint64_t> tag;          // per rank: the collective it is in (kind, type, op, bytes)
    std::vector<pcg_handle *> member;
    int64_t collectives = 0;            // completed collectives (counted once per group)
    int64_t bytes = 0;                  // bytes contributed by all ranks over them
};

namespace {

void group_break(pcg_comm_group *g, const std::string &why) {
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->broken) {
        g->broken = true;
        g->why = why;
    }
    g->cv.notify_all();
}

// 0, or -1 when the group is (or becomes) broken
int group_barrier(pcg_comm_group *g) {
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->broken) return -1;
    const uint64_t my = g->gen;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return 0;
    }
    const bool done = g->cv.wait_for(lk, std::chrono::duration<double>(g->timeout_s),
                                     [&] { return g->gen != my || g->broken; });
    if (g->gen != my) return 0;
    if (!done && !g->broken) {
        g->broken = true;
        g->why = "a rank did not reach the collective within the group's timeout";
        g->cv.notify_all();
    }
    return -1;
}

int group_fail(pcg_handle *h, pcg_comm_group *g) {
    std::lock_guard<std::mutex> lk(g->mu);
    return pcg_fail(h, PCG_ERR_RCCL, "in-process group collective failed: %s",
                    g->why.empty() ? "group broken" : g->why.c_str());
}

uint64_t group_tag(int kind, int t, int op, size_t bytes) {
    return ((uint64_t)kind << 60) | ((uint64_t)t << 56) | ((uint64_t)op << 52) | (uint64_t)(bytes & ((1ull << 52) - 1));
}

// deposit this rank's operand and meet the others; then check every rank is in the same collective
int group_enter(pcg_handle *h, const void *dev, size_t bytes, uint64_t tag) {
    pcg_comm_group *g = (pcg_comm_group *)h->comm;
    const int r = h->comm_rank;
    std::vector<unsigned char> &s = g->slot[r];
    s.resize(bytes);
    hipError_t e = bytes ? hipMemcpyAsync(s.data(), dev, bytes, hipMemcpyDeviceToHost, h->stream) : hipSuccess;
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        group_break(g, std::string("rank ") + std::to_string(r) + ": " + hipGetErrorString(e));
        return group_fail(h, g);
    }
    g->tag[r] = tag;
    if (group_barrier(g)) return group_fail(h, g);
    for (int q = 0; q < g->world; ++q)
        if (g->tag[q] != g->tag[0]) {   // every rank sees the same tags: all of them leave here
            group_break(g, "ranks issued different collectives (kind / type / size) at the same step");
            return group_fail(h, g);
        }
    return PCG_OK;
}

int group_leave(pcg_handle *h, void *dev, const std::vector<unsigned char> &res) {
    pcg_comm_group *g = (pcg_comm_group *)h->comm;
    if (group_barrier(g)) return group_fail(h, g);       // every rank has read every slot
    if (h->comm_rank == 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        ++g->collectives;
    }
    hipError_t e = res.empty() ? hipSuccess
                               : hipMemcpyAsync(dev, res.data(), res.size(), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return pcg_fail(h, PCG_ERR_HIP, "group collective result copy: %s", hipGetErrorString(e));
    return PCG_OK;
}

int group_all_gather(pcg_handle *h, const void *send, void *recv, size_t bytes) {
    pcg_comm_group *g = (pcg_comm_group *)h->comm;
    int rc = group_enter(h, send, bytes, group_tag(1, 0, 0, bytes));
    if (rc) return rc;
    std::vector<unsigned char> all(bytes * (size_t)g->world);
    for (int q = 0; q < g->world; ++q)
        if (bytes) std::memcpy(all.data() + (size_t)q * bytes, g->slot[q].data(), bytes);
    if (h->comm_rank == 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        g->bytes += (int64_t)(bytes * (size_t)g->world);
    }
    return group_leave(h, recv, all);
}

template <typename T>
void reduce_into(std::vector<unsigned char> &out, const std::vector<std::vector<unsigned char>> &slot, size_t count,
                 CommOp op) {
    T *o = (T *)out.data();
    for (size_t i = 0; i < count; ++i) {
        T v = ((const T *)slot[0].data())[i];
        for (size_t q = 1; q < slot.size(); ++q) {
            const T w = ((const T *)slot[q].data())[i];
            v = op == COMM_MAX ? std::max(v, w) : (T)(v + w);
        }
        o[i] = v;
    }
}

int group_all_reduce(pcg_handle *h, void *buf, size_t count, CommType t, CommOp op) {
    pcg_comm_group *g = (pcg_comm_group *)h->comm;
    const size_t bytes = count * (t == COMM_I32 ? 4 : 8);
    int rc = group_enter(h, buf, bytes, group_tag(2, (int)t, (int)op, bytes));
    if (rc) return rc;
    std::vector<unsigned char> res(bytes);
    if (t == COMM_I32) reduce_into<int32_t>(res, g->slot, count, op);
    else reduce_into<int64_t>(res, g->slot, count, op);
    if (h->comm_rank == 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        g->bytes += (int64_t)(bytes * (size_t)g->world);
    }
    return group_leave(h, buf, res);
}

void group_release(pcg_handle *h) {
    pcg_comm_group *g = (pcg_comm_group *)h->comm;
    std::lock_guard<std::mutex> lk(g->mu);
    if (h->comm_rank >= 0 && h->comm_rank < g->world && g->member[h->comm_rank] == h) g->member[h->comm_rank] = nullptr;
}

const CommOps kGroupOps = {"group", group_all_gather, group_all_reduce, group_release};

// agree()'s int64 scratch and finish_sharded's gather: (world + 1) x (5 PCG_MAX_LEVELS + 1) int64
size_t comm_small_bytes(int world) { return sizeof(int64_t) * (size_t)(world + 1) * (5 * PCG_MAX_LEVELS + 1); }

int need_comm(pcg_handle *h) {
    if (!h) return PCG_ERR_INVALID;
    if (!h->comm || !h->comm_ops)
        return pcg_fail(h, PCG_ERR_INVALID, "no communicator: call pcg_comm_init (or pcg_comm_init_group) first");
    return PCG_OK;
}

// Every rank reaches every collective: a rank that fails locally (an allocation, a launch)
// still joins with a "failed" status, and all ranks leave with the same verdict — the failing
// rank its own error, its peers PCG_ERR_PEER — so no rank waits in a collective for a peer that
// returned early. Inside the level loop the status rides in the packed barrier word; outside it
// agree() all-reduces one status int (MAX) first.
//   returns 0 (every rank ok), 1 (some rank failed) or a negative RCCL / HIP error
int agree(pcg_handle *h, int failed) {
    int32_t v = failed ? 1 : 0;
    int32_t *d = (int32_t *)h->comm_status.p;
    PCG_HIP(h, hipMemcpyAsync(d, &v, sizeof(v), hipMemcpyHostToDevice, h->stream));
    if (int rc = h->comm_ops->all_reduce(h, d, 1, COMM_I32, COMM_MAX)) return rc;
    PCG_HIP(h, hipMemcpyAsync(&v, d, sizeof(v), hipMemcpyDeviceToHost, h->stream));
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    return v;
}

// agree() plus a value every rank must hold identically (a plan signature): one all-reduce (MAX)
// of {failed, v, -v}; *same = every rank passed the same v
int agree_value(pcg_handle *h, int failed, int64_t v, bool *same) {
    int64_t a[3] = {failed ? 1 : 0, v, -v};
    int64_t *d = (int64_t *)h->comm_small.p;     // >= 5 * PCG_MAX_LEVELS int64 since pcg_comm_init
    PCG_HIP(h, hipMemcpyAsync(d, a, sizeof(a), hipMemcpyHostToDevice, h->stream));
    if (int rc = h->comm_ops->all_reduce(h, d, 3, COMM_I64, COMM_MAX)) return rc;
    PCG_HIP(h, hipMemcpyAsync(a, d, sizeof(a), hipMemcpyDeviceToHost, h->stream));
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    *same = a[1] == -a[2];
    return (int)a[0];
}

// the verdict of agree() as this rank's return code
int agreed_failure(pcg_handle *h, int local, int g, const char *what) {
    if (g < 0) return g;
    if (local) return local;
    return pcg_fail(h, PCG_ERR_PEER, "%s: another rank failed", what);
}

// [x | y << 32, W union words] per exported row, zero-padded to `rows_out` rows
__global__ void k_pack_rows(const int32_t *xy, const uint64_t *bits, int64_t rows, int W, int64_t rows_out,
                            int64_t *out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = rows_out * (W + 1);
    if (e >= total) return;
    const int64_t r = e / (W + 1);
    const int c = (int)(e - r * (W + 1));
    int64_t v = 0;
    if (r < rows) {
        if (c == 0) v = (int64_t)(uint32_t)xy[2 * r] | ((int64_t)(uint32_t)xy[2 * r + 1] << 32);
        else v = (int64_t)bits[r * W + (c - 1)];
    }
    out[e] = v;
}

// buffers a failed agreement leaves behind are released on EVERY rank, so the ranks' grow-only
// buffers stay equal and the next call's "did anything allocate" decision agrees again
void release_agreed(pcg_handle *h, std::initializer_list<DevBuf *> bufs) {
    (void)hipStreamSynchronize(h->stream);
    for (DevBuf *b : bufs)
        if (b->p) {
            (void)hipFree(b->p);
            b->p = nullptr;
            b->bytes = 0;
        }
}

int sharded_once(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N, double alpha,
                 int max_depth, int flags, int8_t *removed_level) {
    int64_t P = 0;
    if (pcg_level_packed_words(n, &P)) return pcg_fail(h, PCG_ERR_INVALID, "n = %lld", (long long)n);
    const int world = h->comm_world;
    // set-up (buffers, skeleton init). It is agreed by every rank before the first level collective
    // when it allocated anything or is the first of its (n, world) on this communicator; otherwise
    // nothing in it can fail on one rank only (grow-only buffers already sized, arguments equal on
    // every rank), and the host round trip of the agreement is skipped
    const uint64_t a0 = h->alloc_events;
    level_run_begin(h, max_depth);
    int local = PCG_OK;
    if (!pcg_ensure(h, h->comm_packed, sizeof(uint64_t) * (size_t)P) ||
        !pcg_ensure(h, h->comm_gathered, sizeof(uint64_t) * (size_t)P * world))
        local = pcg_fail(h, PCG_ERR_OOM, "packed removal flags");
    if (!local) local = pcg_set_removal_buffer(h, nullptr, 0);   // the handle's own flags
    if (!local) local = pcg_set_world_size(h, world);
    if (!local) local = pcg_skeleton_init(h, C, n, ldc, N, alpha, flags, removed_level);
    // the per-depth barrier (merge, then pcg_level_end's CSR rebuild) must not be able to fail on
    // one rank only: its only allocations, the two neighbour-list buffer sets, are sized here for
    // the complete graph (degrees only fall), inside the agreed set-up. What is left to fail
    // between two collectives is a launch / stream error, i.e. a device fault, not a local OOM.
    for (int t = 0; t < 2 && !local; ++t)
        if (!pcg_ensure(h, h->off2[t], sizeof(int32_t) * (size_t)(n + 1)) ||
            !pcg_ensure(h, h->nbr2[t], sizeof(int32_t) * (size_t)std::max<int64_t>(n * (n - 1), 1)))
            local = pcg_fail(h, PCG_ERR_OOM, "neighbour lists");
    if (local || h->alloc_events != a0 || h->sk_agreed[0] != n || h->sk_agreed[1] != world) {
        const int g = agree(h, local != 0);
        if (g) {
            level_run_abort(h, false);
            pcg_set_world_size(h, 1);
            h->sk_agreed[0] = h->sk_agreed[1] = -1;
            release_agreed(h, {&h->comm_packed, &h->comm_gathered});
            return agreed_failure(h, local, g, "skeleton set-up");
        }
        h->sk_agreed[0] = n;
        h->sk_agreed[1] = world;
    }
    PCG_HT(h, "init:done");
    int rc = PCG_OK, done = 0;
    bool tail_queued = false;
    uint64_t *packed = (uint64_t *)h->comm_packed.p, *gathered = (uint64_t *)h->comm_gathered.p;
    for (int depth = 0; !rc; ++depth) {
        if (max_depth >= 0 && depth > max_depth) break;
        int64_t total = 0, lo = 0, hi = 0;
        PCG_HT(h, "loop:begin");
        // begin is deterministic over the replicated adjacency ("done" agrees on every rank);
        // a local failure of begin / split / run still joins the all-gather below, flagged in
        // the status word, so no peer waits in the collective for this rank
        local = pcg_level_begin(h, depth, &total, nullptr, nullptr);
        if (local == 1) break;
        if (!local) local = pcg_level_split(h, h->comm_rank, world, &lo, &hi);
        if (!local) local = pcg_level_run(h, lo, hi);
        const std::string local_err = local ? h->err : std::string();
        rc = pcg_level_pack(h, packed, local != 0);
        if (rc) {
            // the pack did not launch: send a bare "failed" status word (no flags) instead, so the
            // peers still get this depth's collective and leave with PCG_ERR_PEER
            static const uint64_t failed_word = 1ull << 24;
            (void)hipMemsetAsync(packed, 0, sizeof(uint64_t) * (size_t)(P - 1), h->stream);
            (void)hipMemcpyAsync(packed + (P - 1), &failed_word, sizeof(failed_word), hipMemcpyHostToDevice,
                                 h->stream);
        }
        const int r = h->comm_ops->all_gather(h, packed, gathered, sizeof(uint64_t) * (size_t)P);
        if (rc) break;
        if (r) {
            rc = r;
            break;
        }
        rc = pcg_level_merge(h, gathered, world);
        if (rc) break;
        if (local) {   // this rank's own error, raised after its peers got the verdict
            h->err = local_err;
            rc = local;
            break;
        }
        unsigned long long seq = 0;
        rc = level_end_enqueue(h, &seq);
        if (!rc && level_run_tail_early(h, depth)) {
            rc = level_run_tail_launch(h);
            tail_queued = true;
        }
        if (!rc) rc = level_end_finish(h, depth, seq, nullptr);
        if (!rc) done = depth + 1;
    }
    if (rc) level_run_abort(h, tail_queued);
    else rc = level_run_finish(h, done, tail_queued);
    pcg_set_world_size(h, 1);
    return rc;
}

// The end of a sharded run, in one collective + one host sync: every rank contributes its
// per-depth counters (tests, indep, exact, near-alpha, screened: summed over ranks; replicated
// quantities — calls, degrees, edges — are identical everywhere already) and its exported row
// count (-1 marks a rank that failed to take it) in one all-gather; then the rows themselves,
// packed [x | y << 32, W union words] and zero-padded to the longest rank, in a second all-gather
// and one unpack launch. The row buffers grow-only; their growth (the same decision on every rank:
// all see the same counts) is agreed only when it happens. The rows land stream-ordered in the
// handle's export buffers.
// every rank's gathered rows -> the export buffers, in rank order. The rank prefix is formed on
// the device from the gathered row counts (sd_all: per int64 per rank, the count last), so no
// host buffer has to outlive an asynchronous copy
__global__ void k_unpack_all(const int64_t *in, const int64_t *sd_all, int per, int world, int64_t per_rows, int W,
                             int32_t *xy, uint64_t *bits) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t row = e / (W + 1);
    const int c = (int)(e - row * (W + 1));
    int64_t base = 0;
    int r = 0;
    for (; r < world; ++r) {              // the rank whose rows hold `row`
        const int64_t cnt = sd_all[(int64_t)r * per + per - 1];
        if (row < base + cnt) break;
        base += cnt;
    }
    if (r >= world) return;               // beyond the last rank's rows
    const int64_t v = in[((int64_t)r * per_rows + (row - base)) * (W + 1) + c];
    if (c == 0) {
        xy[2 * row] = (int32_t)(uint32_t)(v & 0xffffffffll);
        xy[2 * row + 1] = (int32_t)(uint32_t)((uint64_t)v >> 32);
    } else {
        bits[row * W + (c - 1)] = (uint64_t)v;
    }
}

int finish_sharded(pcg_handle *h) {
    const int world = h->comm_world, W = h->W;
    const int L = h->st.levels;
    int local = export_sync(h);
    const std::string sync_err = local ? h->err : std::string();
    // [5 L counters, row count] per rank
    const int per = 5 * PCG_MAX_LEVELS + 1;
    std::vector<int64_t> mine((size_t)per, 0), all((size_t)per * world);
    for (int d = 0; d < L && d < PCG_MAX_LEVELS; ++d) {
        mine[d] = h->st.tests[d];
        mine[PCG_MAX_LEVELS + d] = h->st.indep[d];
        mine[2 * PCG_MAX_LEVELS + d] = h->st.exact[d];
        mine[3 * PCG_MAX_LEVELS + d] = h->st.near_alpha[d];
        mine[4 * PCG_MAX_LEVELS + d] = h->st.screened[d];
    }
    mine[per - 1] = local ? -1 : h->export_rows;
    // comm_small holds (world + 1) * per int64 since pcg_comm_init: no allocation between collectives
    int64_t *sd = (int64_t *)h->comm_small.p;
    PCG_HIP(h, hipMemcpyAsync(sd + (size_t)per * world, mine.data(), sizeof(int64_t) * per, hipMemcpyHostToDevice,
                              h->stream));
    if (int rc = h->comm_ops->all_gather(h, sd + (size_t)per * world, sd, sizeof(int64_t) * per)) return rc;
    PCG_HIP(h, hipMemcpyAsync(all.data(), sd, sizeof(int64_t) * all.size(), hipMemcpyDeviceToHost, h->stream));
    PCG_HIP(h, hipStreamSynchronize(h->stream));
    std::vector<int64_t> cnt(world), pre(world + 1, 0);
    bool peer_failed = false;
    int64_t mx = 1;
    for (int r = 0; r < world; ++r) {
        cnt[r] = all[(size_t)r * per + per - 1];
        peer_failed = peer_failed || cnt[r] < 0;
        mx = std::max(mx, cnt[r]);
        pre[r + 1] = pre[r] + std::max<int64_t>(cnt[r], 0);
    }
    if (local) {
        h->err = sync_err;
        return local;
    }
    if (peer_failed) return pcg_fail(h, PCG_ERR_PEER, "sepset gather: another rank failed");
    for (int d = 0; d < L && d < PCG_MAX_LEVELS; ++d) {
        int64_t v[5] = {0, 0, 0, 0, 0};
        for (int r = 0; r < world; ++r)
            for (int k = 0; k < 5; ++k) v[k] += all[(size_t)r * per + k * PCG_MAX_LEVELS + d];
        h->st.tests[d] = v[0];
        h->st.indep[d] = v[1];
        h->st.exact[d] = v[2];
        h->st.near_alpha[d] = v[3];
        h->st.screened[d] = v[4];
    }
    const int64_t total = pre[world];
    const int64_t per_rows = mx, words = per_rows * (W + 1);
    const uint64_t a0 = h->alloc_events;
    if (!pcg_ensure(h, h->comm_packed, sizeof(int64_t) * (size_t)words) ||
        !pcg_ensure(h, h->comm_gathered, sizeof(int64_t) * (size_t)words * world))
        local = pcg_fail(h, PCG_ERR_OOM, "sepset row gather (%lld rows x %d words)", (long long)mx, W + 1);
    if (h->alloc_events != a0) {    // grown (or failed to) on this rank, hence on every rank: agree
        const int g = agree(h, local != 0);
        if (g) {
            release_agreed(h, {&h->comm_packed, &h->comm_gathered});
            h->sk_agreed[0] = h->sk_agreed[1] = -1;
            return agreed_failure(h, local, g, "sepset gather");
        }
    }
    int64_t *pk = (int64_t *)h->comm_packed.p;
    hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, h->stream,
                       (const int32_t *)h->dst_xy, (const uint64_t *)h->dst_bits, cnt[h->comm_rank], W, mx, pk);
    if (int rc = h->comm_ops->all_gather(h, pk, h->comm_gathered.p, sizeof(int64_t) * (size_t)words)) return rc;
    // the last collective of the call: the export buffers grow (their rows are packed already)
    const int64_t cap = std::max<int64_t>(total, 1);
    if (!pcg_ensure(h, h->exportbuf, sizeof(uint64_t) * (size_t)cap * W) ||
        !pcg_ensure(h, h->export_xy, sizeof(int32_t) * 2 * (size_t)cap))
        return pcg_fail(h, PCG_ERR_OOM, "sepset export buffer");
    export_to_own(h, cap);             // every rank's rows land in the handle's own buffers
    const int64_t e = total * (W + 1);
    if (e > 0)
        hipLaunchKernelGGL(k_unpack_all, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, h->stream,
                           (const int64_t *)h->comm_gathered.p, (const int64_t *)sd, per, world, per_rows, W,
                           (int32_t *)h->export_xy.p, (uint64_t *)h->exportbuf.p);
    PCG_HIP(h, hipGetLastError());
    h->export_rows = total;
    h->export_cap = std::max(h->export_cap, cap);
    return PCG_OK;
}

}  // namespace

void pcg_comm_release(pcg_handle *h) {
    if (!h) return;
    h->k1_agreed[0] = h->sk_agreed[0] = -1;   // a new communicator agrees again
    if (h->comm && h->comm_ops) h->comm_ops->release(h);
    h->comm = nullptr;
    h->comm_ops = nullptr;
    for (DevBuf *b : {&h->comm_rm, &h->comm_packed, &h->comm_gathered, &h->comm_small, &h->comm_status})
        if (b->p) {
            (void)hipFree(b->p);
            b->p = nullptr;
            b->bytes = 0;
        }
}

extern "C" int pcg_comm_unique_id(void *id_out, int64_t bytes) {
    if (!id_out || bytes < (int64_t)sizeof(ncclUniqueId)) return PCG_ERR_INVALID;
    if (!rccl().ok) return PCG_ERR_RCCL;
    ncclUniqueId id;
    if (rccl().get_unique_id(&id) != ncclSuccess) return PCG_ERR_RCCL;
    std::memcpy(id_out, &id, sizeof(id));
    return PCG_OK;
}

extern "C" int pcg_comm_init(pcg_handle *h, const void *unique_id, int rank, int world) {
    if (!h || !unique_id || world < 1 || rank < 0 || rank >= world)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_comm_init: rank %d of %d", rank, world);
    if (!rccl().ok) return pcg_fail(h, PCG_ERR_RCCL, "%s", rccl().err.c_str());
    pcg_comm_release(h);
    PCG_HIP(h, hipSetDevice(h->device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    // the status int of agree() and the small stats / row-count buffer exist before the first
    // collective, so no allocation can fail between two collectives later. A failure here still
    // joins the communicator's creation (its peers are blocked in it) and then leaves it.
    const bool bufs = pcg_ensure(h, h->comm_status, 64) && pcg_ensure(h, h->comm_small, comm_small_bytes(world));
    ncclComm_t comm = nullptr;
    PCG_NCCL(h, rccl().comm_init_rank(&comm, world, id, rank));
    if (!bufs) {
        rccl().comm_destroy(comm);
        return pcg_fail(h, PCG_ERR_OOM, "pcg_comm_init: status buffers");
    }
    h->comm = comm;
    h->comm_ops = &kRcclOps;
    h->comm_rank = rank;
    h->comm_world = world;
    return PCG_OK;
}

extern "C" int pcg_comm_group_create(int world, double timeout_s, pcg_comm_group **out) {
    if (!out || world < 1 || world > 4096) return PCG_ERR_INVALID;
    pcg_comm_group *g = new pcg_comm_group();
    g->world = world;
    if (timeout_s > 0) g->timeout_s = timeout_s;
    g->slot.resize((size_t)world);
    g->tag.assign((size_t)world, 0);
    g->member.assign((size_t)world, nullptr);
    *out = g;
    return PCG_OK;
}

extern "C" int pcg_comm_group_destroy(pcg_comm_group *g) {
    if (!g) return PCG_OK;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        for (pcg_handle *m : g->member)
            if (m) return PCG_ERR_INVALID;     // a handle still uses it: pcg_comm_destroy that first
    }
    delete g;
    return PCG_OK;
}

extern "C" int pcg_comm_group_stats(pcg_comm_group *g, int64_t *collectives, int64_t *bytes, int32_t *broken) {
    if (!g) return PCG_ERR_INVALID;
    std::lock_guard<std::mutex> lk(g->mu);
    if (collectives) *collectives = g->collectives;
    if (bytes) *bytes = g->bytes;
    if (broken) *broken = g->broken ? 1 : 0;
    return PCG_OK;
}

extern "C" int pcg_comm_init_group(pcg_handle *h, pcg_comm_group *g, int rank) {
    if (!h || !g || rank < 0 || rank >= g->world)
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_comm_init_group: rank %d", rank);
    pcg_comm_release(h);
    PCG_HIP(h, hipSetDevice(h->device));
    if (!pcg_ensure(h, h->comm_status, 64) || !pcg_ensure(h, h->comm_small, comm_small_bytes(g->world)))
        return pcg_fail(h, PCG_ERR_OOM, "pcg_comm_init_group: status buffers");
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->member[rank]) return pcg_fail(h, PCG_ERR_INVALID, "pcg_comm_init_group: rank %d already joined", rank);
        g->member[rank] = h;
    }
    h->comm = g;
    h->comm_ops = &kGroupOps;
    h->comm_rank = rank;
    h->comm_world = g->world;
    return PCG_OK;
}

extern "C" int pcg_comm_destroy(pcg_handle *h) {
    if (!h) return PCG_ERR_INVALID;
    pcg_comm_release(h);
    h->comm_rank = 0;
    h->comm_world = 1;
    return PCG_OK;
}

extern "C" int pcg_corr_sharded(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C,
                                int64_t ldc) {
    int rc = need_comm(h);
    if (rc) return rc;
    if (!X || !C || N < 2 || n < 1 || ldx < n || ldc < n || n > (1 << 24))
        return pcg_fail(h, PCG_ERR_INVALID, "pcg_corr_sharded: invalid arguments");   // equal on every rank
    PCG_HIP(h, hipSetDevice(h->device));
    const int world = h->comm_world;
    // Set-up: every buffer the launches below use is sized first (the plan — path, moduli, bits,
    // split-K — comes from (n, N) and the K1 knobs). The outcome and the plan signature are agreed
    // by every rank when anything was allocated or this (n, N, world, plan) has not been agreed on
    // this communicator yet; otherwise nothing can fail on one rank only and the agreement's host
    // round trip is skipped (every rank makes the same calls: K1 knobs change on all ranks or none).
    // Ranks started with different knobs thus fail together instead of gathering mismatched units.
    const int64_t sig = k1_plan_signature(h, n, N);
    const uint64_t a0 = h->alloc_events;
    bool crt = false;
    int64_t bytes = 0;
    int local = corr_shard_crt_prepare(h, N, n, world, &crt, &bytes);
    if (!local && !crt) local = pcg_corr_shard_bytes(h, n, N, world, &bytes);
    const size_t b1 = std::max<size_t>((size_t)bytes, 8), b2 = std::max<size_t>((size_t)bytes * world, 8);
    if (!local && (!pcg_ensure(h, h->comm_packed, b1) || !pcg_ensure(h, h->comm_gathered, b2)))
        local = pcg_fail(h, PCG_ERR_OOM, "sharded K1 buffers");
    const bool agreed = h->k1_agreed[0] == n && h->k1_agreed[1] == N && h->k1_agreed[2] == world && h->k1_agreed[3] == sig;
    if (local || h->alloc_events != a0 || !agreed || !crt) {
        // (the digit / fp64 path keeps the synchronous protocol: pcg_corr_shard may allocate inside)
        if (!crt && !local) local = pcg_corr_shard(h, X, N, n, ldx, h->comm_rank, world, (double *)h->comm_packed.p);
        bool same = true;
        const int g = agree_value(h, local != 0, sig, &same);
        if (g || !same) {
            h->k1_agreed[0] = -1;
            release_agreed(h, {&h->comm_packed, &h->comm_gathered, &h->k1_digits});
            if (g) return agreed_failure(h, local, g, "sharded K1");
            return pcg_fail(h, PCG_ERR_INVALID, "sharded K1: the ranks' K1 plans differ (PCG_K1_* knobs)");
        }
        h->k1_agreed[0] = n;
        h->k1_agreed[1] = N;
        h->k1_agreed[2] = world;
        h->k1_agreed[3] = sig;
    }
    if (!crt) {
        if (int r = h->comm_ops->all_gather(h, h->comm_packed.p, h->comm_gathered.p, (size_t)bytes)) return r;
        return pcg_corr_shard_finish(h, (const double *)h->comm_gathered.p, N, n, world, C, ldc);
    }
    // the CRT path: this rank's units (and only its moduli's residue planes), the all-gather and the
    // rebuild, all stream-ordered on the handle's stream with no host sync (a failure from here on
    // is a launch / device fault)
    if ((rc = corr_shard_crt_enqueue(h, X, N, n, ldx, h->comm_rank, world, (double *)h->comm_packed.p))) return rc;
    if ((rc = h->comm_ops->all_gather(h, h->comm_packed.p, h->comm_gathered.p, (size_t)bytes))) return rc;
    return corr_shard_crt_finish_enqueue(h, (const double *)h->comm_gathered.p, N, n, C, ldc);
}

extern "C" int pcg_skeleton_sharded(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                                    double alpha, int max_depth, int flags, int8_t *removed_level,
                                    pcg_stats *stats) {
    int rc = need_comm(h);
    if (rc) return rc;
    for (int attempt = 0; attempt < 6; ++attempt) {
        rc = sharded_once(h, C, n, ldc, N, alpha, max_depth, flags, removed_level);
        if (rc != PCG_ERR_OVERFLOW) break;   // the merged status byte makes every rank rerun
    }
    // level errors (singular, domain, a peer's local failure) end every rank at the same depth
    // through the merged status word, so the collectives below are skipped consistently
    if (!rc) rc = finish_sharded(h);
    if (stats) *stats = h->st;
    return rc;
}
