/*
 * pcgpu.h — C ABI of the MI355X-native PC-fisherz causal-graph engine (libpcgpu.so).
 *
 * The reference (ai4sre/RCAEval) is pure Python; its hot path calls causal-learn's
 * `pc(data, alpha, fisherz, stable=True, uc_rule=0, uc_priority=2, ...)` [U] from
 *   RCAEval/e2e/pc_pagerank.py:19          (pc_pagerank)
 *   RCAEval/graph_construction/pc.py:15-20 (pc_default, used by pc_randomwalk :21)
 *   RCAEval/graph_construction/pc.py:46-56 (pc_fisherz_stable)
 * and scikit-network's `PageRank().fit_transform(adj.T)` [U] from
 *   RCAEval/e2e/pc_pagerank.py:31-32 and RCAEval/graph_heads/page_rank.py:85-89.
 * Each entry point below replaces one piece of that path (cited per function). The
 * Python host layer (rcaeval_amd/) binds them with ctypes; INTEGRATION.md shows the stub.
 *
 * Conventions
 *  - Every call returns 0 (PCG_OK) or a negative PCG_ERR_* code; pcg_last_error() gives text.
 *  - Pointers documented "device" are HIP device pointers (e.g. torch tensor.data_ptr()),
 *    caller-owned; "host" pointers are ordinary host memory. Scratch (adjacency bitmask,
 *    work lists, sepset unions, records) is owned by the handle and grows on demand.
 *  - One handle per (process, device). Calls are ordered on the handle's HIP stream and are
 *    synchronous w.r.t. the host on return unless stated otherwise (pcg_skeleton /
 *    pcg_pc_skeleton return once every result write has completed: their last kernel signals the
 *    host through host-coherent memory and may still be retiring on the handle's stream, which
 *    orders any later work behind it). Not re-entrant per handle;
 *    separate handles may be used from separate threads. No global mutable state.
 *  - Matrices are row-major with an explicit leading dimension (in elements).
 */
#ifndef PCGPU_H
#define PCGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCG_OK 0
#define PCG_ERR_INVALID -1   /* bad argument / unsupported configuration            */
#define PCG_ERR_OOM -2       /* device allocation failed                             */
#define PCG_ERR_HIP -3       /* HIP runtime error                                    */
#define PCG_ERR_SINGULAR -4  /* a CI-test sub-correlation matrix is exactly singular
                                (causal-learn FisherZ raises ValueError) [U]         */
#define PCG_ERR_DOMAIN -5    /* math domain error in the Fisher-z expression
                                (Python math.log/sqrt raise ValueError) [U]          */
#define PCG_ERR_RCCL -6      /* RCCL unavailable or a collective failed               */
#define PCG_ERR_OVERFLOW -7  /* an internal list overflowed its capacity: capacities were
                                enlarged, rerun the skeleton (pcg_skeleton does so itself) */
#define PCG_ERR_PEER -8      /* another rank failed at this depth (edge-sharded skeleton):
                                every rank leaves the level loop at the same depth         */

/* skeleton flags */
#define PCG_FLAG_FULL_P 0x1   /* the p-value mode of the reference arithmetic: every p a caller
                                 can observe is the reference expression's (records, the
                                 near-alpha list). Decisions stay on the monotone |r|
                                 threshold; the +-1e-6 band around it and every test of a
                                 recorded pair go to the exact path, which computes the
                                 reference p (LU like numpy.linalg.inv). Without records,
                                 only the band tests get a p (identical decisions either way) */
#define PCG_FLAG_RECORD 0x2   /* record (a, b, S, p) of every unique test (parity runs), or of
                                 the pcg_set_record_sample pairs; implies FULL_P            */
#define PCG_FLAG_EXACT_ALL 0x4 /* route every test through the LU (numpy.linalg.inv-like)
                                 exact path                                            */

#define PCG_MAX_LEVELS 32
#define PCG_MAX_DEPTH 12      /* deepest conditioning set with per-test records and the
                                 deferred exact-path list; depths 13..PCG_MAX_LEVEL_DEPTH run
                                 on the one-wave-per-set kernel (counts only, no records) */
#define PCG_MAX_LEVEL_DEPTH 30 /* deepest conditioning-set size supported at all          */

typedef struct pcg_handle pcg_handle;

typedef struct {
    int64_t tests[PCG_MAX_LEVELS];     /* unique CI tests evaluated per depth (the reference's
                                          cache misses, GraphClass.py:87-97)              */
    int64_t calls[PCG_MAX_LEVELS];     /* ci_test invocations incl. cache hits per depth    */
    int64_t indep[PCG_MAX_LEVELS];     /* unique tests with p > alpha                       */
    int64_t exact[PCG_MAX_LEVELS];     /* tests resolved by the exact (LU) path             */
    int64_t near_alpha[PCG_MAX_LEVELS];/* tests with |p - alpha| < 1e-9 (enumerated)        */
    int64_t edges_after[PCG_MAX_LEVELS];/* undirected edges left after each depth           */
    int32_t max_degree[PCG_MAX_LEVELS];/* max degree at the start of each depth            */
    double level_ms[PCG_MAX_LEVELS];   /* device wall time per depth (pcg_skeleton: device  */
                                       /* clock stamps; level-step API: HIP events)         */
    double kernel_ms[PCG_MAX_LEVELS];  /* time of the CI-test kernels alone per depth       */
    int32_t levels;                    /* depths run                                        */
    int32_t error;                     /* 0 or PCG_ERR_SINGULAR / PCG_ERR_DOMAIN            */
    int64_t screened[PCG_MAX_LEVELS];  /* tests the fp32 sweep left to its fp64 screen      */
    int32_t driver;                    /* which driver produced the result: PCG_DRIVER_*     */
    int32_t driver_pad;
} pcg_stats;

/* pcg_stats.driver */
#define PCG_DRIVER_LEVELS 0        /* the multi-kernel level loop                            */
#define PCG_DRIVER_SMALL 1         /* the single-workgroup small-graph kernel (n <= 64)      */
#define PCG_DRIVER_SMALL_RERUN 2   /* the small kernel stopped (deeper than its 16 levels or a
                                      full band queue) and the level loop reran the skeleton */

typedef struct {                       /* one unique CI test (PCG_FLAG_RECORD / near-alpha) */
    int32_t a, b;                      /* a < b                                             */
    int32_t d;                         /* |S|                                               */
    int32_t s[PCG_MAX_DEPTH];          /* sorted S, -1 padded                               */
    double p;                          /* Fisher-z p-value                                  */
} pcg_record;

/* ---- ABI identity ------------------------------------------------------------------
 * Bumped whenever a struct above changes layout or an entry point changes signature.
 * v3: pcg_stats gained `screened`. v4: pcg_stats gained `driver`; pcg_corr_shard_bytes takes
 * the handle; pcg_set_tuning / pcg_get_tuning / pcg_k1_plan_signature added.            */
#define PCG_ABI_VERSION 4
/* Sizes of the structs this library writes through caller pointers, and its ABI version;
 * a binding checks them against its own declarations before the first call (host only, no
 * GPU needed). Any out pointer may be NULL.                                             */
int pcg_abi_info(int64_t *stats_bytes, int64_t *record_bytes, int32_t *version);

/* ---- lifetime --------------------------------------------------------------------- */
int pcg_create(int device, pcg_handle **out);
int pcg_destroy(pcg_handle *h);
const char *pcg_last_error(pcg_handle *h);
/* Run every call on this HIP stream (e.g. torch.cuda.current_stream().cuda_stream) so the
 * engine is stream-ordered with the caller's buffers. NULL = the device's default (null)
 * stream — which is what torch's default current stream reports. A new handle starts on
 * its own non-blocking stream until this is called.                                      */
int pcg_set_stream(pcg_handle *h, void *hip_stream);
/* Launch-shape knobs (0 = default). */
int pcg_set_capacity(pcg_handle *h, int64_t record_capacity, int64_t deferred_capacity);
/* PCG_FLAG_RECORD on a fixed sample (full-size parity runs): keep only the unique tests whose
 * canonical pair (a < b) has (a*n + b) % modulus == residue; modulus 0 or 1 = every test.  */
int pcg_set_record_sample(pcg_handle *h, int64_t modulus, int64_t residue);

/* Tuning and testing knobs of one handle. No knob changes a result (every setting is covered
 * by the parity tests); they choose kernels, launch shapes and thresholds. Defaults are read
 * ONCE, in pcg_create, from the environment variable of the knob's name (e.g. PCG_SMALL=0),
 * else the built-in value below; pcg_set_tuning overrides them per handle.             */
#define PCG_TUNE_SMALL 0          /* 1: n <= 64 on the single-workgroup kernel; 0: level loop (1)  */
#define PCG_TUNE_SMALL_QCAP 1     /* band tests per depth the small kernel queues, 1..1024 (1024);
                                     a full queue ends the small run (PCG_DRIVER_SMALL_RERUN)      */
#define PCG_TUNE_LDS_DEEP 2       /* threshold mode: deepest depth on the per-lane k_level_lds,
                                     12..20 (20); deeper levels run one wave per set              */
#define PCG_TUNE_LDS_SPILL_MIN 3  /* depths 17..20 take the per-lane kernel only for levels of at
                                     least this many tests (10000000); below, one wave per set    */
#define PCG_TUNE_WAVE_LO 4        /* >= 5: one wave per conditioning set from this depth on
                                     (0 = the default split)                                     */
#define PCG_TUNE_SCREEN_MASK 5    /* depths (bit 1 << d, d = 2..4) of the fp32-screened sweep;
                                     -1 = pcg_set_screen_precision's choice (0x18)               */
#define PCG_TUNE_NODE_BLOCKS 6    /* depths (bit 1 << d) that stage compact node blocks (0x10)    */
#define PCG_TUNE_EXPORT_INLINE 7  /* graphs of at most this many CSR entries export their sepset
                                     rows on the handle's stream (16384)                          */
#define PCG_TUNE_NB 8             /* narrow-class blocks per depth and rank (0 = per-depth default) */
#define PCG_TUNE_NBW 9            /* wide-class blocks per depth and rank (512)                    */
#define PCG_TUNE_HOST_TRACE 10    /* 1: print the level loop's host timeline to stderr (0)         */
#define PCG_TUNE_K1_I8 11         /* 1: K1 on the int8 matrix cores (1); 0: fp64 MFMA              */
#define PCG_TUNE_K1_CRT 12        /* 1: the CRT residue K1 for n >= PCG_TUNE_K1_CRT_MINN (1)       */
#define PCG_TUNE_K1_CRT_MINN 13   /* (256)                                                         */
#define PCG_TUNE_K1_CRT_BITS 14   /* fewest bits kept per centred value, 32..63 (53)               */
#define PCG_TUNE_K1_CRT_KS 15     /* CRT split-K slabs (0 = cost model)                            */
#define PCG_TUNE_K1_I8_KS 16      /* digit-path split-K slabs (0 = default)                        */
#define PCG_TUNE_K1_SUPER_ORDER 17 /* 1: digit-path tiles in super-rows (1); 0: row-major         */
#define PCG_TUNE_L1Z 18           /* 1: threshold-mode depth 1 grouped by conditioning node on one
                                     rank (k_level1_z, 1); 0: the neighbour-pair kernel           */
#define PCG_TUNE_COUNT 19
int pcg_set_tuning(pcg_handle *h, int key, int64_t value);
int pcg_get_tuning(pcg_handle *h, int key, int64_t *value);

/* ---- K1: correlation -------------------------------------------------------------
 * Replaces FisherZ.__init__'s `np.corrcoef(data.T)` [U]: column means,
 * centred X^T X, *= 1/(N-1), /= s_i, /= s_j, clip to [-1, 1] (numpy's order). The Gram runs on
 * the int8 matrix cores: for n >= 256 as k residue GEMMs combined by the Chinese remainder
 * theorem (exact integer Gram of the values truncated to b >= 56 bits of their column scale,
 * rounded to fp64 once), below that as 45 digit GEMMs; PCG_K1_I8=0 selects fp64 MFMA.
 * X: device, N x n (ldx >= n). C: device, n x n (ldc >= n).                            */
int pcg_corr(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx,
             double *C, int64_t ldc);

/* ---- K1 sharded over ranks (multi-GPU) --------------------------------------------
 * Rank `rank` of `world` computes its share of the Gram work into `packed` (device,
 * pcg_corr_shard_bytes bytes): a contiguous run of (tile, modulus, slab) residue units on the
 * CRT path, else the Gram sums of its zig-zag share of the 64-row tile rows. The caller
 * all-gathers the packed buffers rank-major (RCCL over xGMI) and calls pcg_corr_shard_finish on
 * the same handle (it reads the column exponents pcg_corr_shard left there), which rebuilds,
 * mirrors and normalises: C is bitwise the single-GPU pcg_corr result for every world size.
 * pcg_corr_shard_rows: the digit / fp64 path's rows_per_rank (packed = rows x n doubles).     */
int pcg_corr_shard_bytes(pcg_handle *h, int64_t n, int64_t N, int world, int64_t *bytes_per_rank);
/* A signature of K1's plan for (n, N) under this handle's knobs (path; the CRT path's moduli,
 * bits, split-K and unit count): ranks compare it before exchanging shards. h may be NULL
 * (built-in defaults), also for pcg_corr_shard_bytes.                                      */
int pcg_k1_plan_signature(pcg_handle *h, int64_t n, int64_t N, int64_t *signature);
int pcg_corr_shard_rows(int64_t n, int world, int64_t *rows_per_rank);
int pcg_corr_shard(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, int rank,
                   int world, double *packed);
int pcg_corr_shard_finish(pcg_handle *h, const double *gathered, int64_t N, int64_t n, int world,
                          double *C, int64_t ldc);

/* ---- K2/K3: stable PC skeleton ---------------------------------------------------
 * Replaces causal-learn skeleton_discovery(stable=True) with FisherZ
 * (lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:70-144, GraphClass.py:78-106).
 * C: device n x n correlation (from pcg_corr or caller). N: sample count (FisherZ dof).
 * removed_level: device n x n int8 out; -1 = edge survives, else the depth at which the
 * edge was removed. max_depth < 0: unlimited (the reference's behaviour).
 * stats: host out. Sepset unions are kept in the handle: see pcg_sepset_*.             */
int pcg_skeleton(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                 double alpha, int max_depth, int flags, int8_t *removed_level,
                 pcg_stats *stats);

/* K1 + skeleton in one call: pcg_corr's kernels then pcg_skeleton's on the same stream, with
 * no host round trip between them (the path pc(data) takes: FisherZ.__init__'s corrcoef, then
 * skeleton_discovery). X: device N x n (ldx); C: device n x n out (ldc). Same results as the
 * two calls.                                                                              */
int pcg_pc_skeleton(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx, double *C,
                    int64_t ldc, double alpha, int max_depth, int flags, int8_t *removed_level,
                    pcg_stats *stats);

/* Degrees at the start of each depth of the last pcg_skeleton (host out, levels x n). */
int pcg_degrees(pcg_handle *h, int32_t *deg_host, int64_t capacity);

/* Sepset unions of the last pcg_skeleton: one row per ordered removed pair (x, y) whose
 * union is non-empty: the union of every independent S seen from x's side
 * (SkeletonDiscovery.py:129-130,135-136) as an n-bit mask (W = ceil(n/64) words).      */
int pcg_sepset_count(pcg_handle *h, int64_t *count, int32_t *words_per_row);
int pcg_sepset_export(pcg_handle *h, int32_t *xy_host /* 2*count */,
                      uint64_t *bits_host /* count*W */, int64_t count);
/* Same, into caller-owned device buffers (stream-ordered copy, no host round trip).     */
int pcg_sepset_export_device(pcg_handle *h, int32_t *xy_dev, uint64_t *bits_dev, int64_t count);
/* Export the sepset rows of the following one-GPU pcg_skeleton / pcg_pc_skeleton / level-step
 * runs straight into caller-owned device buffers (xy: 2 x capacity int32, bits: capacity x W
 * uint64, W = ceil(n / 64)) whenever they hold the run's row bound — the ordered pairs entering
 * depth 1 — so no copy follows the call. NULL / 0 restores the handle's own buffers. The buffers
 * must stay valid until the run's result has been read.
 * pcg_sepset_target after a run: *in_caller = 1 when the rows are in the caller's buffers (rows
 * 0 .. count - 1 of pcg_sepset_count), 0 when they are in the handle's own (copy them with
 * pcg_sepset_export_device, which skips a copy onto itself); *capacity_needed = the run's row
 * bound, the capacity that would have held them.                                          */
int pcg_set_sepset_buffers(pcg_handle *h, int32_t *xy_dev, uint64_t *bits_dev, int64_t capacity);
int pcg_sepset_target(pcg_handle *h, int32_t *in_caller, int64_t *capacity_needed);

/* Records of the last pcg_skeleton (PCG_FLAG_RECORD) and the near-alpha list.         */
int pcg_record_count(pcg_handle *h, int64_t *count, int64_t *near_alpha_count);
int pcg_record_export(pcg_handle *h, pcg_record *rec_host, int64_t count,
                      pcg_record *near_host, int64_t near_count);

/* ---- multi-GPU level step (edge-sharded skeleton) ----------------------------------
 * The host drives the level loop: pcg_level_begin prepares depth d from the current
 * adjacency and returns the work size; pcg_level_run evaluates the chunk range
 * [chunk_lo, chunk_hi) (an owner-disjoint slice of the level's work list), writing the
 * removal flags (device n*n uint8, `rm_dev`, zeroed by begin) and sepset unions;
 * the caller merges rm_dev across ranks (RCCL all-reduce MAX over xGMI) and calls
 * pcg_level_end, which applies the removals identically on every rank.               */
int pcg_skeleton_init(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                      double alpha, int flags, int8_t *removed_level);
int pcg_level_begin(pcg_handle *h, int depth, int64_t *total_chunks, int32_t *max_degree,
                    uint8_t **rm_dev);
int pcg_level_run(pcg_handle *h, int64_t chunk_lo, int64_t chunk_hi);
int pcg_level_end(pcg_handle *h, pcg_stats *stats);
/* Work weight of each chunk prefix (host out, total_chunks+1 int64) for load balance.  */
int pcg_level_chunk_work(pcg_handle *h, int64_t *prefix_host, int64_t capacity);
/* The contiguous work-balanced chunk range [lo, hi) of `rank` (the same cut as
 * searchsorted(prefix, total*r/world, 'left') over pcg_level_chunk_work's prefix).       */
int pcg_level_split(pcg_handle *h, int rank, int world, int64_t *chunk_lo, int64_t *chunk_hi);
/* Use a caller-owned device buffer (n*n + PCG_RM_STATUS bytes, e.g. a torch tensor that
 * the caller all-reduces with MAX) for the per-depth removal flags instead of the handle's
 * own; NULL = own. The PCG_RM_STATUS bytes after the n*n flags carry level status that the
 * merge spreads to every rank: [0] an exact-path/record list overflowed (pcg_level_end
 * returns PCG_ERR_OVERFLOW on every rank: grow nothing, rerun the skeleton — capacities
 * have already been enlarged), [1] a singular sub-matrix, [2] a math domain error.      */
#define PCG_RM_STATUS 64
/* Bit-packed level barrier (replaces the n*n-byte all-reduce): pcg_level_pack writes this
 * rank's removal flags as upper-triangle bits plus one status word (`words` u64 from
 * pcg_level_packed_words; 256 KB at n = 2000) into packed_dev — local_error != 0 contributes
 * no flags and marks "this rank failed" so its peers do not wait in the collective; the caller
 * all-gathers the packed words of every rank (RCCL over xGMI, rank-major) and
 * pcg_level_merge ORs the `world` copies back into the removal flags and status bytes;
 * pcg_level_end then returns PCG_ERR_PEER on every rank if any rank failed.
 * Both are stream-ordered on the handle's stream.                                          */
int pcg_level_packed_words(int64_t n, int64_t *words);
int pcg_level_pack(pcg_handle *h, uint64_t *packed_dev, int local_error);
int pcg_level_merge(pcg_handle *h, const uint64_t *gathered_dev, int world);
/* Background knowledge (causal-learn BackgroundKnowledge, RCAEval/graph_construction/pc.py:6-9,19):
 * banned_dev (device n x n uint8, symmetric, or NULL to clear) marks the pairs whose edge is
 * forbidden in BOTH directions; skeleton_discovery removes them at the end of depth 0 whatever
 * their tests said, with an empty separating set (SkeletonDiscovery.py:86-101, stable=True).
 * Applies to the following pcg_skeleton / pcg_pc_skeleton / level-step runs of this handle
 * (in a sharded run the rank owning chunk 0 of depth 0 contributes them to the merge).        */
int pcg_set_forbidden_pairs(pcg_handle *h, const uint8_t *banned_dev);
/* Host orientation with background knowledge [U]: orient_by_background_knowledge, then
 * uc_sepset's collider step skipping (x, y, z) when x->y or z->y is forbidden or y->x or y->z
 * required, then Meek skipping any orientation i->j that is forbidden or whose reverse is
 * required. R0 (the candidates) is enumerated on the graph AFTER the background orientation,
 * as uc_sepset does on its copy of it. priority 2: R0 in that order (triples/scores unused);
 * priority 3 / 4: scores[q] is the max p-value of candidate triples[q] (any order, every R0
 * triple present: pcg_uc_candidates + pcg_fisherz_batch), R0 is stable-sorted by it ascending
 * (3) or descending (4). forbidden / required: host n x n uint8 directed relations
 * (forbidden[i*n + j]: i->j forbidden), either may be NULL. graph: host n x n int32 out.
 * Replaces causal-learn pc_alg's orient_by_background_knowledge + uc_sepset + meek calls with
 * background_knowledge (reached from RCAEval/graph_construction/pc.py:15-20).               */
int pcg_orient_bk(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
                  int64_t count, int priority, const int32_t *triples, const double *scores, int64_t tcount,
                  const uint8_t *forbidden, const uint8_t *required, int32_t *graph);
/* Testing knob: nodes with more than `max_degree` (default and cap 64) neighbours leave the
 * narrow LDS-resident class, so the wide T-group kernel (64-bit masks -> 128-bit) and the
 * staged kernels can be checked on small graphs. Results are identical for any value.      */
int pcg_set_narrow_degree(pcg_handle *h, int max_degree);
/* Testing knob: 1 (default) runs the threshold-mode T-group sweep of depths 2..4 in packed
 * fp32 with an a-priori error bound (tests it cannot make certain are evaluated in fp64:
 * k_level_lds_f); 0 runs the all-fp64 sweep (k_level_lds_t). Results are identical.      */
int pcg_set_screen_precision(pcg_handle *h, int fp32);
/* Capacity (tests) of the fp32 sweep's fp64 screen list (default 2^20 per depth). An overflow
 * makes the level report PCG_ERR_OVERFLOW with the capacity raised; pcg_skeleton /
 * pcg_pc_skeleton rerun by themselves, level-step drivers rerun the skeleton.              */
int pcg_set_screen_capacity(pcg_handle *h, int64_t entries);
/* Number of ranks the level work lists are split over (default 1). The per-depth
 * decomposition sizes its chunks so that each rank's slice still fills its GPU.          */
int pcg_set_world_size(pcg_handle *h, int world);
int pcg_set_removal_buffer(pcg_handle *h, uint8_t *rm_dev, int64_t bytes);

/* ---- native multi-GPU driver (RCCL over xGMI, one process per GPU) -----------------
 * SURVEY §8(b)'s pcg_comm_init / pcg_skeleton_sharded: the whole edge-sharded level loop
 * runs in C with the collectives on the handle's stream — no host language between the
 * per-depth steps. RCCL is resolved at run time (the copy the process already loaded, e.g.
 * PyTorch's, else librccl.so.1), so one RCCL instance serves both.
 * pcg_comm_unique_id: rank 0 creates the id (NCCL_UNIQUE_ID_BYTES = 128 bytes) and the
 * caller hands the bytes to every rank; pcg_comm_init joins rank `rank` of `world`.      */
#define PCG_COMM_ID_BYTES 128
int pcg_comm_unique_id(void *id_out, int64_t bytes);
int pcg_comm_init(pcg_handle *h, const void *unique_id, int rank, int world);
int pcg_comm_destroy(pcg_handle *h);
/* In-process transport for the same driver: a group of `world` handles used from separate
 * threads of ONE process (on one or several devices), with host-staged collectives that
 * complete before they return. RCCL refuses two ranks on one device, so this is the transport
 * that runs the driver's rank-dependent steps (level split, packed all-gather + OR merge, stats
 * all-reduce, sepset gathers) at world 2..8 on a single GPU; results are those of the RCCL
 * transport. Every collective is checked to be the same (kind, type, size) on every rank — a
 * mismatch, a rank failing inside a collective, or a barrier waiting longer than `timeout_s`
 * (<= 0: 300 s) breaks the group and every rank returns PCG_ERR_RCCL instead of hanging.
 * pcg_comm_init_group attaches handle `h` as `rank` (pcg_comm_destroy detaches it);
 * pcg_comm_group_destroy refuses a group that still has an attached handle.
 * pcg_comm_group_stats: collectives completed, bytes contributed by all ranks, broken flag. */
typedef struct pcg_comm_group pcg_comm_group;
int pcg_comm_group_create(int world, double timeout_s, pcg_comm_group **out);
int pcg_comm_group_destroy(pcg_comm_group *g);
int pcg_comm_group_stats(pcg_comm_group *g, int64_t *collectives, int64_t *bytes, int32_t *broken);
int pcg_comm_init_group(pcg_handle *h, pcg_comm_group *g, int rank);
/* K1 on the communicator: this rank's share (pcg_corr_shard's units; on the CRT path only the
 * residue planes of the moduli its units use) + all-gather + rebuild; C is bitwise the
 * single-GPU pcg_corr result on every rank. On the CRT path (n >= 256) the call returns once
 * its work is queued on the handle's stream (stream-ordered, no host sync); the set-up (buffers,
 * the ranks' K1 plan signatures) is agreed across ranks on the first call of an (n, N, world,
 * plan) and whenever a buffer grows, so K1 knobs must change on every rank or on none.       */
int pcg_corr_sharded(pcg_handle *h, const double *X, int64_t N, int64_t n, int64_t ldx,
                     double *C, int64_t ldc);
/* The edge-sharded stable skeleton on the communicator (the level loop of pcg_skeleton, with its
 * device-clock depth stamps and tail kernel): per depth begin / split / run on
 * this rank's work-balanced chunk range / pack / RCCL all-gather of the packed removal bits
 * and status word / merge / end (a rank that fails locally still joins the all-gather, and
 * its peers return PCG_ERR_PEER at the same depth); then the per-level counters are summed over ranks and every rank's
 * sepset rows are all-gathered, so pcg_sepset_* and removed_level describe the whole
 * skeleton on every rank (a pair's row may appear once per rank that saw it: OR them) — the
 * counters and row counts in one all-gather, the rows in a second. The set-up is agreed across
 * ranks on the first call of an (n, world) and whenever a buffer grows.
 * Same arguments and results as pcg_skeleton.                                              */
int pcg_skeleton_sharded(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                         double alpha, int max_depth, int flags, int8_t *removed_level,
                         pcg_stats *stats);

/* ---- K4: PageRank head -------------------------------------------------------------
 * Replaces scikit-network 0.31.0 PageRank(damping_factor, solver='piteration', n_iter,
 * tol).fit_transform(A) [U] (RCAEval/e2e/pc_pagerank.py:31-32,
 * RCAEval/graph_heads/page_rank.py:85-89): A (device, m x m dense, lda) is the matrix
 * passed to fit_transform. scores: device m doubles out. Returns PCG_ERR_INVALID
 * ("The input matrix is empty.") when A has no non-zero (sknetwork check_format).       */
int pcg_pagerank_dense(pcg_handle *h, const double *A, int64_t m, int64_t lda,
                       double damping, int n_iter, double tol, double *scores);
/* Same on a CSR input (device indptr[m+1], indices[nnz], data[nnz]).                   */
int pcg_pagerank_csr(pcg_handle *h, const int32_t *indptr, const int32_t *indices,
                     const double *data, int64_t m, int64_t nnz, double damping,
                     int n_iter, double tol, double *scores);

/* ---- random-walk head ------------------------------------------------------------
 * Replaces RandomWalkScorer._walk (RCAEval/graph_heads/random_walk.py:179-186) for a
 * column-stochastic transition matrix P (device, m x m, column c = distribution of the
 * next node from c, as generate_transition_matrix :159-177 builds it): `num_loop` draws of
 * numpy Generator(PCG64).choice(index, p=P[:, node]) from the given PCG64 state
 * (state_hi/lo, inc_hi/lo: numpy's 128-bit state), start node `start`.
 * counts: device m int64 out (visits per node).                                       */
int pcg_random_walk(pcg_handle *h, const double *P, int64_t m, int64_t ldp, int64_t start,
                    int64_t num_loop, uint64_t state_hi, uint64_t state_lo, uint64_t inc_hi,
                    uint64_t inc_lo, int64_t *counts);

/* ---- host orientation (C++, no device work) ----------------------------------------
 * causal-learn UCSepset.uc_sepset(cg, priority=2) then Meek.meek(cg) [U] over the
 * triple / triangle / kite enumerations of lib/causallearn/graph/GraphClass.py:108-188.
 * adj: host n x n uint8 skeleton; sep_xy/sep_bits: host sepset-union rows as exported
 * by pcg_sepset_export (count rows). graph: host n x n int32 endpoint codes out
 * (TAIL=-1, ARROW=1; i->j <=> g[i,j]=-1, g[j,i]=1).                                     */
int pcg_orient(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
               int64_t count, int priority, int32_t *graph);

/* The R0 list of UCSepset.uc_sepset [U]: unshielded triples (x, y, z), x < z, in
 * find_unshielded_triples order (GraphClass.py:157-165), with y in no S of sepset[x, z].
 * triples: host 3*capacity int32 out (x, y, z); total: host out (all candidates; call
 * again with capacity >= total to get them all).                                       */
int pcg_uc_candidates(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
                      int64_t count, int32_t *triples, int64_t capacity, int64_t *total);
/* uc_sepset's collider step over `triples` in the given order (priority 3/4: R0 sorted
 * by the max CI p-value, ascending / descending — the caller computes those p with
 * pcg_fisherz_batch), then Meek.meek [U]. graph: host n x n int32 endpoint codes out.  */
int pcg_orient_triples(int64_t n, const uint8_t *adj, const int32_t *triples, int64_t tcount,
                       int32_t *graph);

/* ---- batched Fisher-z tests on caller-chosen (x, y, S) -----------------------------
 * Replaces individual `cg.ci_test(x, y, S)` / FisherZ.__call__ [U] calls that do not come
 * from the level enumeration (GraphClass.py:78-98): UCSepset priority 3/4 conditioning
 * sets (GraphClass.py:190-204), the stable=False skeleton (SkeletonDiscovery.py:112-131),
 * FCI possible-d-sep tests. tests: device count x stride int32 rows
 * [a, b, d, s_0 .. s_{d-1}, pad], a < b and S sorted, distinct (the cache-key canonical
 * form, GraphClass.py:87-88), d <= PCG_MAX_LEVEL_DEPTH, stride >= d + 3.
 * p: device count doubles out (the reference p expression; LU like numpy.linalg.inv).
 * status: device count int32 out: 0 ok, 1 singular sub-matrix (LinAlgError -> ValueError),
 * 2 math domain error (ValueError), 3 malformed row (refused, never dereferenced).
 * Synchronous on return.                                                                 */
int pcg_fisherz_batch(pcg_handle *h, const double *C, int64_t n, int64_t ldc, int64_t N,
                      const int32_t *tests, int32_t stride, int64_t count, double *p,
                      int32_t *status);

/* ---- batched discrete CI tests (RCD) ----------------------------------------------
 * Replaces causal-learn's chisq / gsq [U] (utils/cit.py chisq_or_gsq_test, causal-learn
 * 0.1.2.3 of RCAEval's RCD environment) as called from SkeletonDiscovery.py:152-210 /
 * :70-144 by RCAEval/e2e/rcd.py:72-102. data: device n x N int32, variable-major (data[v*N+i]
 * in [0, card[v])); card: device n int32; tests: device count x stride int32 rows
 * [a, b, d, s_0 .. s_{d-1}, pad] (a < b). Per test: the contingency table over the strata of
 * S (empty strata dropped), the chi-square (g_sq = 0) or G-square (g_sq = 1) statistic summed
 * like numpy (bitwise), and its degrees of freedom. stat: device count doubles; df: device count
 * int64; status: device count int32 (0 ok, 3 malformed row or sample, 4 table larger than
 * max_cells). The caller takes p = chi2.sf(stat, df) (p = 1 when df <= 0). Synchronous.  */
int pcg_chisq_batch(pcg_handle *h, const int32_t *data, int64_t N, int64_t n, const int32_t *card,
                    const int32_t *tests, int32_t stride, int64_t count, int g_sq, int64_t max_cells,
                    double *stat, int64_t *df, int32_t *status);

#ifdef __cplusplus
}
#endif
#endif /* PCGPU_H */
