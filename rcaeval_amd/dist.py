"""Edge-sharded stable-PC skeleton across GPUs (one process per GPU, RCCL over xGMI).

Within one depth every (edge, S) test is independent — removals are deferred to the level
barrier (``SkeletonDiscovery.py:141-144``) — so each rank evaluates an owner-disjoint,
work-balanced slice of the depth's chunk list (a chunk = one node x and a run of S ranks;
every test of a chunk, including both sepset sides, is evaluated by its owner). The only
exchange is the removal flags: each rank packs its upper-triangle flags into bits plus one
status word (``pcg_level_pack``: 256 KB at n = 2000 instead of 4 MB of bytes), ONE
all-gather (RCCL over xGMI) collects every rank's words, and ``pcg_level_merge`` ORs them
(RCCL has no bitwise OR). Every rank then applies the identical removals, so adjacency,
degrees and the next depth's work list agree everywhere. A rank whose begin / run fails still
joins the all-gather with its "failed" status bit set, so its peers leave the depth with
``PCG_ERR_PEER`` instead of waiting in the collective. Sepset-union rows stay on their owner
until the end, then are all-gathered once.

``LevelBackend`` abstracts one rank's device work so the protocol can be exercised on the
CPU with ``gloo`` (tests/test_dist_cpu.py injects an oracle-backed backend).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import PcgStats, check


FAILED_WORD = 1 << 24    # barrier.hip k_pack_status: byte 3 of the status word = "this rank failed"


def agree(failed: bool, device="cpu", group=None) -> bool:
    """True when ANY rank of ``group`` reports failure (one all-reduce MAX of a status int).
    Every rank calls it at the same point, so a rank that failed locally outside the level
    loop (set-up, result collection) takes its peers out with it instead of leaving them
    blocked in the next collective."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if failed else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


def agree_value(failed: bool, value: int, device="cpu", group=None) -> tuple[bool, bool]:
    """``agree`` plus a value every rank must hold identically (one all-reduce MAX of
    {failed, v, -v}): (any rank failed, every rank passed the same value)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if failed else 0, int(value), -int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    v = t.cpu().tolist()
    return bool(v[0]), v[1] == -v[2]


def raise_agreed(local_err, what: str):
    """Re-raise this rank's own error, or PCG_ERR_PEER for a peer's."""
    if local_err is not None:
        raise local_err
    raise _lib.PcgError(_lib.PCG_ERR_PEER, f"{what}: another rank failed")


def agreed_backend(factory, device="cpu", group=None):
    """Build this rank's level backend, then agree on every rank's success before the first
    level collective (a rank whose set-up fails, e.g. OOM, raises; its peers raise PEER)."""
    backend, err = None, None
    try:
        backend = factory()
    except Exception as e:   # noqa: BLE001 - must reach the agreement below
        err = e
    if agree(err is not None, device=device, group=group):
        raise_agreed(err, "skeleton set-up")
    return backend


def split_by_work(prefix: np.ndarray, rank: int, world: int) -> tuple[int, int]:
    """Contiguous chunk range of ``rank`` so that every rank gets ~1/world of the work.

    ``prefix`` has total_chunks + 1 entries (prefix[0] = 0, non-decreasing).
    Ranges of consecutive ranks tile [0, total_chunks) exactly.
    """
    total = len(prefix) - 1
    if total <= 0:
        return 0, 0
    W = float(prefix[-1])

    def cut(r: int) -> int:
        if r <= 0:
            return 0
        if r >= world:
            return total
        return int(np.searchsorted(prefix, W * r / world, side="left"))

    lo, hi = cut(rank), cut(rank + 1)
    return min(lo, total), min(max(hi, lo), total)


class GpuLevelBackend:
    """One rank's device work through the C ABI (pcg_skeleton_init / pcg_level_*)."""

    def __init__(self, eng, C, N: int, alpha: float, flags: int, world: int = 1):
        import torch
        self.eng, self.lib, self.h = eng, eng.lib, eng.h
        Cd = eng.to_device(C)
        self.C = Cd
        n = Cd.shape[0]
        self.n = n
        self.rl = torch.empty((n, n), dtype=torch.int8, device=eng.device)
        words = ctypes.c_int64()
        check(self.h, self.lib.pcg_level_packed_words(n, ctypes.byref(words)), "pcg_level_packed_words")
        self.packed = torch.zeros(words.value, dtype=torch.int64, device=eng.device)
        check(self.h, self.lib.pcg_set_removal_buffer(self.h, None, 0), "pcg_set_removal_buffer")
        check(self.h, self.lib.pcg_set_world_size(self.h, int(world)), "pcg_set_world_size")
        check(self.h, self.lib.pcg_skeleton_init(self.h, ctypes.c_void_p(Cd.data_ptr()), n, n, int(N),
                                                 float(alpha), int(flags), ctypes.c_void_p(self.rl.data_ptr())),
              "pcg_skeleton_init")
        self.stats = PcgStats()

    def begin(self, depth: int):
        total, maxdeg, rmp = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_void_p()
        rc = self.lib.pcg_level_begin(self.h, depth, ctypes.byref(total), ctypes.byref(maxdeg), ctypes.byref(rmp))
        if rc == 1:
            return None
        check(self.h, rc, "pcg_level_begin")
        return total.value

    def prefix(self, total: int) -> np.ndarray:
        """Work prefix of the current depth's chunks (pcg_level_chunk_work), for checks."""
        prefix = np.zeros(total + 1, np.int64)
        check(self.h, self.lib.pcg_level_chunk_work(self.h, prefix.ctypes.data_as(ctypes.c_void_p), len(prefix)),
              "pcg_level_chunk_work")
        return prefix

    def split(self, rank: int, world: int):
        """This rank's chunk range, cut in C (pcg_level_split == split_by_work)."""
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        check(self.h, self.lib.pcg_level_split(self.h, rank, world, ctypes.byref(lo), ctypes.byref(hi)),
              "pcg_level_split")
        return lo.value, hi.value

    def run(self, lo: int, hi: int):
        check(self.h, self.lib.pcg_level_run(self.h, int(lo), int(hi)), "pcg_level_run")

    def pack(self, local_error: bool):
        """This rank's removal flags as packed upper-triangle bits + status word (device)."""
        check(self.h, self.lib.pcg_level_pack(self.h, ctypes.c_void_p(self.packed.data_ptr()), int(local_error)),
              "pcg_level_pack")
        return self.packed

    def pack_failed(self):
        """A bare "this rank failed" word (no flags), for when pack itself failed."""
        self.packed.zero_()
        self.packed[-1] = FAILED_WORD
        return self.packed

    def merge(self, gathered, world: int):
        """OR of every rank's packed words (rank-major) back into the removal flags."""
        g = gathered.contiguous()
        check(self.h, self.lib.pcg_level_merge(self.h, ctypes.c_void_p(g.data_ptr()), int(world)), "pcg_level_merge")
        self._keep = g            # the merge is stream-ordered: keep the buffer alive until end()

    def end(self):
        check(self.h, self.lib.pcg_level_end(self.h, ctypes.byref(self.stats)), "pcg_level_end")
        self._keep = None

    def finish(self):
        self.lib.pcg_set_world_size(self.h, 1)
        return self.eng._collect(self.n, self.rl, self.stats, None)


def run_sharded_levels(backend, rank: int, world: int, max_depth: int = -1, group=None, trace=None):
    """The level loop shared by the GPU path and the CPU protocol test. ``trace`` (a list)
    collects (phase, depth, seconds) host timings of begin / run / exchange / end.

    Per depth: begin (identical on every rank: the adjacency is replicated) / split / run on
    this rank's slice / pack / ONE all-gather / merge / end. A local failure of begin, split
    or run is carried through the all-gather as the rank's "failed" status bit and re-raised
    afterwards; its peers raise ``PCG_ERR_PEER`` from end at the same depth."""
    import time

    clock = time.perf_counter
    depth = 0
    while True:
        if max_depth >= 0 and depth > max_depth:
            break
        t0 = clock()
        local_err = None
        t1 = t0
        try:
            work = backend.begin(depth)
            if work is None:
                break                # "done" is decided on replicated state: every rank agrees
            # GPU backend: the cut is made in C; the CPU protocol test hands back the prefix
            lo, hi = backend.split(rank, world) if hasattr(backend, "split") else split_by_work(work, rank, world)
            t1 = clock()
            backend.run(lo, hi)
        except Exception as e:   # noqa: BLE001 - any local failure must still reach the collective
            local_err = e
        t2 = clock()
        try:
            packed = backend.pack(local_err is not None)
        except Exception as e:   # noqa: BLE001 - join the collective with a bare failed word
            local_err = local_err or e
            packed = backend.pack_failed()
        gathered = _gather_tensor(packed, group=group)
        backend.merge(gathered, world)
        t3 = clock()
        if local_err is not None:
            raise local_err
        backend.end()
        if trace is not None:
            trace.extend([("begin", depth, t1 - t0), ("run", depth, t2 - t1),
                          ("exchange", depth, t3 - t2), ("end", depth, clock() - t3)])
        depth += 1
    return depth


def _gather_tensor(t, group=None):
    """All-gather equal-shaped tensors into one (world * rows, ...) tensor: one RCCL
    all-gather into a contiguous buffer under nccl, the list form under gloo."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        return out
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t.contiguous(), group=group)
    return torch.cat(parts)


def _allgather_rows(xy, bits, group=None, failed=None, device=None):
    """All-gather variable-length (xy, bits) device tensors from every rank: one count
    exchange (one host sync), then ONE all-gather of rows packed as [x | y << 32, bits...]
    (int64, padded to the longest rank). ``failed`` (this rank's exception, xy/bits unused)
    travels as a count of -1: every rank then raises (its own error or PCG_ERR_PEER) before
    the rows move."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = device if failed is not None else xy.device
    cnt = torch.tensor([-1 if failed is not None else xy.shape[0]], dtype=torch.int64, device=dev)
    counts = _gather_tensor(cnt, group=group).cpu().tolist()
    if failed is not None or min(counts) < 0:
        raise_agreed(failed, "sepset gather")
    mx = max(max(counts), 1)
    W = bits.shape[1]
    k = xy.shape[0]
    pad = torch.zeros((mx, W + 1), dtype=torch.int64, device=xy.device)
    if k:
        xy64 = xy.to(torch.int64)
        pad[:k, 0] = (xy64[:, 0] & 0xFFFFFFFF) | (xy64[:, 1] << 32)
        pad[:k, 1:] = bits
    allrows = _gather_tensor(pad, group=group).view(world, mx, W + 1)
    rows = torch.cat([allrows[r, :c] for r, c in enumerate(counts)])
    xy_out = torch.stack([rows[:, 0] & 0xFFFFFFFF, rows[:, 0] >> 32], dim=1).to(torch.int32)
    return xy_out.contiguous(), rows[:, 1:].contiguous()


def _allreduce_stats(stats: dict, device, group=None) -> dict:
    import torch
    import torch.distributed as dist
    keys = ("tests", "indep", "exact", "near_alpha", "screened")
    L = stats["levels"]
    t = torch.tensor([stats[k][i] for k in keys for i in range(L)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    vals = t.cpu().numpy().reshape(len(keys), L) if L else np.zeros((len(keys), 0), np.int64)
    out = dict(stats)
    for i, k in enumerate(keys):
        out[k] = [int(v) for v in vals[i]]
    return out


def sharded_corr(eng, X, group=None):
    """K1 sharded over the ranks of ``group``: each rank computes its share of the Gram work
    (residue units on the CRT path, zig-zag tile rows otherwise), one all-gather (RCCL over
    xGMI) assembles them, and every rank rebuilds and normalises locally. Bitwise equal to the
    single-GPU ``eng.corr(X)``."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    cdev = eng.device if dist.get_backend(group) == "nccl" else "cpu"
    N, n = X.shape
    # a local failure (e.g. OOM on the residue planes) and the K1 plan (path, moduli, bits,
    # split-K: pcg_k1_plan_signature under each handle's PCG_TUNE_K1_* knobs) with the share's size
    # are agreed before the all-gather, so no rank waits in it for a peer that raised, or gathers
    # shares it would read in another unit order
    packed, err, sig = None, None, 0
    try:
        sig = int(eng.k1_plan_signature(n, N))
        packed = eng.corr_shard(eng.to_device(X), rank, world)
    except Exception as e:   # noqa: BLE001 - must reach the agreement below
        err = e
    plan = ((sig * 1000003) ^ (packed.numel() if packed is not None else 0)) & ((1 << 62) - 1)
    failed, same = agree_value(err is not None, plan, device=cdev, group=group)
    if failed:
        raise_agreed(err, "sharded K1")
    if not same:
        raise _lib.PcgError(_lib.PCG_ERR_INVALID, "sharded K1: the ranks' K1 plans differ (PCG_TUNE_K1_* knobs)")
    if dist.get_backend(group) == "nccl":
        gathered = torch.empty(world * packed.numel(), dtype=torch.float64, device=eng.device)
        dist.all_gather_into_tensor(gathered, packed, group=group)
    else:   # gloo rehearsal (several ranks on one GPU)
        parts = [torch.empty_like(packed) for _ in range(world)]
        dist.all_gather(parts, packed, group=group)
        gathered = torch.cat(parts)
    return eng.corr_shard_finish(gathered, N, n, world)


def sharded_skeleton(eng, C, N: int, alpha: float = 0.05, max_depth: int = -1, flags: int = 0, group=None,
                     trace=None):
    """Edge-sharded skeleton over the ranks of ``group``; every rank returns the full result."""
    import time

    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    cdev = eng.device if dist.get_backend(group) == "nccl" else "cpu"
    for attempt in range(6):
        t0 = time.perf_counter()
        backend = agreed_backend(lambda: GpuLevelBackend(eng, C, N, alpha, flags, world), device=cdev, group=group)
        if trace is not None:
            trace.append(("init", -1, time.perf_counter() - t0))
        try:
            run_sharded_levels(backend, rank, world, max_depth=max_depth, group=group, trace=trace)
            break
        except _lib.PcgError as e:
            # an exact-path list overflowed on some rank; the merged status byte makes every
            # rank raise at the same level, capacities are already enlarged: rerun everywhere
            if e.code != _lib.PCG_ERR_OVERFLOW or attempt == 5:
                raise
            eng.lib.pcg_set_world_size(eng.h, 1)
    t0 = time.perf_counter()
    out, err = None, None
    try:
        out = backend.finish()
    except Exception as e:   # noqa: BLE001 - carried through the row-count exchange
        err = e
    xy, bits = _allgather_rows(out.sep_xy_dev if out else None, out.sep_bits_dev if out else None, group=group,
                               failed=err, device=cdev)
    out.sep_xy_dev, out.sep_bits_dev = xy, bits
    out._host.clear()
    out.stats = _allreduce_stats(out.stats, eng.device, group=group)
    if trace is not None:
        trace.append(("gather", -1, time.perf_counter() - t0))
    return out


def native_comm(eng, group=None) -> None:
    """Give ``eng`` an RCCL communicator over the ranks of ``group`` (pcg_comm_init): rank 0
    makes the unique id, the existing process group broadcasts its 128 bytes."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = eng.device if dist.get_backend(group) == "nccl" else "cpu"
    buf = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        buf.copy_(torch.frombuffer(bytearray(eng.comm_unique_id()), dtype=torch.uint8))
    dist.broadcast(buf, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    eng.comm_init(bytes(buf.cpu().numpy().tobytes()), rank, world)


class LocalGroup:
    """An in-process group of ``world`` engine handles for the native driver
    (``pcg_comm_group_create``): each rank is a handle driven from its own thread, and the
    driver's collectives are host-staged between them. RCCL refuses two ranks on one device, so
    this runs ``pcg_corr_sharded`` / ``pcg_skeleton_sharded`` — the C level loop bench.py uses at
    N > 1 — with world 2..8 on one GPU. Every collective is checked to be the same on every rank;
    a mismatch, a failing rank or a wait beyond ``timeout_s`` fails every rank with PCG_ERR_RCCL."""

    def __init__(self, world: int, timeout_s: float = 300.0):
        self.lib = _lib.load()
        g = ctypes.c_void_p()
        rc = self.lib.pcg_comm_group_create(int(world), float(timeout_s), ctypes.byref(g))
        if rc != 0:
            raise _lib.PcgError(rc, f"pcg_comm_group_create(world={world}) failed")
        self.g, self.world = g, int(world)

    def stats(self) -> dict:
        c, b, br = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        self.lib.pcg_comm_group_stats(self.g, ctypes.byref(c), ctypes.byref(b), ctypes.byref(br))
        return {"collectives": c.value, "bytes": b.value, "broken": bool(br.value)}

    def close(self):
        if self.g:
            rc = self.lib.pcg_comm_group_destroy(self.g)
            if rc != 0:
                raise _lib.PcgError(rc, "pcg_comm_group_destroy: a handle is still attached")
            self.g = None


def run_local_ranks(world: int, fn, device: int = 0, timeout_s: float = 300.0):
    """Run ``fn(eng, rank, world)`` on ``world`` threads, each with its own engine handle on
    ``device`` and its own torch stream, attached to one ``LocalGroup``. Returns the per-rank
    results in rank order (the first exception is re-raised after every thread ended)."""
    import threading

    import torch

    from .engine import Engine
    group = LocalGroup(world, timeout_s)
    out, errs = [None] * world, [None] * world

    def body(r):
        eng = None
        try:
            s = torch.cuda.Stream(device=device)
            with torch.cuda.stream(s):
                eng = Engine(device, stream=s)
                eng.comm_init_group(group, r)
                out[r] = fn(eng, r, world)
                s.synchronize()
        except BaseException as e:   # noqa: BLE001 - re-raised by the caller's thread
            errs[r] = e
        finally:
            if eng is not None:
                eng.comm_destroy()
                eng.close()

    threads = [threading.Thread(target=body, args=(r,), name=f"pcg-rank{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    stats = group.stats()
    group.close()
    for e in errs:
        if e is not None:
            raise e
    return out, stats


def native_sharded_corr(eng, X):
    """K1 sharded with the all-gather issued from C (needs ``native_comm`` first)."""
    return eng.corr_sharded(X)


def native_sharded_skeleton(eng, C, N: int, alpha: float = 0.05, max_depth: int = -1, flags: int = 0):
    """The edge-sharded skeleton with the whole level loop in C: per depth begin / split / run /
    pack / RCCL all-gather / merge / end on the handle's stream, then the counters summed and
    the sepset rows all-gathered (pcg_skeleton_sharded). Same result as ``sharded_skeleton``."""
    return eng.skeleton_sharded(C, N, alpha=alpha, max_depth=max_depth, flags=flags)


__all__ = ["agree", "agreed_backend", "split_by_work", "run_sharded_levels", "sharded_skeleton", "sharded_corr", "GpuLevelBackend",
           "native_comm", "native_sharded_corr", "native_sharded_skeleton", "LocalGroup", "run_local_ranks"]
_ = _lib
