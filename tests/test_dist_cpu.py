"""CPU: the edge-sharded level protocol of rcaeval_amd.dist with gloo, world_size 2.

The GPU backend is replaced by an oracle-backed backend with the same begin/run/pack/merge/end
contract (chunks = (node x, run of S ranks), owner-disjoint evaluation, removal flags packed
as upper-triangle bits + a status word, all-gathered and OR-merged), so the partitioning, the
merge, the level barrier and the failure protocol are checked against the single-process
oracle skeleton without a GPU.
"""
import os
import socket
from itertools import combinations

import numpy as np
import pytest

from rcaeval_amd.dist import split_by_work


def test_split_by_work_tiles_and_balances():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 4, 8):
        w = rng.integers(0, 100, 1000)
        prefix = np.concatenate([[0], np.cumsum(w)])
        ranges = [split_by_work(prefix, r, world) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == 1000
        for (a, b), (c, d) in zip(ranges, ranges[1:]):
            assert b == c
        loads = [prefix[b] - prefix[a] for a, b in ranges]
        assert max(loads) - min(loads) <= 2 * w.max()
    assert split_by_work(np.array([0]), 0, 2) == (0, 0)


class OracleLevelBackend:
    """CPU stand-in for GpuLevelBackend (test only): same chunking and dedup rule."""

    CH = 3  # S ranks per chunk

    def __init__(self, C, N, alpha=0.05):
        import torch
        from oracle import fisherz
        self.C, self.N, self.alpha = C, N, alpha
        self.n = C.shape[0]
        self.adj = ~np.eye(self.n, dtype=bool)
        self.rl = np.full((self.n, self.n), -1, np.int64)
        self.rm = torch.zeros(self.n * self.n, dtype=torch.uint8)
        self.unions = {}
        self.depth = -1
        self.pv = lambda x, y, S: fisherz.pvalue(C, N, x, y, S)

    def begin(self, depth):
        deg = self.adj.sum(1)
        if not (deg.max() - 1 > depth - 1):
            return None
        self.depth = depth
        self.rm.zero_()
        self.chunks = []
        for x in range(self.n):
            nb = list(np.nonzero(self.adj[x])[0])
            if depth == 0:
                self.chunks.append((x, None, [y for y in nb if y > x]))
                continue
            if len(nb) < depth + 1:
                continue
            subsets = list(combinations(range(len(nb)), depth))
            for i in range(0, len(subsets), self.CH):
                self.chunks.append((x, nb, subsets[i:i + self.CH]))
        work = [len(c[2]) + 1 for c in self.chunks]
        return np.concatenate([[0], np.cumsum(work)]).astype(np.int64)

    def run(self, lo, hi):
        d = self.depth
        for x, nb, items in self.chunks[lo:hi]:
            if d == 0:
                for y in items:
                    if self.pv(x, y, ()) > self.alpha:
                        self.rm[x * self.n + y] = 1
                        self.rm[y * self.n + x] = 1
                continue
            for ks in items:
                S = [int(nb[k]) for k in ks]
                for y in nb:
                    if y in S:
                        continue
                    in_y = all(self.adj[y, s] for s in S)
                    if y < x and in_y:
                        continue
                    if self.pv(x, y, S) > self.alpha:
                        self.rm[x * self.n + y] = 1
                        self.rm[y * self.n + x] = 1
                        self.unions.setdefault((x, int(y), d), set()).update(S)
                        if in_y and y > x:
                            self.unions.setdefault((int(y), x, d), set()).update(S)

    def pack(self, local_error):
        """Upper-triangle bits of the flags (row-major pairs x < y) + one status byte."""
        import torch
        rm = self.rm.numpy().reshape(self.n, self.n).astype(bool)
        iu = np.triu_indices(self.n, 1)
        bits = np.packbits(rm[iu]) if not local_error else np.zeros((len(iu[0]) + 7) // 8, np.uint8)
        return torch.from_numpy(np.concatenate([bits, [8 if local_error else 0]]).astype(np.uint8))

    def merge(self, gathered, world):
        g = gathered.numpy().reshape(world, -1)
        merged = np.bitwise_or.reduce(g, axis=0)
        self.status = int(merged[-1])
        iu = np.triu_indices(self.n, 1)
        up = np.unpackbits(merged[:-1])[:len(iu[0])].astype(bool)
        rm = np.zeros((self.n, self.n), bool)
        rm[iu] = up
        rm |= rm.T
        self.rm.copy_(__import__("torch").from_numpy(rm.reshape(-1).astype(np.uint8)))

    def pack_failed(self):
        import torch
        iu = np.triu_indices(self.n, 1)
        return torch.from_numpy(np.concatenate([np.zeros((len(iu[0]) + 7) // 8, np.uint8), [8]]).astype(np.uint8))

    def end(self):
        from rcaeval_amd import _lib
        if self.status & 8:
            raise _lib.PcgError(_lib.PCG_ERR_PEER, "another rank failed at this depth")
        rm = self.rm.numpy().reshape(self.n, self.n).astype(bool)
        self.rl[rm] = self.depth
        self.adj &= ~rm


class FailingBackend(OracleLevelBackend):
    """Raises inside run() at one depth on one rank (failure-protocol test)."""

    def __init__(self, C, N, fail_rank, rank, fail_depth=1):
        super().__init__(C, N)
        self.fail = rank == fail_rank
        self.fail_depth = fail_depth

    def run(self, lo, hi):
        if self.fail and self.depth == self.fail_depth:
            raise MemoryError("injected local failure")
        super().run(lo, hi)


class FailingPackBackend(OracleLevelBackend):
    """Raises inside pack() at one depth on one rank: the rank must still join the gather."""

    def __init__(self, C, N, fail_rank, rank, fail_depth=1):
        super().__init__(C, N)
        self.fail = rank == fail_rank
        self.fail_depth = fail_depth

    def pack(self, local_error):
        if self.fail and self.depth == self.fail_depth:
            raise RuntimeError("injected pack failure")
        return super().pack(local_error)


def _worker(rank, world, port, C, N, q):
    import torch.distributed as dist
    from rcaeval_amd.dist import run_sharded_levels
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = OracleLevelBackend(C, N)
    run_sharded_levels(be, rank, world)
    unions = [None] * world
    dist.all_gather_object(unions, be.unions)
    dist.destroy_process_group()
    merged = {}
    for u in unions:
        for k, v in u.items():
            merged.setdefault(k, set()).update(v)
    q.put((rank, be.rl, merged))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_levels_match_single_process_oracle(world):
    import multiprocessing as mp
    from oracle import skeleton as osk
    from rcaeval_amd import synth
    n, N = 14, 600
    X = synth.gaussian_sem(n, N, seed=11, w_low=0.3, w_high=0.9, edge_prob=0.25)
    C = np.corrcoef(X.T)
    ref = osk.skeleton_discovery(C, N)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, C, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rl, merged in results:
        np.testing.assert_array_equal(rl, ref.removed_level)
        for (x, y, d), members in merged.items():
            lst = ref.sepset[x, y]
            side = set(int(v) for v in (lst[-2] if x < y else lst[-1]))
            assert ref.removed_level[x, y] == d
            assert members == side


def _fail_worker(rank, world, port, C, N, q):
    import torch.distributed as dist
    from rcaeval_amd import _lib
    from rcaeval_amd.dist import run_sharded_levels
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = FailingBackend(C, N, fail_rank=1, rank=rank)
    try:
        run_sharded_levels(be, rank, world)
        out = ("ok", be.depth)
    except MemoryError:
        out = ("own", be.depth)
    except _lib.PcgError as e:
        out = ("peer" if e.code == _lib.PCG_ERR_PEER else "other", be.depth)
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4])
def test_local_failure_reaches_every_rank_without_hanging(world):
    """A rank that fails inside its slice still joins the level's all-gather: it re-raises its
    own error and every peer raises PCG_ERR_PEER at the same depth (nobody waits forever)."""
    import multiprocessing as mp
    from rcaeval_amd import synth
    n, N = 12, 500
    X = synth.gaussian_sem(n, N, seed=4, w_low=0.3, w_high=0.9, edge_prob=0.3)
    C = np.corrcoef(X.T)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, C, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        kind, depth = res[r]
        assert kind == ("own" if r == 1 else "peer"), res
        assert depth == 1


def _setup_fail_worker(rank, world, port, C, N, mode, q):
    """mode 'init': rank 1's backend constructor fails (OOM-like); 'pack': rank 1's pack fails
    at depth 1; 'finish': rank 1 fails collecting its result before the sepset-row gather."""
    import torch.distributed as dist
    from rcaeval_amd import _lib
    from rcaeval_amd.dist import _allgather_rows, agreed_backend, run_sharded_levels
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = ("ok", -1)
    try:
        def factory():
            if mode == "init" and rank == 1:
                raise MemoryError("injected set-up failure")
            if mode == "pack":
                return FailingPackBackend(C, N, fail_rank=1, rank=rank)
            return OracleLevelBackend(C, N)
        be = agreed_backend(factory)
        run_sharded_levels(be, rank, world)
        if mode == "finish":
            import torch
            xy = torch.zeros((0, 2), dtype=torch.int32)
            bits = torch.zeros((0, 1), dtype=torch.int64)
            err = RuntimeError("injected finish failure") if rank == 1 else None
            _allgather_rows(xy, bits, failed=err, device="cpu")
        out = ("ok", be.depth)
    except (MemoryError, RuntimeError) as e:
        if isinstance(e, _lib.PcgError):
            out = ("peer" if e.code == _lib.PCG_ERR_PEER else "other", -1)
        else:
            out = ("own", -1)
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("mode", ["init", "pack", "finish"])
def test_failures_outside_run_reach_every_rank_without_hanging(mode):
    """Set-up, pack and result-collection failures on one rank: that rank raises its own error,
    every peer raises PCG_ERR_PEER, and no rank is left in a collective (world 3)."""
    import multiprocessing as mp
    from rcaeval_amd import synth
    world = 3
    n, N = 10, 400
    X = synth.gaussian_sem(n, N, seed=5, w_low=0.3, w_high=0.9, edge_prob=0.3)
    C = np.corrcoef(X.T)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_setup_fail_worker, args=(r, world, port, C, N, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r][0] == ("own" if r == 1 else "peer"), (mode, res)


def _gather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from rcaeval_amd.dist import _allgather_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    k = [5, 0, 3][rank]                      # ragged, one rank empty
    xy = torch.randint(0, 4000, (k, 2), generator=g, dtype=torch.int32)
    bits = torch.randint(-2**62, 2**62, (k, 3), generator=g, dtype=torch.int64)
    bits[:, 0] |= -2**63 if k else 0         # sign bit of the packed words survives
    out_xy, out_bits = _allgather_rows(xy, bits)
    dist.destroy_process_group()
    q.put((rank, xy.numpy(), bits.numpy(), out_xy.numpy(), out_bits.numpy()))


def test_allgather_rows_packs_ragged_ranks():
    """The sepset-row gather of the sharded skeleton (dist._allgather_rows): rows of every rank
    in rank order, (x, y) and all 64 bits of every union word preserved, empty ranks allowed."""
    import multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    want_xy = np.concatenate([r[1] for r in res])
    want_bits = np.concatenate([r[2] for r in res])
    for _, _, _, oxy, obits in res:
        np.testing.assert_array_equal(oxy, want_xy)
        np.testing.assert_array_equal(obits, want_bits)


class _FakeK1Engine:
    """Engine stand-in for dist.sharded_corr (test only): shares of 8 doubles per rank; rank 1
    fails ('fail'), sizes its share from another plan ('plan'), or has a plan of the same share
    size but another unit order ('sig', e.g. another split-K)."""
    device = "cpu"

    def __init__(self, rank, mode):
        self.rank, self.mode = rank, mode

    def to_device(self, X):
        import torch
        return torch.as_tensor(X)

    def k1_plan_signature(self, n, N):
        return (1 << 62) | (7 if (self.mode == "sig" and self.rank == 1) else 3) << 32

    def corr_shard(self, Xd, rank, world):
        import torch
        if self.mode == "fail" and rank == 1:
            raise MemoryError("injected residue-plane OOM")
        k = 9 if (self.mode == "plan" and rank == 1) else 8
        return torch.full((k,), float(rank), dtype=torch.float64)

    def corr_shard_finish(self, gathered, N, n, world):
        return gathered.clone()


def _k1_worker(rank, world, port, mode, q):
    import torch.distributed as dist
    from rcaeval_amd import _lib
    from rcaeval_amd.dist import sharded_corr
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = sharded_corr(_FakeK1Engine(rank, mode), np.zeros((6, 3)))
        res = ("ok", out.tolist())
    except MemoryError:
        res = ("own", None)
    except _lib.PcgError as e:
        res = ({_lib.PCG_ERR_PEER: "peer", _lib.PCG_ERR_INVALID: "invalid"}.get(e.code, "other"), None)
    dist.destroy_process_group()
    q.put((rank, res))


@pytest.mark.parametrize("mode", ["ok", "fail", "plan", "sig"])
def test_sharded_corr_agrees_failures_and_plans(mode):
    """dist.sharded_corr: shares gathered in rank order; a rank whose corr_shard raises re-raises
    its own error and every peer raises PCG_ERR_PEER before the all-gather; ranks whose K1 plans
    differ (shares of different sizes, or the same size in another unit order) all raise
    PCG_ERR_INVALID (nobody waits in the gather)."""
    import multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_k1_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        kind, out = res[r]
        if mode == "ok":
            assert kind == "ok" and out == [float(v) for v in range(world) for _ in range(8)]
        elif mode == "fail":
            assert kind == ("own" if r == 1 else "peer"), res
        else:
            assert kind == "invalid", res
