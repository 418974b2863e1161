"""GPU: the native multi-GPU driver (pcg_corr_sharded / pcg_skeleton_sharded — the C level loop
bench.py runs at N > 1) at world 2, 3, 4 and 8 on ONE device, through the in-process transport
(pcg_comm_group_*: one handle per rank, each driven from its own thread and stream, host-staged
collectives). RCCL refuses two ranks on one device (rccl.h ncclCommInitRank), so this is how the
driver's rank-dependent steps run here: the per-depth pcg_level_split cut, the packed all-gather +
OR merge of the removal bits (the level barrier of SkeletonDiscovery.py:141-144), the stats
all-reduce and the sepset count / row gathers. Results are compared with the C oracle (cpc.skeleton
on np.corrcoef(X.T)) and with the single-GPU engine."""
import numpy as np
import pytest

from rcaeval_amd import synth

from tests_support import assert_skeleton_matches, unions_from_engine

pytestmark = pytest.mark.gpu


def _rank_run(X, N, max_depth, flags=0):
    def fn(eng, rank, world):
        Xd = eng.to_device(X)
        C = eng.corr_sharded(Xd)
        out = eng.skeleton_sharded(C, N, max_depth=max_depth, flags=flags)
        return {"C": C.cpu().numpy(), "rl": out.removed_level.copy(), "xy": out.sep_xy.copy(),
                "bits": out.sep_bits.copy(), "stats": out.stats, "near": list(out.near_alpha)}
    return fn


def _as_out(r):
    from types import SimpleNamespace
    return SimpleNamespace(removed_level=r["rl"], sep_xy=r["xy"], sep_bits=r["bits"], stats=r["stats"],
                           near_alpha=r["near"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n,N,seed,max_depth", [(2, 300, 1200, 3, -1), (3, 500, 3000, 5, -1),
                                                      (8, 700, 5000, 7, 4), (8, 300, 1200, 3, -1)])
def test_native_driver_world_matches_oracle(world, n, N, seed, max_depth):
    """Every rank of the native driver returns the oracle's skeleton: removal depth of every pair,
    per-level unique tests (summed over ranks by the stats all-reduce), sepset unions (gathered
    from every rank); C is bitwise the single-GPU K1 on every rank."""
    from oracle import cpc
    from rcaeval_amd.dist import run_local_ranks
    from rcaeval_amd.engine import get_engine
    X = synth.gaussian_sem(n, N, seed=seed)
    ref = cpc.skeleton(np.corrcoef(X.T), N, max_depth=max_depth, want_union=True)
    eng = get_engine(0)
    C1 = eng.corr(X).cpu().numpy()
    one = eng.skeleton(C1, N, max_depth=max_depth)
    res, gst = run_local_ranks(world, _rank_run(X, N, max_depth), timeout_s=240)
    assert not gst["broken"]
    # one all-gather per depth at least, plus the set-up / stats / sepset collectives
    assert gst["collectives"] >= one.stats["levels"] + 4
    for r in res:
        assert np.array_equal(r["C"], C1)
        assert_skeleton_matches(_as_out(r), ref, n)
        np.testing.assert_array_equal(r["rl"], one.removed_level)
        assert r["stats"]["tests"] == one.stats["tests"]
        assert r["stats"]["indep"] == one.stats["indep"]
        assert unions_from_engine(_as_out(r)) == unions_from_engine(one)
    # the work was split: with world ranks every rank still holds the same merged result
    assert all(np.array_equal(r["rl"], res[0]["rl"]) for r in res)


@pytest.mark.timeout(600)
def test_native_driver_full_p_records_world3():
    """FULL_P | RECORD through the native driver at world 3: the exact-path band tests and their
    near-alpha records on each rank's slice; the merged skeleton equals the single-GPU run."""
    from rcaeval_amd import _lib
    from rcaeval_amd.dist import run_local_ranks
    from rcaeval_amd.engine import get_engine
    X = synth.gaussian_sem(260, 900, seed=11)
    eng = get_engine(0)
    fl = _lib.PCG_FLAG_FULL_P
    one = eng.skeleton(eng.corr(X), 900, max_depth=-1, flags=fl)
    res, gst = run_local_ranks(3, _rank_run(X, 900, -1, flags=fl), timeout_s=240)
    assert not gst["broken"]
    for r in res:
        np.testing.assert_array_equal(r["rl"], one.removed_level)
        assert r["stats"]["tests"] == one.stats["tests"]
        assert r["stats"]["exact"] == one.stats["exact"]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_driver_config5_matches_oracle(config5, world):
    """North-star config 5 (2000 vars x 10 000 samples, depth 4) through the native C driver at
    world 2, 4 and 8 on one GPU: K1 sharded by CRT residue units (C bitwise numpy's to 2e-14 and
    identical on every rank), every depth's chunk list cut by pcg_level_split, the packed-bit barrier, the
    counters summed and the sepset rows gathered in C. Each rank's skeleton equals the oracle's."""
    from rcaeval_amd.dist import run_local_ranks
    X, Ch, ref = config5
    res, gst = run_local_ranks(world, _rank_run(X, 10000, 4), timeout_s=600)
    assert not gst["broken"]
    assert all(np.array_equal(res[0]["C"], r["C"]) for r in res)
    assert float(np.abs(res[0]["C"] - Ch).max()) <= 2e-14
    for r in res:
        assert_skeleton_matches(_as_out(r), ref, 2000)
        assert sum(r["stats"]["tests"]) > 4.5e9


def test_group_mismatched_collective_fails_every_rank_instead_of_hanging():
    """The transport's own check: ranks that issue different collectives (rank 0 a sharded K1,
    rank 1 a sharded skeleton — their first all-reduce matches, the second step does not) fail
    together with PCG_ERR_RCCL within the call, not by timeout. Over RCCL this would hang."""
    import time

    from rcaeval_amd import _lib
    from rcaeval_amd.dist import run_local_ranks
    from rcaeval_amd.engine import get_engine
    X = synth.gaussian_sem(300, 1200, seed=1)
    C = get_engine(0).corr(X).cpu().numpy()

    def fn(eng, rank, world):
        try:
            if rank == 0:
                eng.corr_sharded(eng.to_device(X))
            else:
                eng.skeleton_sharded(C, 1200, max_depth=2)
        except _lib.PcgError as e:
            return e.code
        return 0

    t0 = time.perf_counter()
    res, gst = run_local_ranks(2, fn, timeout_s=120)
    assert time.perf_counter() - t0 < 60
    assert gst["broken"]
    assert all(c == _lib.PCG_ERR_RCCL for c in res), res
