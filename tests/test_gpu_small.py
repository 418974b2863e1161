"""GPU: the single-workgroup small-graph skeleton (k_pc_small, n <= 64: the RQ2 cases) against
the level loop (PCG_TUNE_SMALL = 0) and the C oracle: removal depths, per-level unique tests /
calls / independences / edges / max degree / degree snapshots, sepset union rows, near-alpha
lists, FULL_P | RECORD records, EXACT_ALL, background-knowledge bans, depth caps, constant (NaN)
columns, the singular and math-domain errors, and the n = 64 / 65 switch. Every run states which
driver produced it (pcg_stats.driver): a comparison of "small" with the level loop is only made
when the small kernel really ran; its fallback (a full band queue, or deeper than 16 levels) is
forced and checked on its own."""
import numpy as np
import pytest

from oracle import cpc
from oracle import fisherz
from rcaeval_amd import _lib, synth
from tests.tests_support import assert_skeleton_matches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from rcaeval_amd.engine import get_engine
    return get_engine(0)


def _run(eng, monkeypatch, small, C, N, expect=None, **kw):
    """One skeleton with PCG_TUNE_SMALL = small; the driver that produced it must be `expect`
    (default: "small" when small = "1", else "levels")."""
    with eng.tuned(SMALL=int(small)):
        out = eng.skeleton(C, N, **kw)
    want = expect or ("small" if small == "1" else "levels")
    assert out.stats["driver"] == want, (out.stats["driver"], want)
    return out


def _rows(out):
    xy = out.sep_xy.cpu().numpy() if hasattr(out.sep_xy, "cpu") else np.asarray(out.sep_xy)
    bits = out.sep_bits.cpu().numpy() if hasattr(out.sep_bits, "cpu") else np.asarray(out.sep_bits)
    return sorted((int(x), int(y), tuple(int(b) for b in row)) for (x, y), row in zip(xy, bits))


def _same(a, b):
    np.testing.assert_array_equal(a.removed_level, b.removed_level)
    for k in ("levels", "tests", "calls", "indep", "edges_after", "max_degree", "near_alpha", "error"):
        assert a.stats[k] == b.stats[k], k
    np.testing.assert_array_equal(a.deg_levels, b.deg_levels)
    assert _rows(a) == _rows(b)


CASES = [(2, 50, 0, .3, .9, None), (3, 40, 1, .3, .9, None), (12, 300, 2, .3, .9, .3), (20, 500, 1, .3, .9, None),
         (33, 700, 3, .1, .5, .2), (44, 600, 4, .2, .8, .1), (48, 2000, 5, .1, .3, .3), (64, 1000, 4, .2, .8, .08),
         (40, 400, 3, .1, .3, .3)]


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES)
@pytest.mark.parametrize("max_depth", [-1, 0, 2])
def test_small_equals_level_loop_and_oracle(eng, monkeypatch, n, N, seed, wl, wh, ep, max_depth):
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    s = _run(eng, monkeypatch, "1", C, N, max_depth=max_depth)
    lvl = _run(eng, monkeypatch, "0", C, N, max_depth=max_depth)
    _same(s, lvl)
    ref = cpc.skeleton(C, N, max_depth=max_depth)
    assert_skeleton_matches(s, ref, n)
    assert s.levels == ref.levels


@pytest.mark.parametrize("n,N,seed,wl,wh,ep", CASES[2:7])
@pytest.mark.parametrize("flags", [_lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD, _lib.PCG_FLAG_RECORD,
                                   _lib.PCG_FLAG_EXACT_ALL | _lib.PCG_FLAG_RECORD])
def test_small_records_equal_level_loop(eng, monkeypatch, n, N, seed, wl, wh, ep, flags):
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    C = np.corrcoef(X.T)
    # EXACT_ALL queues every test for the wave-per-test exact path: a depth of more than the band
    # queue's 1024 tests ends the small run and the level loop reruns (asserted below)
    exact_all = bool(flags & _lib.PCG_FLAG_EXACT_ALL)
    lvl = _run(eng, monkeypatch, "0", C, N, flags=flags, record_capacity=1_000_000)
    expect = "small_rerun" if exact_all and max(lvl.stats["tests"]) > 1024 else "small"
    s = _run(eng, monkeypatch, "1", C, N, expect=expect, flags=flags, record_capacity=1_000_000)
    _same(s, lvl)

    def recs(o):
        return {(int(r["a"]), int(r["b"]), tuple(int(v) for v in r["s"][: r["d"]])): float(r["p"]) for r in o.records}
    a, b = recs(s), recs(lvl)
    assert set(a) == set(b) and len(a) == sum(s.stats["tests"])
    k = sorted(a)
    assert fisherz.p_close([a[q] for q in k], [b[q] for q in k]).all()


def test_small_banned_pairs_equal_level_loop(eng, monkeypatch):
    n, N = 20, 800
    X = synth.gaussian_sem(n, N, seed=2, w_low=.2, w_high=.8, edge_prob=.2)
    C = np.corrcoef(X.T)
    ban = np.zeros((n, n), bool)
    for i, j in ((0, 1), (3, 7), (2, 9), (5, 6)):
        ban[i, j] = ban[j, i] = True
    s = _run(eng, monkeypatch, "1", C, N, banned=ban)
    lvl = _run(eng, monkeypatch, "0", C, N, banned=ban)
    _same(s, lvl)
    assert all(s.removed_level[i, j] == 0 for i, j in zip(*np.nonzero(ban)) if i != j)


def test_small_constant_column_runs_deep(eng, monkeypatch):
    X = synth.gaussian_sem(17, 400, seed=31, w_low=0.3, w_high=0.9, edge_prob=0.2)
    X[:, 4] = 1.0
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.corrcoef(X.T)
    ref = cpc.skeleton(C, 400)
    s = _run(eng, monkeypatch, "1", C, 400, expect="small" if ref.levels <= 17 else "small_rerun")
    lvl = _run(eng, monkeypatch, "0", C, 400)
    _same(s, lvl)
    assert s.levels == ref.levels > 13
    np.testing.assert_array_equal(s.removed_level, ref.removed_level)


def test_small_singular_and_domain_errors_like_level_loop(eng, monkeypatch):
    X = synth.gaussian_sem(12, 500, seed=1, w_low=.3, w_high=.9, edge_prob=.3)
    X[:, 7] = X[:, 2]
    C = np.corrcoef(X.T)
    for small in ("1", "0"):     # the engine raises causal-learn's ValueError [U] for both
        with pytest.raises(ValueError, match="singular"):
            with eng.tuned(SMALL=int(small)):
                eng.skeleton(C, 500)
    # N - d - 3 < 0: the reference's sqrt of a negative count (math domain error)
    X = synth.gaussian_sem(8, 5, seed=3, w_low=.5, w_high=1.0, edge_prob=.9)
    C = np.corrcoef(X.T)
    outcomes = []
    for small in ("1", "0"):
        try:
            with eng.tuned(SMALL=int(small)):
                out = eng.skeleton(C, 5)
            outcomes.append(("ok", out.removed_level.tolist()))
        except Exception as e:     # noqa: BLE001 - the two drivers must fail alike
            outcomes.append((type(e).__name__, str(e)))
    assert outcomes[0] == outcomes[1]


def test_small_switch_at_64(eng, monkeypatch):
    """n = 64 takes the small kernel, n = 65 the level loop: both equal the oracle."""
    for n in (64, 65):
        X = synth.gaussian_sem(n, 900, seed=n, w_low=.2, w_high=.8, edge_prob=.08)
        C = np.corrcoef(X.T)
        out = _run(eng, monkeypatch, "1", C, 900, expect="small" if n == 64 else "levels")
        assert_skeleton_matches(out, cpc.skeleton(C, 900), n)


def _near_collinear(n=40, N=800, noise=1e-4):
    """Near-duplicate columns: their tests fail the conditioning guard and queue for the exact
    path (the band queue) in threshold mode."""
    rng = np.random.default_rng(11)
    X = synth.gaussian_sem(n, N, seed=12, w_low=0.2, w_high=0.8, edge_prob=0.1)
    for j, i in ((5, 3), (17, 9), (30, 31), (22, 5)):
        X[:, j] = X[:, i] + noise * rng.standard_normal(N)
    return np.corrcoef(X.T), N


@pytest.mark.parametrize("qcap", [1, 4])
def test_small_band_queue_overflow_falls_back_to_level_loop(eng, monkeypatch, qcap):
    """A band queue smaller than a depth's exact-path tests (PCG_TUNE_SMALL_QCAP) ends the small
    run at that depth (status 8) and the level loop reruns the skeleton from scratch
    (PCG_DRIVER_SMALL_RERUN): the result equals the oracle and the level loop. With the default
    queue the same graph runs on the small kernel. (Round 4 kept deciding depths after such an
    overflow, from incomplete removals, and hung a parity test for 60 s)"""
    C, N = _near_collinear()
    ref = cpc.skeleton(C, N)
    if ref.error:
        pytest.skip("this draw is singular")
    full = _run(eng, monkeypatch, "1", C, N)
    assert max(full.stats["exact"]) > qcap            # some depth sent more tests to the exact path
    with eng.tuned(SMALL_QCAP=qcap):
        s = _run(eng, monkeypatch, "1", C, N, expect="small_rerun")
    lvl = _run(eng, monkeypatch, "0", C, N)
    _same(s, lvl)
    _same(full, lvl)
    assert_skeleton_matches(s, ref, C.shape[0])


def test_small_records_without_capacity_grow_the_buffer(monkeypatch):
    """PCG_FLAG_RECORD on a fresh handle (record capacity 0): the small kernel's record list
    overflows, the buffer grows and the small kernel runs again — every record is returned,
    equal to the oracle's (this used to fail with PCG_ERR_OVERFLOW)."""
    from rcaeval_amd.engine import Engine
    e = Engine(0)
    try:
        X = synth.gaussian_sem(24, 600, seed=3, w_low=0.3, w_high=0.9)
        C = np.corrcoef(X.T)
        out = _run(e, monkeypatch, "1", C, 600, flags=_lib.PCG_FLAG_RECORD)
        ref = cpc.skeleton(C, 600, record_cap=1 << 16)
        assert len(out.records) == len(ref.records) == sum(out.stats["tests"])
        assert_skeleton_matches(out, ref, 24)
    finally:
        e.close()
