"""GPU: the single-workgroup small-graph skeleton (k_pc_small, n <= 64: the RQ2 cases) against
the level loop (PCG_SMALL=0) and the C oracle: removal depths, per-level unique tests / calls /
independences / edges / max degree / degree snapshots, sepset union rows, near-alpha lists,
FULL_P | RECORD records, EXACT_ALL, background-knowledge bans, depth caps, constant (NaN)
columns, the singular and math-domain errors, and the n = 64 / 65 switch."""
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


def _run(eng, monkeypatch, small, C, N, **kw):
    monkeypatch.setenv("PCG_SMALL", small)
    return eng.skeleton(C, N, **kw)


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
    s = _run(eng, monkeypatch, "1", C, N, flags=flags, record_capacity=1_000_000)
    lvl = _run(eng, monkeypatch, "0", C, N, flags=flags, record_capacity=1_000_000)
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
    s = _run(eng, monkeypatch, "1", C, 400)
    lvl = _run(eng, monkeypatch, "0", C, 400)
    _same(s, lvl)
    ref = cpc.skeleton(C, 400)
    assert s.levels == ref.levels > 13
    np.testing.assert_array_equal(s.removed_level, ref.removed_level)


def test_small_singular_and_domain_errors_like_level_loop(eng, monkeypatch):
    X = synth.gaussian_sem(12, 500, seed=1, w_low=.3, w_high=.9, edge_prob=.3)
    X[:, 7] = X[:, 2]
    C = np.corrcoef(X.T)
    for small in ("1", "0"):     # the engine raises causal-learn's ValueError [U] for both
        with pytest.raises(ValueError, match="singular"):
            _run(eng, monkeypatch, small, C, 500)
    # N - d - 3 < 0: the reference's sqrt of a negative count (math domain error)
    X = synth.gaussian_sem(8, 5, seed=3, w_low=.5, w_high=1.0, edge_prob=.9)
    C = np.corrcoef(X.T)
    outcomes = []
    for small in ("1", "0"):
        try:
            out = _run(eng, monkeypatch, small, C, 5)
            outcomes.append(("ok", out.removed_level.tolist()))
        except Exception as e:     # noqa: BLE001 - the two drivers must fail alike
            outcomes.append((type(e).__name__, str(e)))
    assert outcomes[0] == outcomes[1]


def test_small_switch_at_64(eng, monkeypatch):
    """n = 64 takes the small kernel, n = 65 the level loop: both equal the oracle."""
    for n in (64, 65):
        X = synth.gaussian_sem(n, 900, seed=n, w_low=.2, w_high=.8, edge_prob=.08)
        C = np.corrcoef(X.T)
        out = _run(eng, monkeypatch, "1", C, 900)
        assert_skeleton_matches(out, cpc.skeleton(C, 900), n)
