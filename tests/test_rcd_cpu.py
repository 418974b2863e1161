"""CPU: RCD's discrete CI test oracle (oracle/chisq.py) pinned to scipy's contingency test,
and the RCD host logic (rcaeval_amd.rcd) driven by the oracle skeleton (no device)."""
import numpy as np
import pytest
from scipy.stats import chi2_contingency

from oracle import chisq as och


@pytest.mark.parametrize("seed", range(8))
def test_unconditional_chisq_equals_scipy_contingency(seed):
    rng = np.random.default_rng(seed)
    cx, cy = int(rng.integers(2, 6)), int(rng.integers(2, 6))
    N = int(rng.integers(50, 3000))
    x = rng.integers(0, cx, N)
    y = (x + rng.integers(0, cy, N) * (seed % 2)) % cy
    codes = np.stack([x, y], 1)
    card = np.array([cx, cy])
    stat, df = och.chisq_or_gsq_stat(codes.T, card)
    table = np.zeros((cx, cy))
    np.add.at(table, (x, y), 1)
    keep_r, keep_c = table.sum(1) > 0, table.sum(0) > 0
    ref = chi2_contingency(table[keep_r][:, keep_c], correction=False)
    assert df == ref.dof
    np.testing.assert_allclose(stat, ref.statistic, rtol=1e-12)
    g, _ = och.chisq_or_gsq_stat(codes.T, card, G_sq=True)
    refg = chi2_contingency(table[keep_r][:, keep_c], correction=False, lambda_="log-likelihood")
    np.testing.assert_allclose(g, refg.statistic, rtol=1e-12)


def test_conditional_chisq_is_sum_of_stratum_tests():
    """With S, the statistic and df are the sums of the per-stratum unconditional tests."""
    rng = np.random.default_rng(3)
    N = 4000
    s = rng.integers(0, 3, N)
    x = (s + rng.integers(0, 2, N)) % 4
    y = (s + rng.integers(0, 3, N)) % 4
    codes = np.stack([s, x, y], 1)
    stat, df = och.chisq_or_gsq_stat(codes.T, np.array([3, 4, 4]))
    tot, tdf = 0.0, 0
    for k in range(3):
        m = s == k
        st_k, df_k = och.chisq_or_gsq_stat(np.stack([x[m], y[m]]), np.array([4, 4]))
        tot += st_k
        tdf += df_k
    np.testing.assert_allclose(stat, tot, rtol=1e-12)
    assert df == tdf


def test_order_neighbors_matches_reference_list_argmax():
    from rcaeval_amd.rcd import _order_neighbors
    p = np.empty(4, object)
    p[0], p[1], p[2], p[3] = [0.01, 0.2], [0.3], [0.01, 0.5], [0.3]
    assert _order_neighbors(["a", "b", "c", "d"], p) == ["a", "c", "d", "b"]


def test_chisq_oversize_table_is_marked_per_test_not_per_batch():
    """A test whose contingency table exceeds MAX_CELLS gets status 4 (raised only when the
    caller consumes it); the other tests of the batch still run on the device."""
    from rcaeval_amd.rcd import ChiSqTester

    class _Eng:
        def __init__(self):
            self.rows = None

        def chisq_batch(self, data, card, N, n, rows, g_sq, cells):
            self.rows = rows.copy()
            assert cells <= ChiSqTester.MAX_CELLS
            k = len(rows)
            return np.full(k, 3.0), np.full(k, 2), np.zeros(k, np.int32)

    ci = ChiSqTester.__new__(ChiSqTester)
    ci.eng, ci.N, ci.n = _Eng(), 100, 6
    ci.card = np.array([2, 2, 1 << 13, 1 << 13, 2, 2])
    ci.data = ci.card_dev = None
    ci.g_sq, ci.cache, ci.no_ci_tests = False, {}, 0
    p, st = ci.pvalues_status([(0, 1, (4,)), (0, 1, (2, 3)), (0, 4, (5,))])
    assert st == [0, 4, 0] and np.isnan(p[1]) and p[0] == p[2] > 0
    assert len(ci.eng.rows) == 2
    with pytest.raises(NotImplementedError):
        ci.raise_for(st[1])


def test_rcd_frame_glue_matches_reference_executed_golden():
    """Sock-Shop cleaning, constant dropping, F-node discretisation, chunking and neighbour
    order against outputs of the reference's own functions (tests/golden/make_rcd_glue_golden.py)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_rcd_glue_golden as G
    from rcaeval_amd import rcd as M
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rcd_glue.json")))
    assert len(gold) == 12
    for rec in gold:
        t = rec["case"]
        df = G.case_frame(t)
        n_df, a_df = df.iloc[:20].copy(), df.iloc[20:].copy()
        if t % 3 == 0:
            a_df = a_df.drop(columns=[df.columns[3]])
        for su in (False, True):
            nn, aa = M.preprocess_sock_shop(n_df.copy(), a_df.copy(), 90, su)
            want = rec[f"sock_shop_{int(su)}"]
            assert list(nn.columns) == want["columns"]
            assert G.frame_digest(nn) == want["normal"] and G.frame_digest(aa) == want["anomalous"]
        assert list(M.drop_constant(df).columns) == rec["drop_constant"]
        np.random.seed(rec["chunks"]["seed"])
        assert [list(c) for c in M.create_chunks(df, rec["chunks"]["gamma"])] == rec["chunks"]["chunks"]
        assert M._order_neighbors([f"v{i}" for i in range(6)], G.case_pvalues(t)) == rec["order"]
        disc = M._preprocess_for_fnode(df.iloc[:20, 1:7].copy(), df.iloc[20:, 1:7].copy(), 5)
        assert list(disc.columns) == rec["discretized"]["columns"]
        assert G.frame_digest(disc) == rec["discretized"]["digest"]
