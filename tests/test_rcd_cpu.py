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
