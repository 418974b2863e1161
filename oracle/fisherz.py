"""Fisher-z conditional-independence test — CPU oracle (test infrastructure only).

Restates causal-learn 0.1.3.3 ``utils/cit.py`` ``FisherZ`` [U] (not on disk; pinned by
``requirements.txt:20``; call sites ``RCAEval/e2e/pc_pagerank.py:19``,
``RCAEval/graph_construction/pc.py:15``) with exactly the library calls it makes:

    __init__ : correlation_matrix = np.corrcoef(data.T)
    __call__ : var = [min(x,y), max(x,y)] + sorted(S)
               sub = C[np.ix_(var, var)]
               inv = np.linalg.inv(sub)            # LinAlgError -> ValueError
               r   = -inv[0,1] / math.sqrt(inv[0,0]*inv[1,1])
               Z   = 0.5 * math.log((1 + r) / (1 - r))
               X   = math.sqrt(N - |S| - 3) * abs(Z)
               p   = 2 * (1 - norm.cdf(abs(X)))

The skeleton cache key is ``(min(x,y), max(x,y), frozenset(S))``
(``lib/causallearn/graph/GraphClass.py:87-90``).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.stats import norm


def check_input(data: np.ndarray) -> None:
    """causal-learn ``CIT_Base.assert_input_data_is_valid`` [U]: no NaN, no inf."""
    assert not np.isnan(data).any(), "Input data contains NaN. Please check."
    assert not np.isinf(data).any(), "Input data contains Inf. Please check."


def corrcoef(data: np.ndarray) -> np.ndarray:
    """``FisherZ.__init__`` [U]: ``np.corrcoef(data.T)`` on an N x n array."""
    return np.corrcoef(np.asarray(data, dtype=float).T)


def pvalue(C: np.ndarray, N: int, x: int, y: int, S) -> float:
    """One Fisher-z test, exactly the [U] expression (see module docstring)."""
    a, b = (int(x), int(y)) if x < y else (int(y), int(x))
    cond = sorted(set(int(s) for s in S))
    var = [a, b] + cond
    sub = C[np.ix_(var, var)]
    try:
        inv = np.linalg.inv(sub)
    except np.linalg.LinAlgError:
        raise ValueError(
            "Data correlation matrix is singular. Cannot run fisherz test. Please check your data."
        )
    r = -inv[0, 1] / math.sqrt(inv[0, 0] * inv[1, 1])
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = (1 + r) / (1 - r)
    Z = 0.5 * math.log(ratio)
    X = math.sqrt(N - len(cond) - 3) * abs(Z)
    return float(2 * (1 - norm.cdf(abs(X))))


def pvalue_from_r(r: float, N: int, d: int) -> float:
    """p from a partial correlation using the same expression (no matrix step)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = (1 + np.float64(r)) / (1 - np.float64(r))
    Z = 0.5 * math.log(ratio)
    X = math.sqrt(N - d - 3) * abs(Z)
    return float(2 * (1 - norm.cdf(abs(X))))


def p_close(p_dev: np.ndarray, p_ref: np.ndarray, rel: float = 1e-9) -> np.ndarray:
    """North-star tolerance: |dp| <= rel*|p_ref| + 2^-51.

    The absolute floor covers the 2^-53 grid of ``1 - cdf`` that the reference's
    ``2*(1 - norm.cdf(X))`` cancellation imposes on small p. NaN matches NaN.
    """
    p_dev = np.asarray(p_dev, dtype=float)
    p_ref = np.asarray(p_ref, dtype=float)
    both_nan = np.isnan(p_dev) & np.isnan(p_ref)
    ok = np.abs(p_dev - p_ref) <= rel * np.abs(p_ref) + 2.0 ** -51
    return ok | both_nan
