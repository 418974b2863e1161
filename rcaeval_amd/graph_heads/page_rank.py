"""PageRank head — scikit-network 0.31.0 ``PageRank`` [U] semantics on the GPU (K4).

``PageRank`` mirrors ``sknetwork.ranking.PageRank(damping_factor=0.85, solver='piteration',
n_iter=10, tol=1e-6)`` as RCAEval uses it (``RCAEval/e2e/pc_pagerank.py:31-32``,
``RCAEval/graph_heads/page_rank.py:85-89``); the power iteration runs in
``pcg_pagerank_dense`` (rcaeval_amd/csrc/pagerank.hip). ``page_rank_preprocess`` and
``page_rank`` mirror ``RCAEval/graph_heads/page_rank.py:7-63`` and ``:66-94``.
"""
from __future__ import annotations

import numpy as np

from ..engine import get_engine


class PageRank:
    """GPU restatement of sknetwork's PageRank (power iteration only)."""

    def __init__(self, damping_factor: float = 0.85, solver: str = "piteration", n_iter: int = 10,
                 tol: float = 1e-6, verbose: bool = False):
        if solver != "piteration":
            raise NotImplementedError(f"solver={solver!r}: only 'piteration' (the RCAEval setting) is built")
        self.damping_factor = damping_factor
        self.solver = solver
        self.n_iter = n_iter
        self.tol = tol
        self.scores_ = None

    def fit(self, input_matrix, device: int | None = None) -> "PageRank":
        """Dense arrays run ``pcg_pagerank_dense``; scipy sparse input (sknetwork's other
        accepted format) runs ``pcg_pagerank_csr`` on its CSR form."""
        try:
            from scipy import sparse
        except ImportError:  # pragma: no cover - scipy is in the image
            sparse = None
        if sparse is not None and sparse.issparse(input_matrix):
            A = sparse.csr_matrix(input_matrix, dtype=np.float64)
            if A.shape[0] != A.shape[1]:
                raise ValueError("PageRank expects a square adjacency matrix (bipartite input not built)")
            if not A.count_nonzero():
                raise ValueError("The input matrix is empty.")   # sknetwork check_format [U]
            A.sort_indices()
            self.scores_ = get_engine(device).pagerank_csr(A.indptr, A.indices, A.data, A.shape[0],
                                                           self.damping_factor, self.n_iter, self.tol)
            return self
        A = np.asarray(input_matrix, dtype=np.float64)
        if A.ndim != 2 or A.shape[0] != A.shape[1]:
            raise ValueError("PageRank expects a square adjacency matrix (bipartite input not built)")
        if not np.count_nonzero(A):
            raise ValueError("The input matrix is empty.")   # sknetwork check_format [U]
        self.scores_ = get_engine(device).pagerank_dense(A, self.damping_factor, self.n_iter, self.tol)
        return self

    def fit_transform(self, input_matrix, device: int | None = None) -> np.ndarray:
        return self.fit(input_matrix, device=device).scores_


# (adj[a,b], adj[b,a]) -> (pr[a,b], pr[b,a]); None = leave untouched; missing key = error
_PAIR_RULES = {
    (0, 0): None, (-1, -1): (1, 1), (1, -1): (1, None), (-1, 1): (None, 1), (0, 1): (0, 1),
    (1, 0): (1, 0), (1, 1): (1, 1), (2, 1): (1, 0), (1, 2): (0, 1), (2, 2): (1, 1),
}
# every rule is its own mirror (rule(u, v) == reversed rule(v, u)), so both visits of a pair
# write the same value and pr[a, b] depends only on (adj[a,b], adj[b,a]): this table
_PAIR_VALUE = {k: (r[0] if r is not None and r[0] is not None else 0) for k, r in _PAIR_RULES.items()}


def page_rank_preprocess(adj: np.ndarray) -> np.ndarray:
    """Endpoint codes -> 0/1 matrix, pair rules of ``page_rank.py:7-63``, as one table lookup
    per cell; an unknown pair raises at the first row-major cell, like the reference loop."""
    adj = np.asarray(adj)
    out = np.zeros_like(adj)
    m = len(adj)
    if m == 0:
        return out
    A = adj.astype(np.int64, copy=False)
    known = np.zeros((m, m), bool)
    for (u, v), val in _PAIR_VALUE.items():
        hit = (A == u) & (A.T == v)
        known |= hit
        if val:
            out[hit] = val
    if not known.all():
        a, b = np.argwhere(~known)[0]
        raise ValueError(f"Unexpected value: {adj[a, b]}, {adj[b, a]}")
    return out


def page_rank(adj, node_names=None, damping_factor=0.85, solver="piteration", n_iter=10, tol=1e-6):
    """``page_rank`` head (``page_rank.py:66-94``): list of (name, score), score-descending."""
    if node_names is None:
        node_names = [f"X{i}" for i in range(len(adj))]
    pr_input = page_rank_preprocess(adj)
    scores = PageRank(damping_factor=damping_factor, solver=solver, n_iter=n_iter, tol=tol).fit_transform(pr_input)
    output = list(zip(node_names, scores))
    output.sort(key=lambda t: t[1], reverse=True)
    return output
