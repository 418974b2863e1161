"""scikit-network 0.31.0 ``PageRank`` (piteration) restatement — tests only.

[U] not on disk (requirements.txt:138). Restated from the pinned release:
``RandomSurferOperator``: a = (d * normalize(A, p=1)).T (CSR), b = (1 - d*out_deg)*seeds,
``_matvec(x) = a.dot(x) + b * x.sum()``; ``get_pagerank`` piteration loop with
``scores_ /= scores_.sum()`` and ``np.linalg.norm(scores - scores_, ord=1) < tol`` break;
``return scores / scores.sum()``. Uses scipy.sparse CSR mat-vec and numpy sums, i.e. the
exact arithmetic the reference would run. Call sites: RCAEval/e2e/pc_pagerank.py:31-32,
RCAEval/graph_heads/page_rank.py:85-89.
"""
from __future__ import annotations

import numpy as np
from scipy import sparse


def pagerank(input_matrix, damping_factor: float = 0.85, n_iter: int = 10, tol: float = 1e-6) -> np.ndarray:
    A = sparse.csr_matrix(np.asarray(input_matrix, dtype=float))
    if A.nnz == 0:
        raise ValueError("The input matrix is empty.")
    n = A.shape[0]
    seeds = np.ones(n) / n
    out_deg = A.dot(np.ones(n)).astype(bool)
    sums = abs(A).dot(np.ones(n))
    inv = np.zeros(n)
    nz = sums != 0
    inv[nz] = 1.0 / sums[nz]
    P = sparse.diags(inv, format="csr").dot(A)
    a = (damping_factor * P).T.tocsr()
    b = (np.ones(n) - damping_factor * out_deg) * seeds
    scores = b
    for _ in range(n_iter):
        s_ = a.dot(scores) + b * scores.sum()
        s_ /= s_.sum()
        if np.linalg.norm(scores - s_, ord=1) < tol:
            break
        scores = s_
    return scores / scores.sum()
