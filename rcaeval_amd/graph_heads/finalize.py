"""``finalize_directed_adj`` — mirror of ``RCAEval/graph_heads/__init__.py:6-79``.

Maps causal-learn endpoint codes (TAIL −1, ARROW 1, CIRCLE 2) to a 0/1
matrix with the reference's convention ``out[j, i] == 1`` ⇔ edge i → j (cause → effect):

    i → j (−1/1 or 0/1)   → out[j, i] = 1
    i — j (−1/−1)         → out[i, j] = out[j, i] = 1   (undirected becomes bidirected)
    i ↔ j (1/1), o-o      → both
    i o→ j (2/1)          → out[j, i] = 1

The reference visits every ordered pair (i, j) in row-major order, diagonal included, and
raises ``ValueError`` at the first pair it has no rule for; the vectorised form evaluates the
same rules for all pairs at once and raises for the same first pair with the same message.
"""
from __future__ import annotations

import numpy as np


def finalize_directed_adj(adj: np.ndarray) -> np.ndarray:
    """``graph_heads/__init__.py:6-79`` (output dtype = input dtype, like ``zeros_like``)."""
    adj = np.asarray(adj)
    a = adj            # adj[i, j]
    b = adj.T          # adj[j, i]
    # rules that write out[i, j] while visiting (i, j): cases 2.2, 2.4, 3, 4, 5.2, 6
    own = ((b == -1) & (a == 1)) | ((b == 0) & (a == 1)) | ((a == -1) & (b == -1)) \
        | ((a == 1) & (b == 1)) | ((a == 1) & (b == 2)) | ((a == 2) & (b == 2))
    # rules that write out[j, i] while visiting (i, j): cases 2.1, 2.3, 3, 4, 5.1, 6
    mirror = ((b == 1) & (a == -1)) | ((b == 1) & (a == 0)) | ((a == -1) & (b == -1)) \
        | ((a == 1) & (b == 1)) | ((a == 2) & (b == 1)) | ((a == 2) & (b == 2))
    known = own | mirror | ((a == 0) & (b == 0))
    if not known.all():
        i, j = (int(v) for v in np.argwhere(~known)[0])
        raise ValueError(f"Unexpected value: adj[i, j]={adj[i, j]!r}, adj[j, i]={adj[j, i]!r}")
    out = np.zeros_like(adj)
    out[own | mirror.T] = 1
    return out


__all__ = ["finalize_directed_adj"]
