"""Random-walk head — mirror of ``RCAEval/graph_heads/random_walk.py:131-321`` on the GPU.

``random_walk(adj, node_names, sli, num_loop, previous_scores)`` builds the same reversed
graph (``:263-296``), the same transition matrix (``generate_transition_matrix`` :159-177,
columns = current node) and draws the walk with numpy's PCG64 stream for
``default_rng(seed=0)`` (``:148``) in ``pcg_random_walk`` (HIP): each step is
``Generator.choice(index, p=column)`` = searchsorted(cumsum(p)/cdf[-1], random(), 'right').
When every column is the same distribution (always true for ``previous_scores=None``, whose
scores are all 0 -> uniform columns, ``:171-177``) the draws are independent of the current
node and the kernel evaluates them in parallel via PCG64 jump-ahead.
"""
from __future__ import annotations

import numpy as np

from ..engine import get_engine

_RHO = 0.5


# endpoint-code pairs (adj[a, b], adj[b, a]) the reference's edge loop accepts (:271-294)
_VALID_PAIRS = {(0, 0), (-1, -1), (1, -1), (-1, 1), (0, 1), (1, 0), (1, 1)}


def _check_codes(adj: np.ndarray) -> None:
    """Raise like ``random_walk.py:293-294`` at the first (row-major) unknown code pair."""
    m = len(adj)
    if m == 0:
        return
    A = adj.astype(np.int64, copy=False)
    ok = np.zeros((m, m), bool)
    for u, v in _VALID_PAIRS:
        ok |= (A == u) & (A.T == v)
    if not ok.all():
        a, b = np.argwhere(~ok)[0]
        raise ValueError(f"Unexpected value: {adj[a, b]}, {adj[b, a]}")


def edge_matrix(adj: np.ndarray) -> np.ndarray:
    """E[u, v]: the nx edge u -> v before ``graph.reverse()`` (``:267-291``), as a bool matrix.

    Visit (a, b) adds b -> a for the pairs (-1,-1), (1,-1), (1,0), (1,1) and a -> b for (-1,1),
    (0,1), (1,1); over both visits of a pair that is a -> b  <=>  adj[b,a] == 1 or both are -1.
    """
    adj = np.asarray(adj)
    _check_codes(adj)
    A = adj.astype(np.int64, copy=False)
    return (A.T == 1) | ((A == -1) & (A.T == -1))


def transition_matrix(adj, node_names, names, score_values=None) -> np.ndarray:
    """Column-stochastic matrix of ``RandomWalkScorer.generate_transition_matrix`` (``:159-177``).

    ``node_names[a]`` names row/column a of ``adj``; ``names`` are the unique names in
    ``scores`` order (Node equality is by name); returns size x size with column c = the
    distribution of the next node from node c. Array form of the reference's per-node loop:
    on the reversed graph, children(c) = {u : u -> v in E, v ~ c} and parents(c) = {v : u -> v
    in E, u ~ c}; parents are written after children (``:160-169``), and each column's
    diagonal sees that column's max before it is set (``:171``).
    """
    adj = np.asarray(adj)
    m = len(adj)
    idx = {nm: i for i, nm in enumerate(names)}
    size = len(names)
    score = np.zeros(size) if score_values is None else np.asarray(score_values, dtype=float)
    E = edge_matrix(adj).astype(np.int64)
    Q = np.zeros((m, size), np.int64)
    Q[np.arange(m), [idx[node_names[a]] for a in range(m)]] = 1
    child = (Q.T @ E @ Q) > 0          # child[ch, c]: reversed edge c -> ch
    parent = (Q.T @ E.T @ Q) > 0       # parent[pa, c]: reversed edge pa -> c
    s = np.abs(score)
    M = np.zeros((size, size))
    M = np.where(child, _RHO * s[:, None], M)
    M = np.where(parent, s[:, None], M)
    diag = np.maximum(s - M.max(axis=0), 0.0) if size else s
    M[np.arange(size), np.arange(size)] = diag
    tot = np.ascontiguousarray(M.T).sum(axis=1)      # per-column pairwise sums, like Series.sum
    pos = tot > 0
    M[:, pos] = M[:, pos] / tot[pos]
    M[:, ~pos] = 1 / size
    return M


def random_walk(adj: np.ndarray, node_names=None, sli=None, num_loop=None, previous_scores=None,
                device: int | None = None):
    """``random_walk`` (``random_walk.py:249-321``): list of (name, score), score-descending."""
    adj = np.asarray(adj)
    if node_names is None:
        node_names = [f"X{i}" for i in range(len(adj))]
    _check_codes(adj)                         # raises on unknown endpoint pairs, like :293-294
    # sli = np.random.choice(nodes): same draw from numpy's global RandomState (:301)
    start_pos = int(np.random.choice(len(node_names)))
    uniq = list(dict.fromkeys(node_names))    # {Node(name): Score} dict semantics
    if previous_scores is None:
        values = None
    else:
        values = [previous_scores[nm] for nm in uniq]
    P = transition_matrix(adj, node_names, uniq, values)
    size = len(uniq)
    if num_loop is None:
        num_loop = size * 10                   # _times (:14-15)
    start = uniq.index(node_names[start_pos])
    bg = np.random.default_rng(0).bit_generator.state["state"]   # RandomWalkScorer seed=0 (:148)
    counts = get_engine(device).random_walk_counts(P, start, int(num_loop), int(bg["state"]), int(bg["inc"]))
    scores = [(nm, counts[i] / num_loop) for i, nm in enumerate(uniq)]
    scores.sort(key=lambda t: t[1], reverse=True)
    return scores
