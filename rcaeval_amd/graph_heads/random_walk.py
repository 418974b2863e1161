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


def _edges_from_adj(adj: np.ndarray, m: int):
    """Directed edges (u, v) of the nx graph before ``graph.reverse()`` (``:267-291``)."""
    edges = []
    for a in range(m):
        for b in range(m):
            ab, ba = int(adj[a, b]), int(adj[b, a])
            if ab == ba == 0:
                continue
            if ab == ba == -1:
                edges.append((b, a))
            elif ab == 1 and ba == -1:
                edges.append((b, a))
            elif ab == -1 and ba == 1:
                edges.append((a, b))
            elif ab == 0 and ba == 1:
                edges.append((a, b))
            elif ab == 1 and ba == 0:
                edges.append((b, a))
            elif ab == 1 and ba == 1:
                edges.append((a, b))
                edges.append((b, a))
            else:
                raise ValueError(f"Unexpected value: {adj[a, b]}, {adj[b, a]}")
    return edges


def transition_matrix(adj, node_names, names, score_values=None) -> np.ndarray:
    """Column-stochastic matrix of ``RandomWalkScorer.generate_transition_matrix`` (``:159-177``).

    ``node_names[a]`` names row/column a of ``adj``; ``names`` are the unique names in
    ``scores`` order (Node equality is by name); returns size x size with column c = the
    distribution of the next node from node c.
    """
    adj = np.asarray(adj)
    m = len(adj)
    idx = {nm: i for i, nm in enumerate(names)}
    size = len(names)
    score = np.zeros(size) if score_values is None else np.asarray(score_values, dtype=float)
    # graph on Node(name): node a of adj maps to names index of its (deduplicated) name
    children = [set() for _ in range(size)]
    parents = [set() for _ in range(size)]
    node_of = [idx[node_names[a]] for a in range(m)]
    for u, v in _edges_from_adj(adj, m):
        # reversed graph: edge v -> u; children(v) gets u, parents(u) gets v
        cu, cv = node_of[u], node_of[v]
        children[cv].add(cu)
        parents[cu].add(cv)
    M = np.zeros((size, size))
    for c in range(size):
        for ch in children[c]:
            M[ch, c] = _RHO * abs(score[ch])
        for pa in parents[c]:
            M[pa, c] = abs(score[pa])
        M[c, c] = max(abs(score[c]) - M[:, c].max(), 0)
        tot = M[:, c].sum()
        if tot > 0:
            M[:, c] = M[:, c] / tot
        else:
            M[:, c] = 1 / size
    return M


def random_walk(adj: np.ndarray, node_names=None, sli=None, num_loop=None, previous_scores=None,
                device: int | None = None):
    """``random_walk`` (``random_walk.py:249-321``): list of (name, score), score-descending."""
    adj = np.asarray(adj)
    if node_names is None:
        node_names = [f"X{i}" for i in range(len(adj))]
    _edges_from_adj(adj, len(adj))            # raises on unknown endpoint pairs, like :293-294
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
