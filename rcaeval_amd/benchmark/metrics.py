"""RQ1 graph-quality metrics — mirror of ``RCAEval/benchmark/metrics.py:8-99``.

``F1`` / ``F1_Skeleton`` compare ``str_edges`` sets exactly as the reference does (set
intersection of directed pairs; the skeleton variant doubles every edge first). ``SHD`` is the
reference's pairwise case analysis over ``combinations(G1.nodes(), 2)`` evaluated on two 0/1
matrices aligned on G1's node order instead of one ``has_edge`` call per pair (n(n−1)/2 Python
iterations ⇒ one vectorised pass). The four SHD cases are mutually exclusive in the reference's
``elif`` chain and each adds 1, so the count is the number of pairs matching any of them.
"""
from __future__ import annotations

import numpy as np

from ..classes.graph import MemoryGraph


def _aligned(g1, g2):
    """Dense 0/1 matrices of G1 and G2 over G1's node order (G2-only nodes drop out; G1 nodes
    absent from G2 have no edges there — ``has_edge`` returns False for them)."""
    nodes = list(g1.nodes())
    index = {v: k for k, v in enumerate(nodes)}
    n = len(nodes)
    a1 = np.zeros((n, n), dtype=bool)
    a2 = np.zeros((n, n), dtype=bool)
    for g, a in ((g1, a1), (g2, a2)):
        for u, v in g.edges():
            iu, iv = index.get(u), index.get(v)
            if iu is not None and iv is not None:
                a[iu, iv] = True
    return a1, a2


def SHD(G1: MemoryGraph, G2: MemoryGraph) -> int:
    """``metrics.py:28-55``."""
    a1, a2 = _aligned(G1._graph, G2._graph)
    i, j = np.triu_indices(a1.shape[0], k=1)      # combinations(nodes, 2) pairs
    f1, b1 = a1[i, j], a1[j, i]
    f2, b2 = a2[i, j], a2[j, i]
    any1, any2 = f1 | b1, f2 | b2
    missing = any1 & ~any2                          # in G1, absent from G2
    extra = ~any1 & any2                            # absent from G1, present in G2
    undirected_vs_directed = (f1 & b1) & (f2 ^ b2)
    wrong_direction = (f1 & ~b1 & b2) | (b1 & ~f1 & f2)
    return int(np.count_nonzero(missing | extra | undirected_vs_directed | wrong_direction))


def _prf(tp: int, n_est: int, n_true: int) -> dict:
    if tp == 0:
        return {"precision": 0, "recall": 0, "f1": 0}
    pre = tp / n_est
    rec = tp / n_true
    return {"precision": pre, "recall": rec, "f1": 2 * pre * rec / (pre + rec)}


def F1(true_graph: MemoryGraph, est_graph: MemoryGraph) -> dict:
    """``metrics.py:58-71``: directed-edge precision / recall / F1 (``len`` of the edge lists,
    not of their sets, in the denominators — as in the reference)."""
    true_edges, est_edges = true_graph.str_edges, est_graph.str_edges
    tp = len(set(true_edges) & set(est_edges))
    return _prf(tp, len(est_edges), len(true_edges))


def F1_Skeleton(true_graph: MemoryGraph, est_graph: MemoryGraph) -> dict:
    """``metrics.py:74-99``: both orientations of every edge, as sets."""
    def doubled(edges):
        out = set()
        for a, b in edges:
            out.add((a, b))
            out.add((b, a))
        return out
    t, e = doubled(true_graph.str_edges), doubled(est_graph.str_edges)
    return _prf(len(t & e), len(e), len(t))


__all__ = ["F1", "F1_Skeleton", "SHD"]
