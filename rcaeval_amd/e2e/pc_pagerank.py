"""``pc_pagerank`` — mirror of ``RCAEval/e2e/pc_pagerank.py:12-40`` on the MI355X engine.

preprocess -> ``pc(data.to_numpy())`` with causal-learn defaults (alpha 0.05, fisherz,
stable, uc_priority 2) -> directed graph from endpoint codes (``:20-27``) -> isolated nodes
dropped, remaining nodes sorted (``:28``) -> dense matrix as networkx 2.5
``to_numpy_matrix`` (``:29``) -> GPU PageRank on its transpose (``:31-32``) -> scores zipped
with the *unfiltered* ``node_names`` (``:33``: names and scores misalign, and the list is
truncated, whenever a node is isolated — reproduced on purpose) -> stable descending sort.
"""
from __future__ import annotations

import numpy as np

from ..causal import pc
from ..graph_heads.page_rank import PageRank
from ..io.time_series import preprocess
from ..phases import phase
from . import rca


def digraph_matrix(adj: np.ndarray):
    """(matrix, nodes) for ``pc_pagerank.py:20-29``: edge i->j when adj[i,j] == -1 or
    adj[j,i] == 1; nodes = sorted non-isolated; M[a,b] = 1.0 iff nodes[a] -> nodes[b]."""
    adj = np.asarray(adj)
    E = (adj == -1) | (adj == 1).T
    nodes = np.nonzero(E.any(axis=0) | E.any(axis=1))[0]
    M = E[np.ix_(nodes, nodes)].astype(np.float64)
    return M, [int(v) for v in nodes]


@rca
def pc_pagerank(data, inject_time=None, dataset=None, dk_select_useful=False, with_bg=False, n_iter=10,
                **kwargs):
    with phase("preprocess"):
        data = preprocess(data=data, dataset=dataset, dk_select_useful=dk_select_useful)
        node_names = data.columns.to_list()
        X = data.to_numpy()
    cg = pc(X)
    with phase("digraph"):
        M, _nodes = digraph_matrix(cg.G.graph)
    with phase("pagerank"):
        scores = PageRank().fit_transform(M.T)
    with phase("rank sort"):
        ranked = sorted(zip(node_names, scores), key=lambda t: t[1], reverse=True)
    return {"adj": M, "node_names": node_names, "ranks": [name for name, _ in ranked]}
