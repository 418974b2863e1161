"""``pc_randomwalk`` — mirror of ``RCAEval/e2e/pc_randomwalk.py:10-30`` on the MI355X engine."""
from __future__ import annotations

from ..graph_construction.pc import pc_default
from ..graph_heads.random_walk import random_walk
from ..io.time_series import preprocess
from . import rca


@rca
def pc_randomwalk(data, inject_time=None, dataset=None, n_iter=None, **kwargs):
    data = preprocess(data=data, dataset=dataset, dk_select_useful=kwargs.get("dk_select_useful", False))
    node_names = data.columns.to_list()
    if n_iter is None:
        n_iter = len(node_names)
    adj = pc_default(data)
    ranks = random_walk(adj, node_names, num_loop=n_iter)
    ranks = sorted(ranks, key=lambda t: t[1], reverse=True)
    return {"adj": adj, "node_names": node_names, "ranks": [name for name, _ in ranks]}
