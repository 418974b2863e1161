"""``pc_randomwalk`` / ``fci_randomwalk`` — mirrors of ``RCAEval/e2e/pc_randomwalk.py:10-30`` and
``:53-72`` on the MI355X engine. ``random_walk`` raises on a circle mark (``random_walk.py:293-294``),
so an FCI PAG with any o-* edge ends in ``@rca``'s dummy ranking, as in the reference."""
from __future__ import annotations

from ..graph_construction.fci import fci_default
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


@rca
def fci_randomwalk(data, inject_time=None, dataset=None, n_iter=None, **kwargs):
    data = preprocess(data=data, dataset=dataset, dk_select_useful=kwargs.get("dk_select_useful", False))
    node_names = data.columns.to_list()
    if n_iter is None:
        n_iter = len(node_names)
    adj = fci_default(data)
    ranks = random_walk(adj, node_names, num_loop=n_iter)
    ranks = sorted(ranks, key=lambda t: t[1], reverse=True)
    return {"adj": adj, "node_names": node_names, "ranks": [name for name, _ in ranks]}
