"""``fci_pagerank`` — mirror of ``RCAEval/e2e/fci_pagerank.py:7-20`` on the MI355X engine:
preprocess -> FCI PAG (``fci_default``) -> ``page_rank(adj, node_names, n_iter)`` (the
``page_rank_preprocess`` pair rules turn circle marks into edges) -> score-descending ranks."""
from __future__ import annotations

from ..graph_construction.fci import fci_default
from ..graph_heads.page_rank import page_rank
from ..io.time_series import preprocess
from . import rca


@rca
def fci_pagerank(data, inject_time=None, dataset=None, dk_select_useful=False, n_iter=10, **kwargs):
    data = preprocess(data=data, dataset=dataset, dk_select_useful=dk_select_useful)
    node_names = data.columns.to_list()
    adj = fci_default(data)
    ranks = page_rank(adj, node_names=node_names, n_iter=n_iter)
    ranks = sorted(ranks, key=lambda x: x[1], reverse=True)
    return {"adj": adj, "node_names": node_names, "ranks": [x[0] for x in ranks]}
