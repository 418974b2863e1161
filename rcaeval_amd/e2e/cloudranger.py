"""``cloudranger`` — mirror of ``RCAEval/e2e/cloudranger.py:154-190`` on the MI355X engine.

PC-fisherz at ``alpha=0.1`` (stable, uc_priority 2) runs on the engine; the ranking head is
the vectorised second-order random walk of ``graph_heads.relato_rank``, seeded by the SLI
column and drawing from numpy's global RandomState exactly like the reference (callers that
want reproducible ranks seed ``np.random`` first, as with the reference). Like the reference
(no ``@rca``), errors — e.g. an SLI name absent from the columns — propagate.
"""
from __future__ import annotations

import numpy as np

from ..causal import pc
from ..graph_heads.finalize import finalize_directed_adj
from ..graph_heads.relato_rank import relaToRank
from ..io.time_series import preprocess


def calc_pearson(matrix, method="default", zero_diag=True):
    """``cloudranger.py:18-66`` — the ``method="numpy"`` branch the method uses."""
    if method != "numpy":
        raise NotImplementedError("calc_pearson(method='default') (pure-Python loops) is not used by cloudranger")
    res = np.corrcoef(np.array(matrix))
    if zero_diag:
        np.fill_diagonal(res, 0.0)
    return res


def cloudranger(data, inject_time=None, dataset=None, num_loop=None, sli=None, **kwargs):
    data = preprocess(data=data, dataset=dataset, dk_select_useful=kwargs.get("dk_select_useful", False))
    np_data = data.to_numpy()
    node_names = data.columns.to_list()
    sli = node_names.index(sli)
    pc_alpha, beta, rho = 0.1, 0.3, 0.2                      # cloudranger.py:165-169
    adj = pc(np_data.astype(float), show_progress=False, alpha=pc_alpha).G.graph
    rela = calc_pearson(np_data.T, method="numpy", zero_diag=False)
    dep_graph = finalize_directed_adj(adj).T
    rank, _, _ = relaToRank(rela, dep_graph, 10, sli, beta=beta, rho=rho)
    return {"adj": adj, "node_names": node_names, "ranks": [node_names[r - 1] for r, _ in rank]}


__all__ = ["calc_pearson", "cloudranger"]
