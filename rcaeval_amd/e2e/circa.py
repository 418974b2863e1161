"""``circa`` — mirror of ``RCAEval/e2e/circa.py:15-41`` on the MI355X engine: preprocess, put
the ``time`` column back (last), stable PC-fisherz on the metric columns (``pc_default``, engine),
then the RHT head (``graph_heads.rht``) and a descending sort of its scores."""
from __future__ import annotations

from ..graph_construction.pc import pc_default
from ..graph_heads.rht import rht
from ..io.time_series import preprocess
from . import rca


@rca
def circa(data, inject_time=None, dataset=None, **kwargs):
    time_col = data["time"]
    data = preprocess(data=data, dataset=dataset, dk_select_useful=kwargs.get("dk_select_useful", False))
    data["time"] = time_col
    pc_input = data.drop(columns=["time"])
    adj = pc_default(pc_input, dataset="ob")
    ranks = rht(adj, inject_time, data)
    ranks = sorted(ranks, key=lambda x: x[1], reverse=True)
    return {"adj": adj, "node_names": data.columns.to_list(), "ranks": [x[0] for x in ranks]}


__all__ = ["circa"]
