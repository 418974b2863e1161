"""PC entry points — mirror of ``RCAEval/graph_construction/pc.py`` on the MI355X engine.

``pc_default`` (``pc.py:12-21``) is the path used by ``pc_randomwalk`` and CIRCA:
``pc(data.to_numpy().astype(float), node_names=..., show_progress=False,
background_knowledge=background_knowledge if with_bg else None)`` -> ``cg.G.graph``.
"""
from __future__ import annotations

from ..background import BackgroundKnowledge
from ..causal import fisherz, pc

# pc.py:6-9: memory / CPU metrics never cause a 50th-percentile latency, nothing causes a
# frontend metric
background_knowledge = BackgroundKnowledge()
background_knowledge.add_forbidden_by_pattern(".*mem$", ".*lat50$")
background_knowledge.add_forbidden_by_pattern(".*cpu$", ".*lat50$")
background_knowledge.add_forbidden_by_pattern(".*", "frontend.*")


def pc_default(data, show_progress=False, with_bg=False, **kwargs):
    """Endpoint-code adjacency (n x n int) of stable PC-fisherz (``pc.py:12-21``)."""
    names = data.columns.to_list()
    cg = pc(data.to_numpy().astype(float), node_names=names, show_progress=show_progress,
            background_knowledge=background_knowledge if with_bg else None)
    return cg.G.graph


def pc_fisherz_stable(data):
    """``pc.py:42-57``: stable PC with ``uc_priority=-1`` (uc_sepset's default priority 3: colliders
    ordered by the max p over neighbour power sets without the middle node, scored with
    batched device CI tests). Returns the ``CausalGraph``."""
    node_names = data.columns.to_list()
    return pc(data=data.to_numpy(), alpha=0.05, indep_test=fisherz, stable=True, uc_rule=0,
              uc_priority=-1, background_knowledge=None, show_progress=False, node_names=node_names)


def pc_fisherz(data):
    """``pc.py:24-39``: order-dependent PC (stable=False, ``rcaeval_amd.skeleton_seq``) with
    ``uc_priority=-1`` (priority 3). Returns the ``CausalGraph``."""
    node_names = data.columns.to_list()
    return pc(data=data.to_numpy(), alpha=0.05, indep_test=fisherz, stable=False, uc_rule=0,
              uc_priority=-1, background_knowledge=None, show_progress=False, node_names=node_names)


__all__ = ["background_knowledge", "pc_default", "pc_fisherz_stable", "pc_fisherz", "fisherz"]
