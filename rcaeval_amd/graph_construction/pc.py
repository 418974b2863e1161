"""PC entry points — mirror of ``RCAEval/graph_construction/pc.py`` on the MI355X engine.

``pc_default`` (``pc.py:12-21``) is the path used by ``pc_randomwalk`` and CIRCA:
``pc(data.to_numpy().astype(float), node_names=..., show_progress=False,
background_knowledge=None)`` -> ``cg.G.graph``.
"""
from __future__ import annotations

from ..causal import fisherz, pc


def pc_default(data, show_progress=False, with_bg=False, **kwargs):
    """Endpoint-code adjacency (n x n int) of stable PC-fisherz (``pc.py:12-21``)."""
    if with_bg:
        raise NotImplementedError("with_bg=True (background-knowledge patterns, pc.py:6-9) is a later-round item")
    names = data.columns.to_list()
    cg = pc(data.to_numpy().astype(float), node_names=names, show_progress=show_progress,
            background_knowledge=None)
    return cg.G.graph


def pc_fisherz_stable(data):
    """``pc.py:42-57`` calls pc(..., uc_priority=-1): causal-learn's default priority 3
    orientation, which issues extra CI tests over neighbour power sets — not built yet."""
    raise NotImplementedError("pc_fisherz_stable (uc_priority=-1 -> priority 3) is a later-round item; "
                              "use rcaeval_amd.causal.pc(data, uc_priority=2) for the RCAEval default")


def pc_fisherz(data):
    """``pc.py:24-39`` (stable=False) — order-dependent PC, a later-round item."""
    raise NotImplementedError("stable=False PC is a later-round item (SURVEY §8(f) rank 3)")


__all__ = ["pc_default", "pc_fisherz_stable", "pc_fisherz", "fisherz"]
