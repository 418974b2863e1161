"""FCI entry point — mirror of ``RCAEval/graph_construction/fci.py:5-14`` on the MI355X engine.

``fci_default``: forward-fill the frame (``data.fillna(method="ffill")``, ``:9``), then
``fci(data.to_numpy().astype(float), node_names=..., verbose=False)`` and return the PAG's
endpoint-code matrix (``output[0].graph``: TAIL -1, ARROW 1, CIRCLE 2).
"""
from __future__ import annotations

from ..fci import fci


def fci_default(data):
    node_names = data.columns.to_list()
    data = data.ffill()                       # fillna(method="ffill") (deprecated spelling in pandas 2)
    X = data.to_numpy().astype(float)
    output = fci(X, node_names=node_names, verbose=False)
    return output[0].graph


__all__ = ["fci_default"]
