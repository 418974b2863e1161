"""``Node`` and ``MemoryGraph`` — mirrors of ``RCAEval/classes/graph.py:35-73,157-221`` (what the
RQ2 scorer and the RQ1 graph metrics need).

A node is an (entity, metric) pair; equality and hashing are by both fields, so the
scorer's ``answer in ranks[:k]`` and ``service in service_ranks[:k]`` behave as in the
reference.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional

import networkx as nx
import numpy as np

from ..graph_heads.finalize import finalize_directed_adj


class Node:
    """``graph.py:35-73``."""

    __slots__ = ("_entity", "_metric")

    def __init__(self, entity: str, metric: str):
        self._entity = entity
        self._metric = metric

    @property
    def entity(self) -> str:
        return self._entity

    @property
    def metric(self) -> str:
        return self._metric

    def asdict(self) -> Dict[str, str]:
        return {"entity": self._entity, "metric": self._metric}

    def __eq__(self, obj: object) -> bool:
        if isinstance(obj, Node):
            return self.entity == obj.entity and self.metric == obj.metric
        return False

    def __hash__(self) -> int:
        return hash((self.entity, self.metric))

    def __repr__(self) -> str:
        return f"Node{(self.entity, self.metric)}"


class LoadingInvalidGraphException(Exception):
    """``graph.py:76-79``: a graph file without ``nodes`` / ``edges``."""


class MemoryGraph:
    """``graph.py:157-221``: a DiGraph (edge cause → effect) of ``Node`` (or plain) nodes."""

    def __init__(self, graph: nx.DiGraph):
        self._graph = graph
        self._nodes = set(graph.nodes)

    @property
    def nodes(self):
        return self._nodes

    @property
    def edges(self) -> List[tuple]:
        return [(i, j) for i, j in self._graph.edges]

    @property
    def str_edges(self):
        """``graph.py:122-129``: ``entity_metric`` pairs, or the raw edge view for plain nodes."""
        try:
            return [(f"{i.entity}_{i.metric}", f"{j.entity}_{j.metric}") for i, j in self._graph.edges]
        except Exception:
            return self._graph.edges

    def children(self, node, **kwargs):
        return set(self._graph.successors(node)) if self._graph.has_node(node) else set()

    def parents(self, node, **kwargs):
        return set(self._graph.predecessors(node)) if self._graph.has_node(node) else set()

    def dump(self, filename: str) -> bool:
        """``graph.py:170-178`` (``utility.dump_json``: indent 2, sorted keys)."""
        nodes = list(self._graph.nodes)
        index = {node: k for k, node in enumerate(nodes)}
        edges = [(index[c], index[e]) for c, e in self._graph.edges]
        try:
            data = dict(nodes=[node.asdict() for node in nodes], edges=edges)
        except Exception:
            data = dict(nodes=list(nodes), edges=edges)
        with open(filename, "w", encoding="utf-8") as f:
            json.dump(data, f, ensure_ascii=False, indent=2, sort_keys=True)
        return None

    @classmethod
    def load(cls, filename: str) -> Optional["MemoryGraph"]:
        """``graph.py:180-193``."""
        with open(filename, encoding="utf-8") as f:
            data = json.load(f)
        if "nodes" not in data or "edges" not in data:
            raise LoadingInvalidGraphException(filename)
        try:
            nodes = [Node(**node) for node in data["nodes"]]
        except Exception:
            nodes = list(data["nodes"])
        g = nx.DiGraph()
        g.add_nodes_from(nodes)
        g.add_edges_from((nodes[c], nodes[e]) for c, e in data["edges"])
        return cls(g)

    @classmethod
    def from_adj(cls, adj, nodes) -> "MemoryGraph":
        """``graph.py:195-210``: endpoint codes → ``finalize_directed_adj`` → edge
        ``nodes[j] → nodes[i]`` for every ``out[i, j] == 1`` (row-major insertion order)."""
        g = nx.DiGraph()
        g.add_nodes_from(nodes)
        if isinstance(adj, list) and len(adj) == 0:
            return cls(g)
        out = finalize_directed_adj(np.asarray(adj))
        ii, jj = np.nonzero(out == 1)
        g.add_edges_from((nodes[j], nodes[i]) for i, j in zip(ii.tolist(), jj.tolist()))
        return cls(g)


__all__ = ["Node", "MemoryGraph", "LoadingInvalidGraphException"]
