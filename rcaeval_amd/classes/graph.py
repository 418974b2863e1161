"""``Node`` — mirror of ``RCAEval/classes/graph.py:35-73`` (what the RQ2 scorer needs).

A node is an (entity, metric) pair; equality and hashing are by both fields, so the
scorer's ``answer in ranks[:k]`` and ``service in service_ranks[:k]`` behave as in the
reference.
"""
from __future__ import annotations

from typing import Dict


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


__all__ = ["Node"]
