"""RQ2 scoring: the ``Evaluator`` interface of ``RCAEval/benchmark/evaluation.py:6-67``.

Stored per case is only where the answer first appears in the ranking (fine-grained: the
(service, metric) node; coarse-grained: its service, via ``Node.entity``), or ``None`` when it
is not in the top five. AC@k is then the fraction of cases whose first hit is below k, and
Avg@k the mean of AC@1..AC@k (summed in that order, so the floats equal the reference's).
Unknown k or an evaluator without cases gives ``None``, as in the reference.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from ..classes.graph import Node

TOP_K = 5


def first_hit(seq: Sequence, target) -> Optional[int]:
    """Index of the first element of ``seq[:TOP_K]`` equal to ``target`` (``in`` semantics)."""
    for i, item in enumerate(seq[:TOP_K]):
        if item is target or item == target:
            return i
    return None


class Evaluator:
    """AC@k / Avg@k over the cases added so far (k = 1..5)."""

    def __init__(self):
        self._hits: List[Optional[int]] = []          # fine-grained first-hit position per case
        self._service_hits: List[Optional[int]] = []  # coarse-grained (service) first-hit position

    def add_case(self, ranks: Sequence[Node], answer: Node):
        self._hits.append(first_hit(ranks, answer))
        self._service_hits.append(first_hit([node.entity for node in ranks[:TOP_K]], answer.entity))

    @property
    def num(self) -> int:
        return len(self._hits)

    @staticmethod
    def _ac(hits: List[Optional[int]], k: int):
        if k not in range(1, TOP_K + 1) or not hits:
            return None
        return float(sum(1 for h in hits if h is not None and h < k)) / len(hits)

    def _avg(self, hits: List[Optional[int]], k: int):
        if self._ac(hits, k) is None:
            return None
        total = 0.0
        for i in range(1, k + 1):
            total += self._ac(hits, i)
        return total / k

    def accuracy(self, k: int):
        return self._ac(self._hits, k)

    def accuracy_service(self, k: int):
        return self._ac(self._service_hits, k)

    def average(self, k: int):
        return self._avg(self._hits, k)

    def average_service(self, k: int):
        return self._avg(self._service_hits, k)


__all__ = ["Evaluator", "first_hit"]
