"""RQ2 scoring — mirror of ``RCAEval/benchmark/evaluation.py:6-67`` (``Evaluator``).

AC@k: the fraction of cases whose answer is among the top-k ranks (fine-grained: the
(service, metric) node; coarse-grained: the service, via ``Node.entity``). Avg@k: the mean
of AC@1..AC@k. Same accumulation order and return conventions (``None`` for an unknown k
or an empty evaluator) as the reference.
"""
from __future__ import annotations

from typing import List, Sequence

from ..classes.graph import Node


class Evaluator:
    """``RCAEval/benchmark/evaluation.py:6-67``."""

    def __init__(self):
        self._accuracy = {k: 0.0 for k in range(1, 6)}
        self._accuracy_service = {k: 0.0 for k in range(1, 6)}
        self._ranks: List[List[Node]] = []

    def add_case(self, ranks: Sequence[Node], answer: Node):
        """``evaluation.py:14-25``: keep the top 5, count hits at k = 1..5."""
        self._ranks.append(list(ranks[:5]))
        service_ranks = [n.entity for n in ranks]
        service_answer = answer.entity
        for k in range(1, 6):
            self._accuracy[k] += int(answer in ranks[:k])
            self._accuracy_service[k] += int(service_answer in service_ranks[:k])

    @property
    def num(self) -> int:
        return len(self._ranks)

    def accuracy(self, k: int):
        if k not in self._accuracy or not self._ranks:
            return None
        return self._accuracy[k] / self.num

    def accuracy_service(self, k: int):
        if k not in self._accuracy_service or not self._ranks:
            return None
        return self._accuracy_service[k] / self.num

    def average(self, k: int):
        if k not in self._accuracy or not self._ranks:
            return None
        return sum(self.accuracy(i) for i in range(1, k + 1)) / k

    def average_service(self, k: int):
        if k not in self._accuracy_service or not self._ranks:
            return None
        return sum(self.accuracy_service(i) for i in range(1, k + 1)) / k


__all__ = ["Evaluator"]
