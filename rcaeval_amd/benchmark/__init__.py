"""Scoring of RCA outputs (mirror of ``RCAEval/benchmark``)."""
from .evaluation import Evaluator

__all__ = ["Evaluator"]
