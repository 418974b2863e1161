"""Scoring of RCA outputs (mirror of ``RCAEval/benchmark``)."""
from .evaluation import Evaluator
from .metrics import F1, F1_Skeleton, SHD

__all__ = ["Evaluator", "F1", "F1_Skeleton", "SHD"]
