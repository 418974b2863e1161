"""Ranking heads on the GPU (mirror of ``RCAEval/graph_heads``)."""
from .page_rank import PageRank, page_rank, page_rank_preprocess
from .random_walk import random_walk

__all__ = ["PageRank", "page_rank", "page_rank_preprocess", "random_walk"]
