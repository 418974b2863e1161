"""Ranking heads on the GPU (mirror of ``RCAEval/graph_heads``)."""
from .finalize import finalize_directed_adj
from .page_rank import PageRank, page_rank, page_rank_preprocess
from .random_walk import random_walk

__all__ = ["finalize_directed_adj", "PageRank", "page_rank", "page_rank_preprocess", "random_walk"]
