"""rcaeval_amd — MI355X-native engine for RCAEval's PC-fisherz causal-graph path.

Drop-in surfaces (same names, arguments and return dicts as the reference):
  rcaeval_amd.e2e.pc_pagerank / pc_randomwalk      (RCAEval/e2e/pc_pagerank.py, pc_randomwalk.py)
  rcaeval_amd.graph_construction.pc.pc_default     (RCAEval/graph_construction/pc.py)
  rcaeval_amd.graph_heads.page_rank / random_walk  (RCAEval/graph_heads/*.py)
  rcaeval_amd.causal.pc                            (causal-learn pc(), fisherz, stable)
The compute runs in libpcgpu.so (HIP, gfx950); see include/pcgpu.h and DESIGN.md.
"""
__version__ = "0.1.0"
