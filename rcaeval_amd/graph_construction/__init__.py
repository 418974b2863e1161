"""Graph construction on the GPU (mirror of ``RCAEval/graph_construction``)."""
