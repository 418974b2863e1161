"""CPU: the glue around the engine against outputs of the REFERENCE functions themselves
(tests/golden/glue.json, made by tests/golden/make_glue_golden.py under python3.9 + networkx
2.6.3 with the reference pc_pagerank / pc_randomwalk / rq2 process executed):

* the rq2 window (rq2.py:211-249), SLI choice (:255-270), n_iter (:252) and result-file name
  (:208) of rcaeval_amd.rq2.load_case on the same seeded case trees;
* pc_pagerank's graph -> matrix -> PageRank -> zip glue (pc_pagerank.py:20-35) of
  rcaeval_amd.e2e.pc_pagerank.digraph_matrix, with the sknetwork restatement as PageRank.
The GPU halves (engine graph + GPU PageRank / random walk) are in tests/test_gpu_e2e.py.
"""
import json
import os
import sys

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)


def _glue():
    return json.load(open(os.path.join(GOLD, "glue.json")))


def test_rq2_window_matches_reference_process(tmp_path):
    from make_glue_golden import frame_digest, write_trees
    from rcaeval_amd import rq2
    write_trees(str(tmp_path))
    cases = _glue()["rq2"]
    assert len(cases) == 17
    for c in cases:
        p = os.path.join(str(tmp_path), c["rel"])
        got = rq2.load_case(p, is_synthetic=c["dataset"] == "synthetic")
        w = got["data"]
        assert frame_digest(w) == c["window_digest"], c["rel"]
        assert w.shape[0] == c["rows"] and list(w.columns) == c["columns"]
        assert got["inject_time"] == c["inject_time"], c["rel"]
        assert got["num_node"] == c["n_iter"] and got["sli"] == c["sli"], c["rel"]
        assert got["result_name"] == c["result_file"], c["rel"]


@pytest.mark.parametrize("k", range(6))
def test_pc_pagerank_glue_matches_reference(k):
    from oracle import pagerank as opr
    from rcaeval_amd.e2e.pc_pagerank import digraph_matrix
    case = _glue()["pagerank"][k]
    g = np.array(case["graph"])
    M, nodes = digraph_matrix(g)
    np.testing.assert_array_equal(M, np.array(case["adj"]))
    scores = opr.pagerank(M.T)
    ranked = sorted(zip(case["node_names"], scores), key=lambda t: t[1], reverse=True)
    assert [n for n, _ in ranked] == case["ranks"]


def test_golden_covers_the_misaligned_zip():
    """At least one case drops isolated nodes, so names and scores misalign (pc_pagerank.py:33)."""
    assert any(len(c["ranks"]) < len(c["node_names"]) for c in _glue()["pagerank"])
