"""GPU: the RQ1 harness (rcaeval_amd.rq1, ``rq1.py --method pc``) end to end on the engine —
order-dependent PC on CIRCA-shaped trees, dumped est graphs and F1 / F1-S / SHD — equal to the
CPU restatement's pipeline case by case."""
import os

import numpy as np
import pytest

from test_metrics_cpu import _oracle_est

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("num_node,rows,ep", [(10, 600, 0.3), (20, 800, 0.15)])
def test_rq1_pc_matches_oracle_pipeline(tmp_path, num_node, rows, ep):
    from rcaeval_amd import rq1, synth
    from rcaeval_amd.benchmark.metrics import F1, SHD, F1_Skeleton
    root = str(tmp_path / "syn_circa")
    paths = synth.write_rq1_dataset(root, num_node=num_node, graphs=2, cases=2, rows=rows, seed=num_node,
                                    edge_prob=ep)
    res = str(tmp_path / "results")
    out = rq1.run(root, res)
    assert len(out["cases"]["Case"]) == len(paths)
    for p in paths:
        _, gi, ci = rq1._indices(p)
        got = rq1.MemoryGraph.load(os.path.join(res, f"{gi}_{ci}_est_graph.json"))
        want = _oracle_est(p)
        assert sorted(got.str_edges) == sorted(want.str_edges), p
        tg = rq1.true_graph(p)
        k = out["cases"]["Case"].index(f"{gi}_{ci}_est_graph.json")
        assert out["cases"]["F1-Score"][k] == F1(tg, want)["f1"]
        assert out["cases"]["F1-Skel"][k] == F1_Skeleton(tg, want)["f1"]
        assert out["cases"]["SHD"][k] == SHD(tg, want)
    assert np.isfinite(out["summary"]["F1"])
