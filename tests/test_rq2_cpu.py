"""CPU: the RQ2 harness (rcaeval_amd.rq2) and scorer (Evaluator) — SURVEY §8(f) rank 1.

The scorer is pinned by tests/golden/evaluator.json, produced by the REFERENCE
``RCAEval.benchmark.evaluation.Evaluator`` (tests/golden/make_golden.py); the case loader
and the per-fault evaluation follow rq2.py:173-450 and are checked on synthetic case trees.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

from rcaeval_amd import rq2, synth
from rcaeval_amd.benchmark.evaluation import Evaluator
from rcaeval_amd.classes.graph import Node

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_evaluator_matches_reference_golden():
    g = json.load(open(os.path.join(GOLD, "evaluator.json")))
    s_ev, f_ev = Evaluator(), Evaluator()
    for c in g["cases"]:
        f_ev.add_case([Node(*x.split("_")[:2]) for x in c["ranks"]], Node(*c["answer"]))
        s_ev.add_case([Node(x.split("_")[0], "unknown") for x in c["ranks"]], Node(c["answer"][0], "unknown"))
    for k in range(0, 7):
        assert [f_ev.accuracy(k), f_ev.accuracy_service(k), f_ev.average(k), f_ev.average_service(k)] == g["metric"][str(k)]
        assert [s_ev.accuracy(k), s_ev.accuracy_service(k), s_ev.average(k), s_ev.average_service(k)] == g["service"][str(k)]
    assert [Evaluator().accuracy(1), Evaluator().average(5)] == g["empty"]


def _tree(tmp_path, **kw):
    root = os.path.join(str(tmp_path), "data", "online-boutique")
    return root, synth.write_rq2_dataset(root, **kw)


def test_load_case_window_sli_and_cleaning(tmp_path):
    root, paths = _tree(tmp_path, services=["cartservice"], faults=("cpu",), cases=1, rows=1000)
    p = paths[0]
    df = pd.read_csv(p)
    df.loc[10, "cartservice_cpu"] = np.inf                       # inf -> NaN -> ffill
    df.loc[0, "adservice_mem"] = np.nan                          # leading NaN -> fillna(0)
    df["time.1"] = df["time"]
    df.to_csv(p, index=False)
    c = rq2.load_case(p)
    inject = int(open(os.path.join(os.path.dirname(p), "inject_time.txt")).read())
    assert c["inject_time"] == inject and c["service"] == "cartservice" and c["metric"] == "cpu"
    d = c["data"]
    assert "time.1" not in d and len(d) == 600                     # 10 min -> 300 + 300 rows
    assert (d["time"] < inject).sum() == 300 and (d["time"] >= inject).sum() == 300
    assert c["num_node"] == len(d.columns) - 1
    assert c["sli"] == "frontend_latency-90"                       # rq2.py:267-270
    assert not np.isinf(d.to_numpy()).any() and not d.isna().any().any()
    row10 = df.index.get_loc(10)
    assert c["result_name"] == "cartservice_cpu_1.json"
    assert row10 == 10


def test_list_cases_sorted_and_prefers_simple_data(tmp_path):
    root, paths = _tree(tmp_path, services=["adservice", "cartservice"], faults=("cpu", "mem"), cases=1, rows=200)
    simple = paths[1].replace("data.csv", "simple_data.csv")
    pd.read_csv(paths[1]).to_csv(simple, index=False)
    got = rq2.list_cases(root)
    assert got == sorted(got) and simple in got and paths[1] not in got and len(got) == 4
    assert rq2.list_cases(root, test=True) == got[:2]


def test_evaluate_hand_example(tmp_path):
    res = os.path.join(str(tmp_path), "results")
    os.makedirs(res)
    cases = {
        "cartservice_cpu_1.json": ["cartservice_cpu", "adservice_mem", "frontend_latency-90"],
        "cartservice_cpu_2.json": ["adservice_cpu", "cartservice_mem", "cartservice_cpu"],
        "adservice_delay_1.json": ["adservice_latency", "adservice-db_cpu", "cartservice_cpu"],
    }
    for name, ranks in cases.items():
        rq2.dump_json(os.path.join(res, name), {0: ranks})
    out = rq2.evaluate(res)
    ed = out["eval_data"]
    rows = dict(zip(ed["service-fault"], range(len(ed["service-fault"]))))
    r = rows["cartservice_cpu"]
    assert ed["top_1_metric"][r] == 0.5 and ed["top_3_metric"][r] == 1.0
    assert ed["top_1_service"][r] == 0.5 and ed["top_3_service"][r] == 1.0     # svc dedup: adservice, cartservice
    r = rows["adservice_delay"]
    assert ed["top_1_service"][r] == 1.0 and ed["top_1_metric"][r] == 0.0      # answer Node(svc, "delay")
    assert rows["adservice_cpu"] is not None and ed["top_1_service"][rows["adservice_cpu"]] is None
    # per-fault-type summary: delay scored against Node(service, "latency")
    assert out["summary"]["Avg@5-CPU"] == round((0.5 + 1 + 1 + 1 + 1) / 5, 2)
    assert out["summary"]["Avg@5-DELAY"] == 1.0
    assert "Avg@5-MEM" not in out["summary"]


def test_run_deals_cases_round_robin(tmp_path, monkeypatch):
    """rank r of world w takes cases r, r+w, ... of the sorted list (no GPU: a stub method)."""
    root, paths = _tree(tmp_path, services=["adservice", "cartservice"], faults=("cpu",), cases=2, rows=200)
    seen = []

    def stub(data, inject_time, **kw):
        seen.append(kw["n_iter"])
        return {"ranks": list(data.columns[1:][::-1])}
    monkeypatch.setattr(rq2, "methods", lambda: {"stub": stub})
    out_dir = os.path.join(str(tmp_path), "out")
    mine = [rq2.run(root, "stub", "online-boutique", out_dir, rank=r, world=3)["my_cases"] for r in range(3)]
    assert mine == [2, 1, 1] and len(seen) == 4
    res = rq2.evaluate(os.path.join(out_dir, "results"))
    assert sorted(res["eval_data"]["service-fault"])[:2] == ["adservice_cpu", "cartservice_cpu"]


def test_run_prefetch_gives_the_sequential_results_in_order(tmp_path, monkeypatch):
    """Loader threads (prefetch > 0) read and window later cases while the current one runs: the
    cases reach the method in the sorted order, with the same frames, and the result files are
    identical to the sequential loop's; a load error surfaces at its own case, after every earlier
    case was processed (like the reference's loop)."""
    import json
    import pandas as pd
    from rcaeval_amd import phases
    root, paths = _tree(tmp_path, services=["adservice", "cartservice", "emailservice"], faults=("cpu", "mem"),
                        cases=2, rows=200)
    runs = {}
    for pf in (0, 1, 3):
        seen = []

        def stub(data, inject_time, **kw):
            seen.append((inject_time, data.shape, float(data.to_numpy().sum())))
            return {"ranks": list(data.columns[1:][::-1])}
        monkeypatch.setattr(rq2, "methods", lambda: {"stub": stub})
        out_dir = os.path.join(str(tmp_path), f"out{pf}")
        phases.enable()
        res = rq2.run(root, "stub", "online-boutique", out_dir, prefetch=pf)
        phases.enable(False)
        assert {"read_csv", "window", "method (total)", "json"} <= set(res["phases"])
        files = sorted(os.listdir(os.path.join(out_dir, "results")))
        runs[pf] = (seen, files, [json.load(open(os.path.join(out_dir, "results", f))) for f in files])
    assert runs[0] == runs[1] == runs[3]
    assert len(runs[0][0]) == len(paths)
    # a broken case in the middle: earlier cases done, the error raised at its turn
    bad = sorted(paths)[3]
    with open(bad, "w") as f:
        f.write("")
    seen = []

    def stub2(data, inject_time, **kw):
        seen.append(1)
        return {"ranks": []}
    monkeypatch.setattr(rq2, "methods", lambda: {"stub": stub2})
    with pytest.raises(pd.errors.EmptyDataError):
        rq2.run(root, "stub", "online-boutique", os.path.join(str(tmp_path), "outbad"), prefetch=2)
    assert len(seen) == 3
