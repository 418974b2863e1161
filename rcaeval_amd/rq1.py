"""RQ1 harness (causal-graph quality) on the MI355X engine — restates ``rq1.py:122-298``.

For every ``data.csv`` under the dataset tree the reference runs ``pc(np_data, stable=False,
show_progress=False).G.graph`` on ``|ffill(data).fillna(0)|`` (``rq1.py:216-239``), wraps the
endpoint matrix with ``MemoryGraph.from_adj`` (``Node("SIM", i)`` names for CIRCA data,
``rq1.py:270-275``) and dumps ``<graph>_<case>_est_graph.json``; ``evaluate`` then scores every
estimate against the tree's true graph with F1, F1_Skeleton and SHD (``rq1.py:128-199``).

Only ``--method pc`` runs on the engine (order-dependent PC, ``rcaeval_amd.skeleton_seq``,
default ``uc_priority=2``); the other graph learners of ``AVAILABLE_METHODS`` are out of scope
 and raise ``NotImplementedError``. CAUSIL's pickled ground truth is never unpickled:
CIRCA (``graph.json``) and RCD (``true_graph.json``) trees are supported.
"""
from __future__ import annotations

import glob
import math
import os
from os.path import basename, dirname, exists, join

import numpy as np
import pandas as pd

from .benchmark.metrics import F1, SHD, F1_Skeleton
from .causal import pc
from .classes.graph import MemoryGraph, Node

DATASET_MAP = {
    "circa10": "data/syn_circa/10", "circa50": "data/syn_circa/50",
    "causil10": "data/syn_causil/10", "causil50": "data/syn_causil/50",
    "rcd10": "data/syn_rcd/10", "rcd50": "data/syn_rcd/50",
}


def _indices(data_path: str):
    """``rq1.py:140-149,201-214``: (num_node, graph_idx, case_idx) from the tree layout."""
    if "causil" in data_path:
        raise NotImplementedError("CAUSIL trees keep their ground truth as a pickle (DAG.gpickle), which is not loaded")
    num_node = int(basename(dirname(dirname(dirname(dirname(data_path))))))
    graph_idx = int(basename(dirname(dirname(dirname(data_path)))))
    case_idx = int(basename(dirname(data_path)))
    return num_node, graph_idx, case_idx


def load_data(data_path: str, length=None):
    """``rq1.py:216-228``: CIRCA csvs have no header row; ffill, then 0, then |x|."""
    if "circa" in data_path:
        data = pd.read_csv(data_path, header=None)
    else:
        data = pd.read_csv(data_path)
    data = data.ffill().fillna(value=0)
    np_data = np.absolute(data.to_numpy().astype(float))
    if length is not None:
        np_data = np_data[:length, :]
    return data, np_data


def process(data_path: str, result_path: str, method: str = "pc", length=None) -> MemoryGraph:
    """``rq1.py:200-285`` for one case; returns the estimated graph (also dumped)."""
    _, graph_idx, case_idx = _indices(data_path)
    data, np_data = load_data(data_path, length)
    if method != "pc":
        raise NotImplementedError(f"method={method!r}: only 'pc' runs on the MI355X engine")
    adj = pc(np_data, stable=False, show_progress=False).G.graph
    if "circa" in data_path:
        est = MemoryGraph.from_adj(adj, nodes=[Node("SIM", str(i)) for i in range(len(adj))])
    else:
        est = MemoryGraph.from_adj(adj, nodes=data.columns.to_list())
    est.dump(join(result_path, f"{graph_idx}_{case_idx}_est_graph.json"))
    return est


def true_graph(data_path: str) -> MemoryGraph:
    """``rq1.py:158-173``."""
    root = dirname(dirname(dirname(data_path)))
    if "circa" in data_path:
        return MemoryGraph.load(join(root, "graph.json"))
    if "rcd" in data_path:
        return MemoryGraph.load(join(root, "true_graph.json"))
    raise NotImplementedError(f"no ground-truth rule for {data_path!r}")


def evaluate(data_paths, result_path: str) -> dict:
    """``rq1.py:128-199``: per-case scores and the printed averages (SHD floored)."""
    rows = {k: [] for k in ("Case", "Precision", "Recall", "F1-Score", "Precision-Skel",
                            "Recall-Skel", "F1-Skel", "SHD")}
    for data_path in data_paths:
        _, graph_idx, case_idx = _indices(data_path)
        name = f"{graph_idx}_{case_idx}_est_graph.json"
        path = join(result_path, name)
        if not exists(path):
            continue
        est = MemoryGraph.load(path)
        tg = true_graph(data_path)
        e, es = F1(tg, est), F1_Skeleton(tg, est)
        rows["Case"].append(name)
        rows["Precision"].append(e["precision"])
        rows["Recall"].append(e["recall"])
        rows["F1-Score"].append(e["f1"])
        rows["Precision-Skel"].append(es["precision"])
        rows["Recall-Skel"].append(es["recall"])
        rows["F1-Skel"].append(es["f1"])
        rows["SHD"].append(SHD(tg, est))
    summary = {"F1": float(np.mean(rows["F1-Score"])), "F1-S": float(np.mean(rows["F1-Skel"])),
               "SHD": math.floor(np.mean(rows["SHD"])) if rows["SHD"] else None}
    return {"cases": rows, "summary": summary}


def run(dataset_dir: str, result_path: str, method: str = "pc", length=None, test: bool = False) -> dict:
    """``rq1.py:122-125,288-298`` + ``evaluate``: every ``**/data.csv`` under ``dataset_dir``."""
    os.makedirs(result_path, exist_ok=True)
    data_paths = list(glob.glob(os.path.join(dataset_dir, "**/data.csv"), recursive=True))
    if test:
        data_paths = data_paths[:2]
    for p in data_paths:
        process(p, result_path, method=method, length=length)
    return evaluate(data_paths, result_path)


__all__ = ["DATASET_MAP", "load_data", "process", "true_graph", "evaluate", "run"]
