"""RQ2 harness on the MI355X engine — ``rq2.py:150-452`` restated; cases sharded over GPUs.

The reference runs every case of a dataset through one RCA method in a sequential loop
(``rq2.py:301-302``), writing ``{service}_{metric}_{case}.json`` = ``{0: ranks}``
(``:173-296``), then scores the result files per (service, fault) and per fault type with
``Evaluator`` (``:309-450``). ``load_case`` / ``process`` / ``evaluate`` below follow those
lines statement for statement (window cut, inf/NaN handling, SLI choice, ``n_iter=num_node``).

Batching (BASELINE config 2): the sorted case list is dealt round-robin to the
ranks of ``torchrun`` — one process per GPU, each rank's engine on its own device. Cases are
independent, so the data path has no collective; rank 0 waits on one barrier and scores
every result file.

    python -m rcaeval_amd.rq2 --method pc_pagerank --dataset online-boutique --data-root DIR
    python -m torch.distributed.run --nproc-per-node 8 -m rcaeval_amd.rq2 ...
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import time
from os.path import basename, dirname, exists, join

import numpy as np
import pandas as pd

from . import phases
from .benchmark.evaluation import Evaluator
from .classes.graph import Node

DATASET_MAP = {                                   # rq2.py:135-144
    "circa10": "data/rca_circa/10",
    "circa50": "data/rca_circa/50",
    "rcd10": "data/rca_rcd/10",
    "rcd50": "data/rca_rcd/50",
    "online-boutique": "data/online-boutique",
    "sock-shop-1": "data/sock-shop-1",
    "sock-shop-2": "data/sock-shop-2",
    "train-ticket": "data/train-ticket",
}


def methods():
    """Methods this engine serves (``rq2.py:36-59`` resolves them by name)."""
    from .e2e import circa, cloudranger, pc_pagerank, pc_randomwalk
    return {"pc_pagerank": pc_pagerank, "pc_randomwalk": pc_randomwalk, "cloudranger": cloudranger,
            "circa": circa}


def dump_json(filename: str, data) -> None:
    """``RCAEval/utility/__init__.py:20-25``."""
    with open(filename, "w", encoding="utf-8") as obj:
        json.dump(data, obj, ensure_ascii=False, indent=2, sort_keys=True)


def load_json(filename: str):
    with open(filename, encoding="utf-8") as obj:
        return json.load(obj)


def list_cases(dataset_dir: str, test: bool = False) -> list:
    """``rq2.py:150-159``: every ``data.csv`` (``simple_data.csv`` when present), sorted as
    the loop at ``:301`` visits them. (The reference truncates ``--test`` runs to two paths
    in glob order before sorting; here the two are taken after sorting, deterministically.)"""
    paths = list(glob.glob(os.path.join(dataset_dir, "**/data.csv"), recursive=True))
    out = []
    for p in paths:
        simple = p.replace("data.csv", "simple_data.csv")
        out.append(simple if os.path.exists(simple) else p)
    out = sorted(out)
    return out[:2] if test else out


def _first_line(path: str) -> str:
    with open(path) as f:
        return f.readlines()[0].strip()


def load_case(data_path: str, length=None, tdelta: int = 0, is_synthetic: bool = False) -> dict:
    """``rq2.py:178-270``: the windowed case frame and everything ``process`` passes on."""
    if length is None:
        length = 10 if not is_synthetic else 2000
    data_length = length * 60 // 2
    data_dir = dirname(data_path)
    sli = None
    inject_time = None
    if "rca_" in data_path:                                            # :185-201
        case = basename(dirname(data_path))
        service = "SIM"
        with open(join(data_dir, "root_cause.txt")) as f:
            metric = f.read().splitlines()[0]
        inject_time = int(_first_line(join(data_dir, "inject_time.txt"))) + tdelta
        sli = "SIM_" + _first_line(join(data_dir, "fe_service.txt"))
    else:                                                              # :203-206
        service, metric = basename(dirname(dirname(data_path))).split("_")
        case = basename(dirname(data_path))
    rp_name = f"{service}_{metric}_{case}.json"                        # :208

    t_read = time.perf_counter()
    data = pd.read_csv(data_path)                                      # :211-235
    t_read = time.perf_counter() - t_read
    t_win = time.perf_counter()
    if "time.1" in data:
        data = data.drop(columns=["time.1"])
    if "rca_" in data_path:
        data.columns = ["SIM_" + c for c in data.columns]
    if "time" not in data:
        data["time"] = data.index
    if "sock-shop" in data_path:
        data = data.loc[:, ~data.columns.str.endswith("_lat_50")]
        data = data.loc[:, ~data.columns.str.endswith("_lat_99")]
    if "train-ticket" in data_path:
        time_col = data["time"]
        data = data.loc[:, data.columns.str.startswith("ts-")]
        data["time"] = time_col
    data = data.replace([np.inf, -np.inf], np.nan)
    data = data.ffill()                                                # fillna(method="ffill")
    data = data.fillna(0)

    if "rca_" in data_dir:                                             # :237-249
        normal_df = data[data["time"] < inject_time].tail(data_length)
        anomal_df = data[data["time"] >= inject_time].head(data_length)
    else:
        inject_time = int(_first_line(join(data_dir, "inject_time.txt"))) + tdelta
        normal_df = data[data["time"] < inject_time].tail(data_length)
        anomal_df = data[data["time"] >= inject_time].head(data_length)
    data = pd.concat([normal_df, anomal_df], ignore_index=True)

    num_node = len(data.columns) - 1                                   # :252
    if "my-sock-shop" in data_path:                                    # :255-270
        sli = "front-end_cpu"
        if f"{service}_latency" in data:
            sli = f"{service}_latency"
    elif "sock-shop" in data_path:
        sli = "front-end_cpu"
        if f"{service}_lat_90" in data:
            sli = f"{service}_lat_90"
    elif "train-ticket" in data_path:
        sli = "ts-ui-dashboard_latency-90"
        if f"{service}_latency" in data:
            sli = f"{service}_latency"
    elif "online-boutique" in data_path:
        sli = "frontend_latency-90"
        if f"{service}_latency" in data:
            sli = f"{service}_latency"
    # load timings travel with the case: a prefetching loader thread does not share the
    # caller's phase accounting (rcaeval_amd.phases is per thread)
    return {"data": data, "inject_time": inject_time, "service": service, "metric": metric, "case": case,
            "sli": sli, "num_node": num_node, "result_name": rp_name,
            "load_s": {"read_csv": t_read, "window": time.perf_counter() - t_win}}


def process(data_path: str, method: str, dataset: str, result_path: str, length=None, tdelta: int = 0,
            is_synthetic: bool = False) -> dict:
    """``rq2.py:173-296`` for one case: run the method, dump ``{0: ranks}``."""
    c = load_case(data_path, length=length, tdelta=tdelta, is_synthetic=is_synthetic)
    return process_loaded(c, method, dataset, result_path)


def process_loaded(c: dict, method: str, dataset: str, result_path: str) -> dict:
    """The method and the JSON dump of a case ``load_case`` returned (``rq2.py:272-289``)."""
    for k, v in c.get("load_s", {}).items():
        phases.add(k, v)
    func = methods()[method]
    t0 = time.perf_counter()
    out = func(c["data"], c["inject_time"], dataset=dataset, anomalies=None, dk_select_useful=False,
               sli=c["sli"], verbose=False, n_iter=c["num_node"], args=None)
    seconds = time.perf_counter() - t0
    phases.add("method (total)", seconds)
    ranks = out.get("ranks")
    rp = join(result_path, c["result_name"])
    with phases.phase("json"):
        dump_json(filename=rp, data={0: ranks})
    return {"path": rp, "ranks": ranks, "seconds": seconds}


def _dedup(nodes):
    """``rq2.py:356-366``: keep the first occurrence of each service node."""
    if not nodes:
        return []
    return [nodes[0]] + [nodes[i] for i in range(1, len(nodes)) if nodes[i] not in nodes[:i]]


def evaluate(result_path: str, is_synthetic: bool = False) -> dict:
    """``rq2.py:309-450``: per (service, fault) AC@1/3/5 and Avg@5, service- and
    metric-level, plus Avg@5 per fault type (or overall for synthetic datasets)."""
    rps = glob.glob(join(result_path, "*.json"))
    services = sorted(list(set([basename(x).split("_")[0] for x in rps])))
    faults = sorted(list(set([basename(x).split("_")[1] for x in rps])))
    keys = ["service-fault", "top_1_service", "top_3_service", "top_5_service", "avg@5_service",
            "top_1_metric", "top_3_metric", "top_5_metric", "avg@5_metric"]
    eval_data = {k: [] for k in keys}
    groups = {name: (Evaluator(), Evaluator()) for name in ("all", "cpu", "mem", "lat", "loss", "io")}
    fault_group = {"cpu": ("cpu", None), "mem": ("mem", None), "delay": ("lat", "latency"),
                   "loss": ("loss", "latency"), "disk": ("io", "latency")}

    def add_row(label, s_ev, f_ev):
        eval_data["service-fault"].append(label)
        eval_data["top_1_service"].append(s_ev.accuracy(1))
        eval_data["top_3_service"].append(s_ev.accuracy(3))
        eval_data["top_5_service"].append(s_ev.accuracy(5))
        eval_data["avg@5_service"].append(s_ev.average(5))
        eval_data["top_1_metric"].append(f_ev.accuracy(1))
        eval_data["top_3_metric"].append(f_ev.accuracy(3))
        eval_data["top_5_metric"].append(f_ev.accuracy(5))
        eval_data["avg@5_metric"].append(f_ev.average(5))

    for service in services:
        for fault in faults:
            s_evaluator, f_evaluator = Evaluator(), Evaluator()
            for rp in rps:
                s, m = basename(rp).split("_")[:2]
                if s != service or m != fault:
                    continue
                data = load_json(rp)
                if "error" in data:
                    continue
                for _, ranks in data.items():
                    s_ranks = _dedup([Node(x.split("_")[0].replace("-db", ""), "unknown") for x in ranks])
                    f_ranks = [Node(x.split("_")[0], x.split("_")[1]) for x in ranks]
                    s_answer = Node(service, "unknown")
                    s_evaluator.add_case(ranks=s_ranks, answer=s_answer)
                    f_evaluator.add_case(ranks=f_ranks, answer=Node(service, fault))
                    if fault in fault_group:
                        grp, metric_name = fault_group[fault]
                        f_answer = Node(service, metric_name or fault)
                        groups[grp][0].add_case(ranks=s_ranks, answer=s_answer)
                        groups[grp][1].add_case(ranks=f_ranks, answer=f_answer)
                        groups["all"][0].add_case(ranks=s_ranks, answer=s_answer)
                        groups["all"][1].add_case(ranks=f_ranks, answer=f_answer)
                    if is_synthetic:
                        groups["all"][0].add_case(ranks=s_ranks, answer=s_answer)
                        groups["all"][1].add_case(ranks=f_ranks, answer=Node(service, fault))
            add_row(f"{service}_{fault}", s_evaluator, f_evaluator)

    summary = {}
    if is_synthetic:
        avg = groups["all"][1].average(5)
        summary["Avg@5"] = round(avg, 2) if avg is not None else None
    else:
        for name, grp in (("cpu", "cpu"), ("mem", "mem"), ("io", "io"), ("delay", "lat"), ("loss", "loss")):
            s_ev, f_ev = groups[grp]
            add_row(f"overall_{name}", s_ev, f_ev)
            label = "disk" if name == "io" else name
            if s_ev.average(5) is not None:
                summary[f"Avg@5-{label.upper()}"] = round(s_ev.average(5), 2)
    return {"eval_data": eval_data, "summary": summary}


_LOADERS = None


def _loader_ready(_):
    return os.getpid()


def start_loaders(n: int):
    """A pool of ``n`` loader PROCESSES (spawned: fresh interpreters that import pandas and this
    module, never the GPU) reading and windowing cases for ``run``; kept for later runs. pandas'
    CSV parser holds the GIL, so loader threads contend with the GPU thread (measured: 3.5 ms of
    read_csv per case alone, ~10 ms per case on two threads); processes do not."""
    global _LOADERS
    if n <= 0:
        return None
    if _LOADERS is not None and _LOADERS[1] == n:
        return _LOADERS[0]
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    stop_loaders()
    pool = ProcessPoolExecutor(max_workers=n, mp_context=multiprocessing.get_context("spawn"))
    list(pool.map(_loader_ready, range(n)))          # every worker up (imports done)
    _LOADERS = (pool, n)
    return pool


def stop_loaders() -> None:
    global _LOADERS
    if _LOADERS is not None:
        _LOADERS[0].shutdown(wait=True)
        _LOADERS = None


def run(dataset_dir: str, method: str, dataset: str, output: str = "output", length=None, tdelta: int = 0,
        test: bool = False, rank: int = 0, world: int = 1, prefetch: int = 2, loader: str = "thread") -> dict:
    """Every case of ``dataset_dir`` through ``method``; rank ``r`` of ``world`` takes cases
    ``r, r + world, ...`` of the sorted list. Returns this rank's timings and, on rank 0,
    the evaluation (after a barrier when ``world > 1``). ``prefetch`` loaders read the next
    cases ahead of the GPU thread: threads by default (safe from any caller); ``loader="process"``
    uses spawned processes (faster — pandas' parser holds the GIL — but the caller's script needs
    an ``if __name__ == "__main__"`` guard; ``main`` and ``bench.py`` opt in, and ``main`` stops them
    at its end)."""
    is_synthetic = "circa" in dataset or "rcd" in dataset
    result_path = join(output, "results")
    os.makedirs(result_path, exist_ok=True)
    paths = list_cases(dataset_dir, test=test)
    mine = paths[rank::world]
    t0 = time.perf_counter()
    per_case = []
    if prefetch > 0 and len(mine) > 1:
        # loaders (threads by default, or spawned processes) read and window the next cases while this
        # thread runs the current case on the GPU; cases are still processed, and their errors
        # raised, in the sorted order of the sequential loop
        from collections import deque
        from concurrent.futures import ThreadPoolExecutor
        kw = dict(length=length, tdelta=tdelta, is_synthetic=is_synthetic)
        own = None
        if loader == "process":
            ex = start_loaders(prefetch)
        else:
            ex = own = ThreadPoolExecutor(max_workers=prefetch)
        depth = 2 * prefetch                       # cases in flight ahead of the GPU thread
        try:
            queue = deque((p, ex.submit(load_case, p, **kw)) for p in mine[:depth])
            nxt = len(queue)
            while queue:
                _, fut = queue.popleft()
                c = fut.result()
                if nxt < len(mine):
                    queue.append((mine[nxt], ex.submit(load_case, mine[nxt], **kw)))
                    nxt += 1
                per_case.append(process_loaded(c, method, dataset, result_path))
        finally:
            for _, f in (queue if "queue" in locals() else ()):
                f.cancel()
            if own is not None:
                own.shutdown(wait=True)
    else:
        for p in mine:
            per_case.append(process(p, method, dataset, result_path, length=length, tdelta=tdelta,
                                    is_synthetic=is_synthetic))
    wall = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
    out = {"cases": len(paths), "my_cases": len(mine), "wall_s": wall,
           "method_s": [c["seconds"] for c in per_case]}
    if phases.enabled():
        out["phases"] = phases.take()
    if rank == 0:
        out.update(evaluate(result_path, is_synthetic=is_synthetic))
        out["avg_speed"] = round(wall / max(len(mine), 1), 4)                # rq2.py:303-306
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="RCAEval RQ2 on the MI355X engine")
    ap.add_argument("--method", type=str, required=True)
    ap.add_argument("--dataset", type=str, required=True, choices=sorted(DATASET_MAP))
    ap.add_argument("--data-root", type=str, default=".", help="directory holding data/<dataset> (no downloads)")
    ap.add_argument("--output", type=str, default="output")
    ap.add_argument("--length", type=int, default=None)
    ap.add_argument("--tdelta", type=int, default=0)
    ap.add_argument("--test", action="store_true")
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("gloo")          # one barrier; cases need no device collective
    dataset_dir = join(args.data_root, DATASET_MAP[args.dataset])
    if not exists(dataset_dir):
        raise SystemExit(f"{dataset_dir} not found (datasets are not downloaded here)")
    try:
        res = run(dataset_dir, args.method, args.dataset, args.output, args.length, args.tdelta, args.test,
                  rank, world, loader="process")
    finally:
        stop_loaders()
    if rank == 0:
        print("--- Evaluation results ---")
        for k, v in res["summary"].items():
            print(f"{k}:".ljust(12), v)
        print("---")
        print("Avg speed:", res["avg_speed"])
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
