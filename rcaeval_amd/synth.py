"""Synthetic inputs of the shapes BASELINE.json names (no datasets travel offline).

``gaussian_sem`` is the SURVEY §8(d) config-5 generator: a linear Gaussian SEM over an
Erdős–Rényi DAG on a random topological order, edge probability ``2/(n-1)`` (≈n true
edges), weights ±U(w_low, w_high), N(0,1) noise, ``numpy.random.default_rng(seed)``.

``telemetry_frame`` builds a DataFrame shaped like an RCAEval RQ2 case (a ``time`` column
plus ``<service>_<metric>`` columns, ≤600 rows, a few constant columns) for the
``pc_pagerank`` / ``pc_randomwalk`` drop-in paths (configs 1–4).
"""
from __future__ import annotations

import numpy as np


def sem_dag(n: int, edge_prob: float | None = None, w_low: float = 0.1, w_high: float = 0.5,
            seed: int = 0):
    """Return (W, order): W[i, j] != 0 <=> edge i -> j, order = topological order."""
    rng = np.random.default_rng(seed)
    if edge_prob is None:
        edge_prob = 2.0 / max(n - 1, 1)
    order = rng.permutation(n)
    pos_mask = np.triu(rng.random((n, n)) < edge_prob, k=1)        # position-space DAG
    weights = rng.uniform(w_low, w_high, (n, n)) * rng.choice([-1.0, 1.0], (n, n))
    Wp = np.where(pos_mask, weights, 0.0)
    W = np.zeros((n, n))
    W[np.ix_(order, order)] = Wp
    return W, order, rng


def gaussian_sem(n_vars: int = 2000, n_samples: int = 10000, edge_prob: float | None = None,
                 w_low: float = 0.1, w_high: float = 0.5, seed: int = 0) -> np.ndarray:
    """N x n float64 C-order samples of X = X W + E, E ~ N(0, 1)."""
    W, order, rng = sem_dag(n_vars, edge_prob, w_low, w_high, seed)
    E = rng.standard_normal((n_samples, n_vars))
    X = np.zeros((n_samples, n_vars))
    # X_j = sum_i W[i, j] X_i + E_j in topological order (sparse parents).
    for j in order:
        parents = np.nonzero(W[:, j])[0]
        col = E[:, j].copy()
        if parents.size:
            col += X[:, parents] @ W[parents, j]
        X[:, j] = col
    return np.ascontiguousarray(X)


def discrete_sem(n_vars: int = 50, n_samples: int = 2000, levels: int = 6, seed: int = 0) -> np.ndarray:
    """rcd50-shaped discrete data (values 0..levels-1) from a thresholded Gaussian SEM."""
    X = gaussian_sem(n_vars, n_samples, w_low=0.5, w_high=1.0, seed=seed)
    qs = np.quantile(X, np.linspace(0, 1, levels + 1)[1:-1], axis=0)
    out = np.zeros_like(X)
    for j in range(n_vars):
        out[:, j] = np.searchsorted(qs[:, j], X[:, j])
    return out


def telemetry_frame(n_metrics: int = 49, n_rows: int = 600, n_constant: int = 2, seed: int = 0,
                    services=None):
    """RCAEval-case-shaped DataFrame: ``time`` + ``<svc>_{cpu,mem,latency}`` columns."""
    import pandas as pd

    rng = np.random.default_rng(seed)
    X = gaussian_sem(n_metrics, n_rows, w_low=0.3, w_high=0.9, seed=seed)
    kinds = ["cpu", "mem", "latency"]
    services = services or [f"svc{i}" for i in range((n_metrics + 2) // 3)]
    cols = []
    for i in range(n_metrics):
        cols.append(f"{services[i // 3]}_{kinds[i % 3]}")
    X = X * rng.uniform(0.5, 5.0, n_metrics) + rng.uniform(0, 100, n_metrics)
    for j, c in enumerate(cols):
        if c.endswith("_mem"):
            X[:, j] = np.abs(X[:, j]) * 1e7
    const_idx = rng.choice(n_metrics, size=min(n_constant, n_metrics), replace=False)
    for j in const_idx:
        X[:, j] = float(j)
    df = pd.DataFrame(X, columns=cols)
    df.insert(0, "time", np.arange(1692569000, 1692569000 + n_rows))
    return df


OB_SERVICES = ["adservice", "cartservice", "checkoutservice", "currencyservice", "emailservice", "frontend",
               "paymentservice", "productcatalogservice", "recommendationservice", "shippingservice", "redis"]
OB_METRICS = ["cpu", "mem", "latency-50", "latency-90"]
FAULT_METRIC = {"cpu": "cpu", "mem": "mem", "delay": "latency-90", "loss": "latency-90", "disk": "mem"}
# Sock Shop: <svc>_{cpu,mem,lat_50,lat_90,lat_99}; rq2.py:228-230 drops lat_50 / lat_99 columns
# and takes <svc>_lat_90 (else front-end_cpu) as the SLI (:259-262)
SS_SERVICES = ["carts", "catalogue", "front-end", "orders", "payment", "shipping", "user", "carts-db",
               "orders-db", "user-db"]
SS_METRICS = ["cpu", "mem", "lat_50", "lat_90", "lat_99"]
SS_FAULT_METRIC = {"cpu": "cpu", "mem": "mem", "delay": "lat_90", "loss": "lat_90", "disk": "mem"}


def rq2_case_frame(services=None, metrics=None, rows: int = 1200, root_service: str = "cartservice",
                   fault: str = "cpu", seed: int = 0, t0: int = 1692569000, fault_metric=None):
    """One RCAEval-RQ2-shaped case: ``time`` + ``<service>_<metric>`` columns, ``rows``
    one-second samples, a fault injected at the midpoint (returned as ``inject_time``):
    the root-cause metric shifts by 4 sigma and the shift propagates to its SEM descendants.
    Returns (DataFrame, inject_time)."""
    import pandas as pd

    services = services or OB_SERVICES
    metrics = metrics or OB_METRICS
    cols = [f"{s}_{m}" for s in services for m in metrics]
    n = len(cols)
    W, order, rng = sem_dag(n, edge_prob=3.0 / max(n - 1, 1), w_low=0.3, w_high=0.9, seed=seed)
    E = rng.standard_normal((rows, n))
    half = rows // 2
    root = cols.index(f"{root_service}_{(fault_metric or FAULT_METRIC)[fault]}")
    E[half:, root] += 4.0
    X = np.zeros((rows, n))
    for j in order:
        parents = np.nonzero(W[:, j])[0]
        col = E[:, j].copy()
        if parents.size:
            col += X[:, parents] @ W[parents, j]
        X[:, j] = col
    X = X * rng.uniform(0.5, 5.0, n) + rng.uniform(10, 100, n)
    for j, c in enumerate(cols):
        if c.endswith("_mem"):
            X[:, j] = np.abs(X[:, j]) * 1e6
    df = pd.DataFrame(X, columns=cols)
    df.insert(0, "time", np.arange(t0, t0 + rows))
    return df, t0 + half


def write_rq2_dataset(root: str, services=None, faults=("cpu", "mem", "delay"), cases: int = 2,
                      rows: int = 1200, seed: int = 0, flavor: str = "online-boutique") -> list:
    """An RQ2 case tree under ``root``: ``<service>_<fault>/<case>/{data.csv, inject_time.txt}``
    (``rq2.py:203-206,244-245``), Online-Boutique-shaped (``<svc>_{cpu,mem,latency-50,latency-90}``)
    or, with ``flavor="sock-shop"``, Sock-Shop-shaped (``<svc>_{cpu,mem,lat_50,lat_90,lat_99}``)."""
    import os

    ss = flavor == "sock-shop"
    all_services = SS_SERVICES if ss else OB_SERVICES
    kw = {"services": SS_SERVICES, "metrics": SS_METRICS, "fault_metric": SS_FAULT_METRIC} if ss else {}
    skip = ("front-end",) if ss else ("frontend", "redis")
    services = services or [s for s in all_services if s not in skip][:4]
    paths = []
    k = 0
    for svc in services:
        for fault in faults:
            for case in range(1, cases + 1):
                d = os.path.join(root, f"{svc}_{fault}", str(case))
                os.makedirs(d, exist_ok=True)
                df, inject = rq2_case_frame(root_service=svc, fault=fault, rows=rows, seed=seed + k, **kw)
                df.to_csv(os.path.join(d, "data.csv"), index=False)
                with open(os.path.join(d, "inject_time.txt"), "w") as f:
                    f.write(f"{inject}\n")
                paths.append(os.path.join(d, "data.csv"))
                k += 1
    return paths


def write_rq1_dataset(root: str, num_node: int = 10, graphs: int = 2, cases: int = 2, rows: int = 600,
                      seed: int = 0, edge_prob: float | None = None) -> list:
    """A CIRCA-shaped RQ1 tree (``rq1.py:122,201-204,158-160``):
    ``<root>/<num_node>/<graph_idx>/cases/<case_idx>/data.csv`` (no header row, one column per
    node) and ``<root>/<num_node>/<graph_idx>/graph.json`` (``MemoryGraph.dump`` layout, nodes
    ``Node("SIM", str(i))``, edges cause → effect as node indices)."""
    import json
    import os

    paths = []
    for g in range(graphs):
        gdir = os.path.join(root, str(num_node), str(g))
        os.makedirs(gdir, exist_ok=True)
        W, _, _ = sem_dag(num_node, edge_prob, 0.3, 0.9, seed=seed + 1000 * g)
        edges = [[int(i), int(j)] for i, j in zip(*np.nonzero(W))]
        with open(os.path.join(gdir, "graph.json"), "w") as f:
            json.dump({"nodes": [{"entity": "SIM", "metric": str(i)} for i in range(num_node)],
                       "edges": edges}, f, indent=2, sort_keys=True)
        for c in range(cases):
            cdir = os.path.join(gdir, "cases", str(c))
            os.makedirs(cdir, exist_ok=True)
            X = gaussian_sem(num_node, rows, edge_prob, 0.3, 0.9, seed=seed + 1000 * g)
            X += np.random.default_rng(seed + 1000 * g + c + 1).standard_normal(X.shape) * 0.1 * c
            np.savetxt(os.path.join(cdir, "data.csv"), X, delimiter=",", fmt="%.17g")
            paths.append(os.path.join(cdir, "data.csv"))
    return paths
