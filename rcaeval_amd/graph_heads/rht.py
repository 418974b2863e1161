"""CIRCA's regression-based hypothesis testing head — mirror of ``RCAEval/graph_heads/rht.py``
(``rht`` ``:331-403``, ``RHTScorer`` ``:158-235``, ``ANMRegressor`` ``:134-155``) and of the data
plumbing it goes through (``RCAEval/classes/data.py``: ``DataLoader.preprocess`` ``:64-108``,
``CaseData`` ``:152-243`` with ``lookup_window=120``, ``detect_window=10``, 1 s interval).

Same semantics, restated for batch execution:

* the case graph holds only nodes that appear in an edge (``graph.add_edge`` per endpoint pair,
  ``:350-379``), reversed (``:381``); a node's regressors are its parents in that graph;
* every column's series is resampled once, all columns together (``resample(1 s,
  origin="start").mean()``, time interpolation both ways, back-fill) — per column the same
  operations the reference runs node by node on the same (timestamp, value) rows, so the values
  are identical; series with one distinct value are pruned (``data.py:236-238``);
* per node: ``LinearRegression`` of the first ``train_window`` (111) points on its parents,
  residual z-scores of the last ``test_window`` (10) points against the training residuals
  (``StandardScaler``), ``max |z|`` (Python ``max``) is the score; parentless nodes (or
  regression ``ValueError``) use the plain z-score of the series;
* the global ``np.random`` stream advances by the reference's one ``np.random.choice(nodes)``
  (the SLI draw, ``:385``; the scorer never reads it).

The reference iterates Python sets of ``Node`` (``graph.nodes``, ``graph.parents``), so its
parent column order — and thus the last bits of each regression — depend on string hashing
(``PYTHONHASHSEED``); scores here use parents in ascending column order and agree with the
reference to rounding (tests compare at 1e-9 relative), ranks identical away from ties.
"""
from __future__ import annotations

from datetime import timedelta

import networkx as nx
import numpy as np
import pandas as pd
from scipy.stats import norm
from sklearn.linear_model import LinearRegression
from sklearn.preprocessing import StandardScaler

LOOKUP_WINDOW = 120           # CaseData defaults (data.py:158-176)
DETECT_WINDOW = 10
TRAIN_WINDOW = LOOKUP_WINDOW - DETECT_WINDOW + 1
TEST_WINDOW = DETECT_WINDOW


def zscore(train_y: np.ndarray, test_y: np.ndarray) -> np.ndarray:
    """``rht.py:23-29``."""
    scaler = StandardScaler().fit(train_y.reshape(-1, 1))
    return scaler.transform(test_y.reshape(-1, 1))[:, 0]


def zscore_conf(score: float) -> float:
    """``rht.py:32-36``."""
    return 1 - 2 * norm.cdf(-abs(score))


def _nodes(names):
    """``rht.py:344``: ``Node(name.split("_")[0], name.split("_")[1])`` keys as (entity, metric)."""
    return [(nm.split("_")[0], nm.split("_")[1]) for nm in names if nm != "time"]


def case_graph(adj, nodes) -> nx.DiGraph:
    """``rht.py:345-381``: endpoint pairs → edges (undirected → both ways), then reversed."""
    adj = np.asarray(adj)
    g = nx.DiGraph()
    n = len(adj)
    for a in range(n):
        for b in range(n):
            p, q = adj[a, b], adj[b, a]
            if p == q == 0:
                continue
            if p == q == -1 or (p == 1 and q == -1):
                g.add_edge(nodes[b], nodes[a])
            elif p == -1 and q == 1:
                g.add_edge(nodes[a], nodes[b])
            else:
                raise ValueError(f"Unexpected value: {p}, {q}")
    return g.reverse()


def resample_frame(times, frame: pd.DataFrame, start: float, end: float):
    """``DataLoader.preprocess`` (``data.py:64-108``) for all columns at once; None when no
    timestamp falls in [start, end]."""
    t = np.asarray(times, dtype=float)
    keep = (t >= start) & (t <= end)
    if not keep.any():
        return None
    vals = frame.to_numpy(dtype=float)[keep]
    tt = np.concatenate([t[keep], [start, end]])
    vals = np.vstack([vals, np.full((2, vals.shape[1]), np.nan)])
    df = pd.DataFrame(vals, columns=frame.columns)
    df.index = pd.to_datetime(tt, unit="s", utc=True)
    df = df.resample(timedelta(seconds=1), origin="start").mean()
    df = df.interpolate(method="time", limit_direction="both")
    df = df.bfill()
    return df.sort_index()


def _regress(train_x, test_x, train_y, test_y):
    """``Regressor.score`` + ``ANMRegressor._score`` (``rht.py:115-155``)."""
    if len(train_x) == 0:
        return zscore(train_y, test_y)
    try:
        reg = LinearRegression().fit(train_x, train_y)
        return zscore(train_y - reg.predict(train_x), test_y - reg.predict(test_x))
    except ValueError:
        return zscore(train_y, test_y)


def _pymax(values) -> float:
    """Python ``max`` over an array (first maximum, NaN semantics of ``>``)."""
    it = iter(values)
    try:
        best = next(it)
    except StopIteration:
        raise ValueError("max() arg is an empty sequence") from None
    for v in it:
        if v > best:
            best = v
    return best


def rht(adj, inject_time, data: pd.DataFrame, sli=None, num_loop=None, previous_scores=None):
    """``rht.py:331-403``: [("entity_metric", score)] sorted by score, descending."""
    names = data.columns.to_list()
    nodes = _nodes(names)
    graph = case_graph(adj, nodes)
    np.random.choice(len(nodes))                      # the reference's SLI draw (rht.py:385)
    present = {}
    for nm in names:
        if nm == "time":
            continue
        parts = nm.split("_")
        key = f"{parts[0]}_{parts[1]}"
        if key in data.columns:
            present[(parts[0], parts[1])] = key
    current = max(inject_time + 300, inject_time)
    start = inject_time - LOOKUP_WINDOW * 1.0
    length = int((current - start) / 1.0) + 1
    gnodes = [v for v in graph.nodes if v in present]
    series = {}
    if gnodes:
        cols = list(dict.fromkeys(present[v] for v in gnodes))
        rs = resample_frame(data["time"], data[cols], start, current)
        if rs is not None:
            for v in gnodes:
                s = rs[present[v]].to_numpy()
                if len(s) and len(set(s.tolist())) > 1:
                    series[v] = s[:length]
    order = {v: k for k, v in enumerate(nodes)}
    out = []
    for v, s in series.items():
        parents = sorted((p for p in graph.predecessors(v) if p in series), key=lambda p: order[p])
        y = np.asarray(s)
        if parents:
            x = np.array([series[p] for p in parents]).T
        else:
            x = np.zeros((0, 0))
        train_x, test_x = x[:TRAIN_WINDOW, :], x[-TEST_WINDOW:, :]
        train_y, test_y = y[:TRAIN_WINDOW], y[-TEST_WINDOW:]
        z = _pymax(np.abs(_regress(train_x, test_x, train_y, test_y)))
        out.append((f"{v[0]}_{v[1]}", z))
    out.sort(key=lambda t: t[1], reverse=True)
    return out


__all__ = ["rht", "zscore", "zscore_conf", "case_graph", "resample_frame"]
