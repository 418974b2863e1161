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
