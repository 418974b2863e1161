"""RCD (root-cause discovery with the F-node Psi-PC) on the MI355X engine.

Mirror of ``RCAEval/e2e/rcd.py:18-493``: the F-node data layout (``add_fnode_and_concat``
``:64-67``), k-means discretisation (``_discretize`` ``:278-289``), the chunked phase-1 /
phase-2 search (``run_level`` ``:318-375``, ``run_multi_phase`` ``:378-446``), the alpha sweep of
``run_psi_pc`` (``:121-208``) and ``run_pc`` (``:72-102``), whose skeletons are
``local_skeleton_discovery`` (``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:152-210``,
the default ``localized=True``) or the order-dependent ``skeleton_discovery(stable=False)``
(``:70-144``) — with causal-learn's ``chisq`` CI test [U] (``CI_TEST = chisq``, ``:21``).

The discrete CI tests run on the device (``pcg_chisq_batch``: contingency tables, the
chi-square statistic summed like numpy, and df); p = ``scipy.stats.chi2.sf(stat, df)`` is taken
on the host for each batch (p = 1 when df <= 0, as causal-learn does). The global
``numpy.random`` stream is consumed exactly where the reference consumes it
(``np.random.permutation`` in ``create_chunks`` ``:309`` and in every depth of
``local_skeleton_discovery`` ``:183``), so a seeded run reproduces the reference's chunks and
visit orders. causal-learn 0.1.2.3's ``chisq`` is not on disk: **parity unpinned** beyond the
restated arithmetic.
"""
from __future__ import annotations

from itertools import combinations

import numpy as np

from . import _lib
from .engine import get_engine
from .io.time_series import convert_mem_mb, drop_extra, drop_time
from .io.time_series import drop_constant as _drop_constant_ts

CI_TEST = "chisq"
START_ALPHA = 0.001
ALPHA_STEP = 0.1
ALPHA_LIMIT = 1
F_NODE = "F-node"
LOCAL_ALPHA = 0.01
DEFAULT_GAMMA = 5


# ---------------------------------------------------------------- device CI test
class ChiSqTester:
    """``cg.ci_test`` with chisq / gsq (``GraphClass.py:78-98`` cache key and call count) on the
    device; ``data`` are the integer codes of ``np.apply_along_axis(_unique, 0, data)``."""

    MAX_CELLS = 1 << 26          # largest contingency table one device test builds

    def __init__(self, codes: np.ndarray, cardinalities: np.ndarray, g_sq: bool = False, device: int | None = None):
        import torch
        self.eng = get_engine(device)
        codes = np.asarray(codes, dtype=np.int64)
        self.N, self.n = codes.shape
        self.card = np.asarray(cardinalities, dtype=np.int64)
        self.data = torch.from_numpy(np.ascontiguousarray(codes.T.astype(np.int32))).to(self.eng.device)
        self.card_dev = torch.from_numpy(self.card.astype(np.int32)).to(self.eng.device)
        self.g_sq = bool(g_sq)
        self.cache: dict = {}
        self.no_ci_tests = 0

    @staticmethod
    def key(i, j, S):
        i, j = (int(i), int(j)) if i < j else (int(j), int(i))
        return i, j, frozenset(int(s) for s in S)

    def pvalues_status(self, tests):
        from scipy.stats import chi2
        keys = [self.key(i, j, S) for (i, j, S) in tests]
        self.no_ci_tests += len(keys)
        todo = list(dict.fromkeys(k for k in keys if k not in self.cache))
        if todo:
            dmax = max(len(k[2]) for k in todo)
            if dmax > _lib.PCG_MAX_LEVEL_DEPTH:
                raise NotImplementedError(f"conditioning set of size {dmax} > {_lib.PCG_MAX_LEVEL_DEPTH}")
            # a table beyond MAX_CELLS is marked per test (status 4) instead of failing the batch:
            # it raises only if the caller consumes that test (the reference may stop before it)
            fits, cells = [], 1
            for k in todo:
                c = int(np.prod(self.card[sorted(k[2]) + [k[0], k[1]]], dtype=np.float64))
                if c > self.MAX_CELLS:
                    self.cache[k] = (float("nan"), 4)
                else:
                    fits.append(k)
                    cells = max(cells, c)
            if fits:
                rows = np.full((len(fits), 3 + max(dmax, 1)), -1, np.int32)
                for r, (a, b, S) in enumerate(fits):
                    s = sorted(S)
                    rows[r, 0], rows[r, 1], rows[r, 2] = a, b, len(s)
                    rows[r, 3:3 + len(s)] = s
                stat, df, st = self.eng.chisq_batch(self.data, self.card_dev, self.N, self.n, rows, self.g_sq, cells)
                with np.errstate(invalid="ignore"):
                    p = np.where(df > 0, chi2.sf(stat, np.maximum(df, 1)), 1.0)
                for r, k in enumerate(fits):
                    self.cache[k] = (float(p[r]), int(st[r]))
        got = [self.cache[k] for k in keys]
        return [g[0] for g in got], [g[1] for g in got]

    @staticmethod
    def raise_for(status: int) -> None:
        if status == 4:
            raise NotImplementedError(f"contingency table beyond {ChiSqTester.MAX_CELLS} cells")
        if status != 0:
            raise AssertionError("X, Y cannot be in condition_set.")

    def pvalues(self, tests):
        p, st = self.pvalues_status(tests)
        for s_ in st:
            self.raise_for(s_)
        return p

    def __call__(self, i, j, S) -> float:
        return self.pvalues([(i, j, S)])[0]


def _unique(column):
    return np.unique(column, return_inverse=True)[1]


def discrete_codes(data: np.ndarray):
    """``SkeletonDiscovery.py:163-170``: per-column integer codes and cardinalities."""
    codes = np.apply_along_axis(_unique, 0, data).astype(np.int64)
    return codes, np.max(codes, axis=0) + 1


def _append_value(array, i, j, value):
    if array[i, j] is None:
        array[i, j] = [value]
    else:
        array[i, j].append(value)


class LocalGraph:
    """The ``CausalGraph`` fields RCD reads (``GraphClass.py:18-60``): endpoint matrix, sepset,
    p_values, mi, no_ci_tests, labels; ``f_children`` = ``to_nx_graph`` + ``successors``."""

    def __init__(self, n: int, labels: dict):
        self.graph = -np.ones((n, n), int) + np.eye(n, dtype=int)      # complete, TAIL-TAIL
        self.sepset = np.empty((n, n), object)
        self.p_values = np.empty((n, n), object)
        self.mi = np.empty(n, object)
        self._mi_index = 0
        self.labels = labels if labels else {i: f"X{i + 1}" for i in range(n)}
        self.no_ci_tests = 0

    def neighbors(self, i):
        return np.where(self.graph[i, :] != 0)[0]

    def max_degree(self):
        return max(np.sum(self.graph != 0, axis=1))

    def remove_edge(self, x, y):
        self.graph[x, y] = self.graph[y, x] = 0

    def append_to_mi(self, node):
        self.mi[self._mi_index] = node
        self._mi_index += 1

    def successors(self, node: int) -> list:
        """``to_nx_graph`` (``GraphClass.py:219-240``) adds i -> j for both orders of every
        undirected edge in row-major order of the endpoint matrix, so the successors of a node
        are its neighbours in ascending index order."""
        return [self.labels[int(j)] for j in np.flatnonzero((self.graph[:, node] == -1) & (self.graph[node, :] == -1))]


def local_skeleton_discovery(data: np.ndarray, local_node: int, alpha: float, mi=(), labels=None,
                             g_sq: bool = False, device: int | None = None) -> LocalGraph:
    """``SkeletonDiscovery.py:152-210`` with the device chisq test: only the local node's edges
    are tested; per depth its neighbours are visited in ``np.random.permutation`` order, y's
    conditioning candidates are y's neighbours adjacent to x (read live), and the first
    independent S removes the edge at once (and records y in ``mi`` at depth 0)."""
    assert type(data) == np.ndarray
    assert local_node <= data.shape[1]
    assert 0 < alpha < 1
    n = data.shape[1]
    codes, card = discrete_codes(data)
    ci = ChiSqTester(codes, card, g_sq=g_sq, device=device)
    cg = LocalGraph(n, dict(labels or {}))
    x = local_node
    for i in mi:
        cg.remove_edge(x, i)
    depth = -1
    while cg.max_degree() - 1 > depth:
        depth += 1
        local_neigh = np.random.permutation(cg.neighbors(x))
        for y in local_neigh:
            Neigh_y = cg.neighbors(y)
            Neigh_y = np.delete(Neigh_y, np.where(Neigh_y == x))
            Neigh_y_f = []
            if depth > 0:
                Neigh_y_f = [s for s in Neigh_y if x in cg.neighbors(s)]
            subsets = list(combinations(Neigh_y_f, depth))
            if not subsets:
                continue
            p, st = ci.pvalues_status([(x, y, S) for S in subsets])   # one device batch per y
            for S, pv, s_ in zip(subsets, p, st):
                cg.no_ci_tests += 1                # reference ci_test calls: up to the first p > alpha
                ci.raise_for(s_)
                if pv > alpha:
                    cg.remove_edge(x, y)
                    _append_value(cg.sepset, x, y, S)
                    _append_value(cg.sepset, y, x, S)
                    if depth == 0:
                        cg.append_to_mi(y)
                    break
                _append_value(cg.p_values, x, y, pv)
    return cg


def skeleton_unstable_discrete(data: np.ndarray, alpha: float, labels=None, g_sq: bool = False,
                               device: int | None = None) -> LocalGraph:
    """``skeleton_discovery(stable=False)`` with chisq (``run_pc(localized=False)``, ``:90-99``)."""
    from .skeleton_seq import skeleton_unstable
    codes, card = discrete_codes(data)
    ci = ChiSqTester(codes, card, g_sq=g_sq, device=device)
    sk = skeleton_unstable(ci, alpha=alpha)
    n = data.shape[1]
    cg = LocalGraph(n, dict(labels or {}))
    cg.graph = np.where(sk.adj, -1, 0)
    cg.sepset = sk.sepset
    cg.p_values = sk.p_values
    cg.no_ci_tests = int(sum(sk.calls))
    return cg


# ---------------------------------------------------------------- the RCD search (rcd.py)
# Reference behaviour kept: every frame operation that decides values or column order, the two
# numpy.random consumption points (create_chunks; local_skeleton_discovery per depth), the
# in-place F-node column on the frames handed to run_psi_pc (``add_fnode_and_concat``), and the
# quirks of the result (object-array argmax in the neighbour order, ``filter(None, mi)``).
import re
from typing import NamedTuple


class PsiResult(NamedTuple):
    """``run_psi_pc``'s 4-tuple (``rcd.py:121-208``): ranks, graph, mi labels, CI-test count."""
    ranks: list
    graph: object
    mi: list
    ci_tests: int


def drop_constant(df):
    """Columns with some value different from the first row (``rcd.py:31-32``; NaN counts as
    different)."""
    return df.loc[:, df.ne(df.iloc[0]).any(axis=0)]


def add_fnode_and_concat(normal_df, anomalous_df):
    """Label the windows ("0" normal, "1" anomalous) IN PLACE and stack them, normal first
    (``rcd.py:64-67``)."""
    import pandas as pd
    for frame, flag in ((normal_df, "0"), (anomalous_df, "1")):
        frame[F_NODE] = flag
    return pd.concat([normal_df, anomalous_df])


def _discretize(data, bins):
    """k-means binning of every column but the (last) F-node, all codes as int
    (``rcd.py:278-289``, scikit-learn KBinsDiscretizer on the host)."""
    import warnings

    import pandas as pd
    from sklearn.preprocessing import KBinsDiscretizer
    values = data.iloc[:, :-1]
    binner = KBinsDiscretizer(n_bins=bins, encode="ordinal", strategy="kmeans")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        coded = binner.fit(values).transform(values)
    out = pd.DataFrame(coded, columns=list(values.columns))
    out[F_NODE] = list(data[F_NODE])
    return out.astype({c: int for c in out.columns})


def _preprocess_for_fnode(normal_df, anomalous_df, bins):
    joined = add_fnode_and_concat(normal_df, anomalous_df)
    return joined if bins is None else _discretize(joined, bins)


def run_pc(data, alpha, localized=False, labels=None, mi=(), verbose=False, device=None):
    """Skeleton of the F-node frame (``rcd.py:72-102``): the localized search around the last
    column (the F-node), or the full order-dependent skeleton."""
    labels = labels or dict(enumerate(data.columns))
    X = data.to_numpy()
    if not localized:
        return skeleton_unstable_discrete(X, alpha, labels=labels, device=device)
    return local_skeleton_discovery(X, X.shape[1] - 1, alpha, mi=mi, labels=labels, device=device)


def _order_neighbors(neigh, p_values):
    """Repeatedly take the neighbour whose p-value list is largest (``np.argmax`` over the object
    array of lists: lexicographic) and put it in front: the first taken ends last
    (``rcd.py:211-222``)."""
    pending, scores, taken = list(neigh), p_values.copy(), []
    while pending:
        k = int(np.argmax(scores))
        taken.append(pending.pop(k))
        scores = np.delete(scores, k)
    return taken[::-1]


def run_psi_pc(normal_df, anomalous_df, bins=None, mi=None, localized=False, start_alpha=None, min_nodes=-1,
               verbose=False, device=None) -> PsiResult:
    """Psi-PC (``rcd.py:121-208``): raise alpha from ``start_alpha`` in steps of 0.1 below 1; each
    run's new F-node children join the ranking, ordered by their p-values, until ``min_nodes``
    (default: every variable) are ranked."""
    if len(normal_df.columns) == 0 or len(anomalous_df.columns) == 0:
        return PsiResult([], None, [], 0)
    data = _preprocess_for_fnode(normal_df, anomalous_df, bins)
    names = list(data.columns)
    fnode = len(names) - 1
    target = fnode if min_nodes == -1 else min_nodes
    assert target < len(data)
    index_of = {nm: k for k, nm in enumerate(names)}
    label_of = dict(enumerate(names))
    mi_index = [index_of.get(v) for v in (mi or [])]
    ranks, ci_total, cg = [], 0, None
    first = START_ALPHA if start_alpha is None else start_alpha
    for alpha in np.arange(first, ALPHA_LIMIT, ALPHA_STEP):
        cg = run_pc(data, alpha, localized=localized, mi=mi_index, labels=label_of, device=device)
        ci_total += cg.no_ci_tests
        fresh = [v for v in cg.successors(fnode) if v not in ranks]
        if not fresh:
            continue
        ranks += _order_neighbors(fresh, cg.p_values[-1][[index_of[v] for v in fresh]])
        if len(ranks) == target:
            break
    # filter(None, ...) drops the unset slots and node index 0 alike (reference quirk)
    mi_labels = [label_of.get(k) for k in filter(None, cg.mi)] if cg is not None else []
    return PsiResult(ranks, cg, mi_labels, ci_total)


def create_chunks(df, gamma):
    """Random partition of the columns into runs of ``gamma`` (``rcd.py:307-315``); draws one
    ``np.random.permutation``."""
    order = np.random.permutation(df.columns)
    chunks = [order[k:k + gamma] for k in range(0, (df.shape[1] // gamma + 1) * gamma, gamma)]
    if len(chunks[-1]) == 0:
        chunks.pop()
    return chunks


def run_level(normal_df, anomalous_df, gamma, localized, bins, verbose, device=None):
    """Phase 1, one level (``rcd.py:318-375``): Psi-PC on each chunk from alpha 0.01 until one
    F-node child is found; returns (children, mi labels, CI tests) over all chunks."""
    children, mi_labels, ci_total = [], [], 0
    for cols in create_chunks(normal_df, gamma):
        res = run_psi_pc(normal_df.loc[:, cols], anomalous_df.loc[:, cols], bins=bins, localized=localized,
                         start_alpha=LOCAL_ALPHA, min_nodes=1, verbose=verbose, device=device)
        children.extend(res.ranks)
        mi_labels.extend(res.mi)
        ci_total += res.ci_tests
    return children, mi_labels, ci_total


def run_multi_phase(normal_df, anomalous_df, gamma, localized, bins, verbose, device=None):
    """Phase 1 levels until at most ``gamma`` candidates remain or a level removes none, then
    phase 2: a full Psi-PC ranking of the survivors (``rcd.py:378-446``; the mi collected in
    phase 1 is discarded before phase 2, as there)."""
    survivors = normal_df.columns
    count = len(survivors)
    while True:
        survivors, _, _ = run_level(normal_df.loc[:, survivors], anomalous_df.loc[:, survivors], gamma, localized,
                                    bins, verbose, device=device)
        if len(survivors) <= gamma or len(survivors) == count:
            break
        count = len(survivors)
    return run_psi_pc(normal_df.loc[:, survivors], anomalous_df.loc[:, survivors], bins=bins, mi=[],
                      localized=localized, verbose=verbose, device=device).ranks


# --- window cleaning before the search (rcd.py:36-55, 227-275, 466-483)
_LAT_ANY = re.compile(r"lat_\d{2}$")


def _select_lat(df, per):
    """Non-latency columns plus the ``_lat_<per>`` ones (``rcd.py:271-272``)."""
    return df[[c for c in df.columns if _LAT_ANY.search(c) is None or c.endswith(f"_lat_{per}")]]


def _scale_down_mem(df):
    """``*_mem`` columns in MB, truncated to int (``rcd.py:259-268``)."""
    out = df.copy()
    for c in out.columns:
        if c.endswith("_mem"):
            out[c] = (out[c] / 1e6).astype(int)
    return out


def _select_useful_cols(df):
    """Columns whose std over both windows exceeds 1, F-node kept last; None when none is
    (``rcd.py:240-251``)."""
    wide = df.loc[:, df.columns != F_NODE].std() > 1
    keep = [c for c, w in wide.items() if w] + [F_NODE]
    if len(keep) == 1:
        return None
    return df if len(keep) == len(df.columns) else df[keep]


def _split_windows(normal_df, anomal_df, clean, select_useful):
    """Clean each window, keep their common columns (normal's order), optionally the useful
    ones, and split back on the F-node label."""
    normal_df, anomal_df = clean(normal_df), clean(anomal_df)
    common = [c for c in normal_df.columns if c in anomal_df.columns]
    joined = add_fnode_and_concat(normal_df[common], anomal_df[common])
    if select_useful is True:
        joined = _select_useful_cols(joined)
    flag = joined[F_NODE]
    return joined[flag == "0"].drop(columns=[F_NODE]), joined[flag == "1"].drop(columns=[F_NODE])


def preprocess_sock_shop(n_df, a_df, per, dk_select_useful=False):
    """Sock Shop / real-outage cleaning (``rcd.py:36-55``)."""
    def clean(df):
        return drop_constant(_select_lat(_scale_down_mem(df.loc[:, ~df.columns.isin(["time"])]), per))
    return _split_windows(n_df, a_df, clean, dk_select_useful)


def _preprocess_generic(n_df, a_df, dk_select_useful=False):
    """Every other named dataset (``rcd.py:474-483``: time dropped, memory in MB, constants
    dropped)."""
    return _split_windows(n_df, a_df, lambda df: _drop_constant_ts(convert_mem_mb(drop_time(df))),
                          dk_select_useful)


def rcd(data, inject_time, dk_select_useful=False, gamma=5, localized=True, bins=5, verbose=False, dataset=None,
        seed=None, device=None, **kwargs):
    """``rcd.py:449-493``: split at ``inject_time``, clean per dataset, seed the global stream,
    run both phases; returns ``{"ranks": ...}``."""
    normal_df = data[data["time"] < inject_time]
    anomal_df = data[data["time"] >= inject_time]
    if dk_select_useful is True:
        normal_df, anomal_df = drop_extra(normal_df), drop_extra(anomal_df)
    if dataset == "sock-shop":
        normal_df, anomal_df = preprocess_sock_shop(normal_df, anomal_df, 90, dk_select_useful)
    elif dataset is not None:
        normal_df, anomal_df = _preprocess_generic(normal_df, anomal_df, dk_select_useful)
    if seed is not None:
        np.random.seed(seed)
    return {"ranks": run_multi_phase(normal_df, anomal_df, gamma, localized, bins, verbose, device=device)}


__all__ = ["rcd", "ChiSqTester", "local_skeleton_discovery", "run_psi_pc", "run_multi_phase", "run_level",
           "create_chunks", "PsiResult"]
