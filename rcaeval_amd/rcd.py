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
            rows = np.full((len(todo), 3 + max(dmax, 1)), -1, np.int32)
            cells = 1
            for r, (a, b, S) in enumerate(todo):
                s = sorted(S)
                rows[r, 0], rows[r, 1], rows[r, 2] = a, b, len(s)
                rows[r, 3:3 + len(s)] = s
                cells = max(cells, int(np.prod(self.card[s + [a, b]], dtype=np.float64)))
            if cells > (1 << 26):
                raise NotImplementedError(f"contingency table of {cells} cells")
            stat, df, st = self.eng.chisq_batch(self.data, self.card_dev, self.N, self.n, rows, self.g_sq, cells)
            with np.errstate(invalid="ignore"):
                p = np.where(df > 0, chi2.sf(stat, np.maximum(df, 1)), 1.0)
            for r, k in enumerate(todo):
                self.cache[k] = (float(p[r]), int(st[r]))
        got = [self.cache[k] for k in keys]
        return [g[0] for g in got], [g[1] for g in got]

    @staticmethod
    def raise_for(status: int) -> None:
        if status == 4:
            raise NotImplementedError("contingency table too large for the device batch")
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


# ---------------------------------------------------------------- rcd.py
def drop_constant(df):
    """``rcd.py:31-32``."""
    return df.loc[:, (df != df.iloc[0]).any()]


def add_fnode_and_concat(normal_df, anomalous_df):
    """``rcd.py:64-67`` (mutates both frames, like the reference)."""
    import pandas as pd
    normal_df[F_NODE] = "0"
    anomalous_df[F_NODE] = "1"
    return pd.concat([normal_df, anomalous_df])


def run_pc(data, alpha, localized=False, labels=None, mi=(), verbose=False, device=None):
    """``rcd.py:72-102``."""
    if not labels:
        labels = {i: name for i, name in enumerate(data.columns)}
    np_data = data.to_numpy()
    if localized:
        return local_skeleton_discovery(np_data, np_data.shape[1] - 1, alpha, mi=mi, labels=labels, device=device)
    return skeleton_unstable_discrete(np_data, alpha, labels=labels, device=device)


def _order_neighbors(neigh, p_values):
    """``rcd.py:211-222``."""
    _neigh = neigh.copy()
    _p_values = p_values.copy()
    stack = []
    while len(_neigh) != 0:
        i = np.argmax(_p_values)
        node = _neigh[i]
        stack = [node] + stack
        _neigh.remove(node)
        _p_values = np.delete(_p_values, i)
    return stack


def _discretize(data, bins):
    """``rcd.py:278-289`` (scikit-learn KBinsDiscretizer, k-means strategy, on the host)."""
    import warnings

    import pandas as pd
    from sklearn.preprocessing import KBinsDiscretizer
    d = data.iloc[:, :-1]
    discretizer = KBinsDiscretizer(n_bins=bins, encode="ordinal", strategy="kmeans")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        discretizer.fit(d)
        disc_d = discretizer.transform(d)
    disc_d = pd.DataFrame(disc_d, columns=d.columns.values.tolist())
    disc_d[F_NODE] = data[F_NODE].tolist()
    for c in disc_d:
        disc_d[c] = disc_d[c].astype(int)
    return disc_d


def _preprocess_for_fnode(normal_df, anomalous_df, bins):
    df = add_fnode_and_concat(normal_df, anomalous_df)
    if df is None:
        return None
    return _discretize(df, bins) if bins is not None else df


def run_psi_pc(normal_df, anomalous_df, bins=None, mi=None, localized=False, start_alpha=None, min_nodes=-1,
               verbose=False, device=None):
    """``rcd.py:121-208``: the alpha sweep; returns (rc, graph, mi, no_ci)."""
    if mi is None:
        mi = []
    if 0 in [len(normal_df.columns), len(anomalous_df.columns)]:
        return ([], None, [], 0)
    data = _preprocess_for_fnode(normal_df, anomalous_df, bins)
    if min_nodes == -1:
        min_nodes = len(data.columns) - 1
    assert min_nodes < len(data)
    G = None
    no_ci = 0
    i_to_labels = {i: name for i, name in enumerate(data.columns)}
    labels_to_i = {name: i for i, name in enumerate(data.columns)}
    processed_mi = [labels_to_i.get(i) for i in mi]
    rc = []
    cg = None
    _alpha = START_ALPHA if start_alpha is None else start_alpha
    for i in np.arange(_alpha, ALPHA_LIMIT, ALPHA_STEP):
        cg = run_pc(data, i, localized=localized, mi=processed_mi, labels=i_to_labels, verbose=verbose,
                    device=device)
        G = cg
        no_ci += cg.no_ci_tests
        f_neigh = cg.successors(data.shape[1] - 1)
        new_neigh = [x for x in f_neigh if x not in rc]
        if len(new_neigh) == 0:
            continue
        f_p_values = cg.p_values[-1][[labels_to_i.get(key) for key in new_neigh]]
        rc += _order_neighbors(new_neigh, f_p_values)
        if len(rc) == min_nodes:
            break
    mi_out = [i_to_labels.get(i) for i in list(filter(None, cg.mi))] if cg is not None else []
    return (rc, G, mi_out, no_ci)


def create_chunks(df, gamma):
    """``rcd.py:307-315``."""
    chunks = list()
    names = np.random.permutation(df.columns)
    for i in range(df.shape[1] // gamma + 1):
        chunks.append(names[i * gamma:(i * gamma) + gamma])
    if len(chunks[-1]) == 0:
        chunks.pop()
    return chunks


def run_level(normal_df, anomalous_df, gamma, localized, bins, verbose, device=None):
    """``rcd.py:318-375`` (phase 1: one Psi-PC per chunk of gamma variables)."""
    ci_tests = 0
    chunks = create_chunks(normal_df, gamma)
    f_child_union = []
    mi_union = []
    for c in chunks:
        rc, _, mi, ci = run_psi_pc(normal_df.loc[:, c], anomalous_df.loc[:, c], bins=bins, localized=localized,
                                   start_alpha=LOCAL_ALPHA, min_nodes=1, verbose=verbose, device=device)
        f_child_union += rc
        mi_union += mi
        ci_tests += ci
    return f_child_union, mi_union, ci_tests


def run_multi_phase(normal_df, anomalous_df, gamma, localized, bins, verbose, device=None):
    """``rcd.py:378-446``."""
    f_child_union = normal_df.columns
    mi_union = []
    prev = len(f_child_union)
    while True:
        f_child_union, mi, ci_tests = run_level(normal_df.loc[:, f_child_union], anomalous_df.loc[:, f_child_union],
                                                gamma, localized, bins, verbose, device=device)
        mi_union += mi
        len_child = len(f_child_union)
        if len_child <= gamma or len_child == prev:
            break
        prev = len(f_child_union)
    mi_union = []
    new_nodes = f_child_union
    rc, _, mi, ci = run_psi_pc(normal_df.loc[:, new_nodes], anomalous_df.loc[:, new_nodes], bins=bins, mi=mi_union,
                               localized=localized, verbose=verbose, device=device)
    return rc


# sock-shop / real-outage preprocessing (rcd.py:36-55, 227-275)
_rm_time = lambda df: df.loc[:, ~df.columns.isin(["time"])]   # noqa: E731


def _list_intersection(l1, l2):
    return [x for x in l1 if x in l2]


def _match_columns(n_df, a_df):
    cols = _list_intersection(n_df.columns, a_df.columns)
    return (n_df[cols], a_df[cols])


def _scale_down_mem(df):
    def update_mem(x):
        if not x.name.endswith("_mem"):
            return x
        x /= 1e6
        x = x.astype(int)
        return x
    return df.apply(update_mem)


def _select_lat(df, per):
    return df.filter(regex=(r".*(?<!lat_\d{2})$|_lat_" + str(per) + "$"))


def _select_useful_cols(df):
    i = df.loc[:, df.columns != F_NODE].std() > 1
    cols = i[i].index.tolist()
    cols.append(F_NODE)
    if len(cols) == 1:
        return None
    elif len(cols) == len(df.columns):
        return df
    return df[cols]


def preprocess_sock_shop(n_df, a_df, per, dk_select_useful=False):
    _process = lambda df: _select_lat(_scale_down_mem(_rm_time(df)), per)   # noqa: E731
    n_df = drop_constant(_process(n_df))
    a_df = drop_constant(_process(a_df))
    n_df, a_df = _match_columns(n_df, a_df)
    df = add_fnode_and_concat(n_df, a_df)
    if dk_select_useful is True:
        df = _select_useful_cols(df)
    n_df = df[df[F_NODE] == "0"].drop(columns=[F_NODE])
    a_df = df[df[F_NODE] == "1"].drop(columns=[F_NODE])
    return (n_df, a_df)


def rcd(data, inject_time, dk_select_useful=False, gamma=5, localized=True, bins=5, verbose=False, dataset=None,
        seed=None, device=None, **kwargs):
    """``rcd.py:449-493``: returns ``{"ranks": rc}``."""
    normal_df = data[data["time"] < inject_time]
    anomal_df = data[data["time"] >= inject_time]
    if dk_select_useful is True:
        normal_df = drop_extra(normal_df)
        anomal_df = drop_extra(anomal_df)
    if dataset == "sock-shop":
        normal_df, anomal_df = preprocess_sock_shop(normal_df, anomal_df, 90, dk_select_useful)
    elif dataset is not None:
        normal_df = _drop_constant_ts(convert_mem_mb(drop_time(normal_df)))
        anomal_df = _drop_constant_ts(convert_mem_mb(drop_time(anomal_df)))
        normal_df, anomal_df = _match_columns(normal_df, anomal_df)
        df = add_fnode_and_concat(normal_df, anomal_df)
        if dk_select_useful is True:
            df = _select_useful_cols(df)
        normal_df = df[df[F_NODE] == "0"].drop(columns=[F_NODE])
        anomal_df = df[df[F_NODE] == "1"].drop(columns=[F_NODE])
    if seed is not None:
        np.random.seed(seed)
    rc = run_multi_phase(normal_df, anomal_df, gamma, localized, bins, verbose, device=device)
    return {"ranks": rc}


__all__ = ["rcd", "ChiSqTester", "local_skeleton_discovery", "run_psi_pc", "run_multi_phase"]
