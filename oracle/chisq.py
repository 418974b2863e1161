"""Discrete CI tests and RCD's local skeleton — CPU oracle, TEST INFRASTRUCTURE ONLY.

* ``chisq_or_gsq_test`` restates causal-learn's ``utils/cit.py`` contingency test [U]
  (causal-learn 0.1.2.3 of RCAEval's RCD environment, ``requirements_rcd.lock:20``; not on
  disk): stratum index over [S..., X, Y] with ``cardCumProd`` (S[0] fastest), empty strata
  dropped, E = Sx * Sy / Sm, chi-square = sum (T - E)^2 / (E or 1), G-square = 2 sum T log(T/E)
  (ratio 0 -> 1), df = sum_k (|X| - 1 - zero rows_k) (|Y| - 1 - zero cols_k), p = chi2.sf.
  Pinned for S = {} against ``scipy.stats.chi2_contingency(correction=False)`` (CPU tests).
* ``local_skeleton_discovery`` restates ``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:
  152-210`` statement by statement (one ``ci_test`` call at a time, cache key of
  ``GraphClass.py:87-97``).
"""
from __future__ import annotations

from itertools import combinations

import numpy as np
from scipy.stats import chi2


def chisq_or_gsq_stat(dataSXY: np.ndarray, cardSXY: np.ndarray, G_sq: bool = False):
    """(statistic, df) of the [U] test; dataSXY is (|S| + 2) x N integer codes."""
    cardSXY = np.asarray(cardSXY, dtype=np.int64)
    cardX, cardY = cardSXY[-2:]
    if len(cardSXY) == 2:
        xyIndexed = dataSXY[0] * cardY + dataSXY[1]
        xy = np.bincount(xyIndexed, minlength=cardX * cardY).reshape((cardX, cardY))
        xm, ym = np.sum(xy, axis=1), np.sum(xy, axis=0)
        c = xy[None]
        e = (np.outer(xm, ym) / dataSXY.shape[1])[None]
    else:
        cardS = int(np.prod(cardSXY[:-2]))
        cum = np.ones_like(cardSXY)
        cum[1:] = np.cumprod(cardSXY[:-1])
        idx = np.dot(cum[None], dataSXY)[0]
        T = np.bincount(idx, minlength=cardS * cardX * cardY).reshape((cardY, cardX, cardS))
        T = np.transpose(T, (2, 1, 0))
        Sm = np.sum(T, axis=(1, 2))
        keep = Sm != 0
        Sm, T = Sm[keep], T[keep]
        Sx, Sy = np.sum(T, axis=2), np.sum(T, axis=1)
        c = T
        e = Sx[:, :, None] * Sy[:, None, :] / Sm[:, None, None]
    zero = e == 0
    e1 = np.copy(e)
    e1[zero] = 1
    if not G_sq:
        stat = np.sum(((c - e) ** 2) / e1)
    else:
        div = np.divide(c, e1)
        div[div == 0] = 1
        stat = 2 * np.sum(c * np.log(div))
    zr = zero.all(axis=2).sum(axis=1)
    zc = zero.all(axis=1).sum(axis=1)
    df = int(np.sum((c.shape[1] - 1 - zr) * (c.shape[2] - 1 - zc)))
    return float(stat), df


def chisq(data, X, Y, S, cardinalities, G_sq=False):
    """causal-learn ``chisq(data, X, Y, conditioning_set, cardinalities)`` [U]."""
    idx = list(S) + [X, Y]
    stat, df = chisq_or_gsq_stat(data[:, idx].T, cardinalities[idx], G_sq)
    return 1.0 if df <= 0 else float(chi2.sf(stat, df))


def _unique(column):
    return np.unique(column, return_inverse=True)[1]


class LocalCG:
    def __init__(self, n, labels):
        self.graph = -np.ones((n, n), int) + np.eye(n, dtype=int)
        self.sepset = np.empty((n, n), object)
        self.p_values = np.empty((n, n), object)
        self.mi = np.empty(n, object)
        self._mi_index = 0
        self.labels = labels
        self.no_ci_tests = 0
        self.cache = {}

    def neighbors(self, i):
        return np.where(self.graph[i, :] != 0)[0]

    def max_degree(self):
        return max(np.sum(self.graph != 0, axis=1))

    def remove_edge(self, x, y):
        self.graph[x, y] = self.graph[y, x] = 0

    def append_to_mi(self, node):
        self.mi[self._mi_index] = node
        self._mi_index += 1

    def successors(self, node):
        return [self.labels[int(j)] for j in np.flatnonzero((self.graph[:, node] == -1) & (self.graph[node, :] == -1))]


def _append(array, i, j, v):
    if array[i, j] is None:
        array[i, j] = [v]
    else:
        array[i, j].append(v)


def local_skeleton_discovery(data, local_node, alpha, mi=(), labels=None, G_sq=False):
    """``SkeletonDiscovery.py:152-210`` with ``chisq``."""
    n = data.shape[1]
    codes = np.apply_along_axis(_unique, 0, data).astype(np.int64)
    card = np.max(codes, axis=0) + 1
    cg = LocalCG(n, dict(labels or {i: f"X{i + 1}" for i in range(n)}))

    def ci_test(i, j, S):
        cg.no_ci_tests += 1
        i, j = (i, j) if i < j else (j, i)
        key = (int(i), int(j), frozenset(int(s) for s in S))
        if key not in cg.cache:
            cg.cache[key] = chisq(codes, i, j, S, card, G_sq)
        return cg.cache[key]

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
            for S in combinations(Neigh_y_f, depth):
                p = ci_test(x, y, S)
                if p > alpha:
                    cg.remove_edge(x, y)
                    _append(cg.sepset, x, y, S)
                    _append(cg.sepset, y, x, S)
                    if depth == 0:
                        cg.append_to_mi(y)
                    break
                else:
                    _append(cg.p_values, x, y, p)
    return cg
