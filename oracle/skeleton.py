"""PC skeleton discovery — CPU oracle (test infrastructure only, pure Python loops).

Restates ``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:70-144`` (vendored copy of
the causal-learn loop; same loop in upstream 0.1.3.3 [U]) for ``background_knowledge=None``:

* start from the complete undirected graph (``GraphClass.py:26-28``);
* ``while max_degree() - 1 > depth`` (``:72``, ``GraphClass.py:104-106``);
* for x ascending, ``Neigh_x = np.where(g[x] != 0)`` (``GraphClass.py:100-102``);
  skip x if ``len(Neigh_x) < depth - 1`` (``:83``) — also skips its sepset appends;
* for y in Neigh_x, for S in ``combinations(Neigh_x \\ {y}, depth)`` (``:106``):
  ``p = ci_test(x, y, S)`` memoised on ``(min, max, frozenset(S))`` (``GraphClass.py:78-98``);
  ``p > alpha`` -> stable: defer removal of (x,y),(y,x) and union S into ``sepsets``
  (``:124-130``), non-stable: remove now, append S, break (``:112-123``);
  else ``append_value(p_values, x, y, p)`` (``:131-132``);
* stable: after the S loop append ``tuple(sepsets)`` to sepset[x,y] and [y,x]
  (``:135-136``); after all x remove every deferred edge (``:141-144``).

Only usable for small graphs (tests); ``cpc`` is the C restatement for larger ones.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from itertools import combinations

import numpy as np

from . import fisherz


def append_value(array: np.ndarray, i: int, j: int, value) -> None:
    """causal-learn ``PCUtils/Helper.append_value`` [U]."""
    if array[i, j] is None:
        array[i, j] = [value]
    else:
        array[i, j].append(value)


@dataclass
class SkeletonResult:
    adj: np.ndarray                      # n x n bool, symmetric
    sepset: np.ndarray                   # n x n object (lists of tuples) or None
    p_values: np.ndarray                 # n x n object (lists of floats) or None
    cache: dict                          # (a, b, S-tuple) -> p   (unique tests)
    removed_level: np.ndarray            # n x n int, -1 = never removed
    tests_per_level: list = field(default_factory=list)   # unique tests per depth
    calls_per_level: list = field(default_factory=list)   # ci_test invocations per depth
    max_depth_run: int = -1


def skeleton_discovery(C: np.ndarray, N: int, alpha: float = 0.05, stable: bool = True,
                       max_depth: int = -1, pvalue=None, forbidden=None) -> SkeletonResult:
    """Run the restated loop on a correlation matrix ``C`` (n x n) for ``N`` samples.
    ``forbidden``: n x n bool (background knowledge, x -> y forbidden); a pair forbidden both
    ways is queued for removal at every visit while its tests still run (``:86-106``, stable)."""
    assert 0 < alpha < 1
    assert forbidden is None or stable, "background knowledge is restated for the stable branch only"
    n = C.shape[0]
    pvalue = pvalue or (lambda x, y, S: fisherz.pvalue(C, N, x, y, S))
    g = np.ones((n, n), dtype=bool)
    np.fill_diagonal(g, False)
    sepset = np.empty((n, n), object)
    p_values = np.empty((n, n), object)
    removed_level = np.full((n, n), -1, dtype=np.int64)
    cache: dict = {}
    tests, calls = [], []

    def ci_test(x, y, S):
        a, b = (x, y) if x < y else (y, x)
        key = (int(a), int(b), tuple(sorted(int(s) for s in S)))
        if key in cache:
            return cache[key]
        p = pvalue(a, b, key[2])
        cache[key] = p
        return p

    depth = -1
    while g.sum(axis=1).max() - 1 > depth:
        if max_depth >= 0 and depth >= max_depth:
            break
        depth += 1
        before = len(cache)
        ncalls = 0
        edge_removal = []
        for x in range(n):
            Neigh_x = np.where(g[x])[0]
            if len(Neigh_x) < depth - 1:
                continue
            for y in Neigh_x:
                sepsets = set()
                if forbidden is not None and forbidden[x, y] and forbidden[y, x]:
                    edge_removal.append((x, y))
                    edge_removal.append((y, x))
                Neigh_x_noy = np.delete(Neigh_x, np.where(Neigh_x == y))
                for S in combinations(Neigh_x_noy, depth):
                    p = ci_test(x, y, S)
                    ncalls += 1
                    if p > alpha:
                        if not stable:
                            g[x, y] = g[y, x] = False
                            removed_level[x, y] = removed_level[y, x] = depth
                            append_value(sepset, x, y, S)
                            append_value(sepset, y, x, S)
                            break
                        edge_removal.append((x, y))
                        edge_removal.append((y, x))
                        for s in S:
                            sepsets.add(s)
                    else:
                        append_value(p_values, x, y, p)
                append_value(sepset, x, y, tuple(sepsets))     # :135-136, both modes
                append_value(sepset, y, x, tuple(sepsets))
        for x, y in set(edge_removal):
            g[x, y] = g[y, x] = False
            removed_level[x, y] = removed_level[y, x] = depth
        tests.append(len(cache) - before)
        calls.append(ncalls)
    return SkeletonResult(g, sepset, p_values, cache, removed_level, tests, calls, depth)


def endpoint_graph(adj: np.ndarray) -> np.ndarray:
    """Skeleton as causal-learn endpoint codes: i -- j  <=>  g[i,j] = g[j,i] = -1."""
    return np.where(adj, -1, 0).astype(int)
