"""Order-dependent PC skeleton (``stable=False``) on the MI355X engine.

Restates the ``not stable`` branch of ``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py:70-144``
(``RCAEval/graph_construction/pc.py:24-39`` ``pc_fisherz``; ``rq1.py:240-244``):

* depth loop ``while max_degree() - 1 > depth`` (``:72``); x ascending; ``Neigh_x`` taken from the
  current graph when x's turn comes (``:81``) and fixed for the rest of x's turn; skip x when
  ``len(Neigh_x) < depth - 1`` (``:83``);
* for y in Neigh_x: S over ``combinations(Neigh_x \\ {y}, depth)`` in lexicographic order; the first
  S with ``p > alpha`` removes x — y at once, appends S to sepset[x,y] and [y,x], and ends y's
  loop (``:112-123``); then ``()`` is appended to both (``:135-136``, ``sepsets`` stays empty
  in this branch).

Within x's turn every y is independent of the others (Neigh_x is fixed, and x's removals touch
only x's own edges), so one turn is one device batch: the pending (y, S) tests of every y are
sent to ``pcg_fisherz_batch`` in lexicographic chunks that grow geometrically, and each y stops
at its first independent S. Turns are sequential — x + 1 sees x's removals — exactly the
reference's order dependence. The arithmetic is the device LU path (``CITester``).
"""
from __future__ import annotations

from itertools import combinations, islice

import numpy as np

from .citest import CITester

_FIRST_CHUNK = 16
_MAX_CHUNK = 1 << 16


def append_value(array: np.ndarray, i: int, j: int, value) -> None:
    """causal-learn ``PCUtils.Helper.append_value`` [U]."""
    if array[i, j] is None:
        array[i, j] = [value]
    else:
        array[i, j].append(value)


class SeqSkeleton:
    """Result: adjacency, sepset lists (reference layout), removal depth, per-depth counts."""

    def __init__(self, n: int):
        self.adj = ~np.eye(n, dtype=bool)
        self.sepset = np.empty((n, n), object)
        self.p_values = np.empty((n, n), object)       # dependent p per (x, y), :131-132
        self.removed_level = np.full((n, n), -1, np.int64)
        self.calls: list = []
        self.levels = 0

    def sep_rows(self):
        """(sep_xy, sep_bits) rows for the orientation entry points: per ordered pair, the
        union of every tuple in sepset[x, y]."""
        n = self.adj.shape[0]
        W = (n + 63) // 64
        xy, bits = [], []
        for x in range(n):
            for y in range(n):
                lst = self.sepset[x, y]
                if x == y or not lst:
                    continue
                row = np.zeros(W, np.uint64)
                for S in lst:
                    for s in S:
                        row[int(s) >> 6] |= np.uint64(1 << (int(s) & 63))
                if row.any():
                    xy.append((x, y))
                    bits.append(row)
        return (np.array(xy, np.int32).reshape(-1, 2),
                np.array(bits, np.uint64).reshape(-1, W))


def skeleton_unstable(ci: CITester, alpha: float = 0.05, max_depth: int = -1) -> SeqSkeleton:
    n = ci.n
    out = SeqSkeleton(n)
    g = out.adj
    depth = -1
    while g.sum(axis=1).max() - 1 > depth:
        if 0 <= max_depth <= depth:
            break
        depth += 1
        calls = 0
        for x in range(n):
            nb = np.flatnonzero(g[x])
            if len(nb) < depth - 1:
                continue
            its = {int(y): combinations([int(v) for v in nb if v != y], depth) for y in nb}
            first: dict = {}
            k = _FIRST_CHUNK
            while its:
                tests, owner = [], []
                for y in list(its):
                    part = list(islice(its[y], k))
                    if not part:
                        del its[y]
                        continue
                    tests.extend((x, y, S) for S in part)
                    owner.extend((y, S) for S in part)
                if not tests:
                    break
                p, st = ci.pvalues_status(tests)
                for (y, S), pv, s_ in zip(owner, p, st):
                    if y in its:
                        calls += 1              # the reference's ci_test calls: up to the first p > alpha
                        ci.raise_for(s_)        # only tests the reference reaches may fail
                        if pv > alpha:
                            first[y] = S
                            del its[y]
                        else:
                            append_value(out.p_values, x, y, pv)
                k = min(4 * k, _MAX_CHUNK)
            for y in nb:
                y = int(y)
                S = first.get(y)
                if S is not None:
                    g[x, y] = g[y, x] = False
                    out.removed_level[x, y] = out.removed_level[y, x] = depth
                    append_value(out.sepset, x, y, S)
                    append_value(out.sepset, y, x, S)
                append_value(out.sepset, x, y, ())
                append_value(out.sepset, y, x, ())
        out.calls.append(calls)
    out.levels = depth + 1
    return out


__all__ = ["skeleton_unstable", "SeqSkeleton"]
