"""Caller-driven Fisher-z CI tests on the MI355X engine, and the orientation rules that need them.

``CITester`` mirrors the part of causal-learn's ``CausalGraph.ci_test`` [V]
(``lib/causallearn/graph/GraphClass.py:78-98``) and ``FisherZ.__call__`` [U] that callers
outside the level enumeration use: canonical cache key ``(min(i,j), max(i,j), frozenset(S))``,
a memo shared by every call, ``ValueError`` for a singular sub-matrix or a math domain error,
``AssertionError`` when x or y is in S. Tests are evaluated in batches by
``pcg_fisherz_batch`` (one lane per test, LU like ``numpy.linalg.inv``) — there is no host
arithmetic and no CPU fallback.

``uc_orient`` is ``UCSepset.uc_sepset(cg, priority)`` [U] + ``Meek.meek`` [U] for priorities
2, 3 and 4: the R0 candidates come from host C++ (``pcg_uc_candidates``), priority 3 / 4
score each candidate by the max p over ``find_cond_sets_without_mid`` / ``_with_mid``
(``GraphClass.py:190-204``), stable-sort ascending / descending (``sort_dict_ascending``),
and the collider step + Meek run in host C++ (``pcg_orient_triples``).
"""
from __future__ import annotations

from itertools import chain, combinations

import numpy as np

from . import _lib
from .engine import get_engine, orient, orient_bk, orient_triples, uc_candidates

# upper bound on the tests one priority-3/4 orientation may issue (the power sets of two
# neighbourhoods grow as 2^deg; the reference would not finish either)
MAX_UC_TESTS = 50_000_000
_BATCH = 1 << 20


def powerset(L):
    """``causallearn.utils.PCUtils.Helper.powerset`` [U]: subsets by size, combinations order."""
    s = list(L)
    return list(chain.from_iterable(combinations(s, r) for r in range(len(s) + 1)))


def list_union(L1, L2):
    """``Helper.list_union`` [U]: L1, then the members of L2 that are not in L1."""
    seen = set(L1)
    return L1 + [x for x in L2 if x not in seen]


class CITester:
    """Memoised Fisher-z tests of one data set on one device (``cg.ci_test`` semantics)."""

    def __init__(self, C, N: int, device: int | None = None):
        self.eng = get_engine(device)
        self.C = self.eng.to_device(C)
        self.n = int(self.C.shape[0])
        self.N = int(N)
        self.cache: dict = {}
        self.no_ci_tests = 0

    @staticmethod
    def key(i, j, S):
        i, j = (int(i), int(j)) if i < j else (int(j), int(i))
        return i, j, frozenset(int(s) for s in S)

    def pvalues(self, tests) -> list:
        """p of every ``(i, j, S)`` in ``tests`` (cache misses evaluated in device batches);
        raises like the reference on the first failing test."""
        p, st = self.pvalues_status(tests)
        for s_ in st:
            self.raise_for(s_)
        return p

    @staticmethod
    def raise_for(status: int) -> None:
        if status == 1:
            raise ValueError("Data correlation matrix is singular. Cannot run fisherz test. "
                             "Please check your data.")
        if status == 2:
            raise ValueError("math domain error")
        if status != 0:
            raise AssertionError("X, Y cannot be in condition_set.")

    def pvalues_status(self, tests):
        """(p list, status list) without raising: status 0 ok, 1 singular, 2 math domain, 3
        malformed — for callers that must only fail on tests the reference would reach."""
        keys = [self.key(i, j, S) for (i, j, S) in tests]
        self.no_ci_tests += len(keys)
        todo = list(dict.fromkeys(k for k in keys if k not in self.cache))
        for lo in range(0, len(todo), _BATCH):
            part = todo[lo:lo + _BATCH]
            dmax = max(len(k[2]) for k in part)
            if dmax > _lib.PCG_MAX_LEVEL_DEPTH:
                raise NotImplementedError(f"conditioning set of size {dmax} > {_lib.PCG_MAX_LEVEL_DEPTH}")
            rows = np.full((len(part), 3 + max(dmax, 1)), -1, np.int32)
            for r, (a, b, S) in enumerate(part):
                s = sorted(S)
                rows[r, 0], rows[r, 1], rows[r, 2] = a, b, len(s)
                rows[r, 3:3 + len(s)] = s
            p, st = self.eng.fisherz_batch(self.C, self.N, rows)
            for r, k in enumerate(part):
                self.cache[k] = (float(p[r]), int(st[r]))
        got = [self.cache[k] for k in keys]
        return [g[0] for g in got], [g[1] for g in got]

    def __call__(self, i, j, S) -> float:
        return self.pvalues([(i, j, S)])[0]


def uc_orient(adj: np.ndarray, sep_xy: np.ndarray, sep_bits: np.ndarray, priority: int,
              ci: CITester | None = None, knowledge: tuple | None = None) -> np.ndarray:
    """``uc_sepset(cg, priority)`` then ``meek`` → endpoint-code matrix (int32).
    ``knowledge=(forbidden, required)`` masks (``BackgroundKnowledge.masks``): the run goes through
    ``orient_by_background_knowledge`` first and both steps skip what the masks rule out."""
    if priority == 2:
        if knowledge is not None:
            return orient_bk(adj, sep_xy, sep_bits, *knowledge, priority=2)
        return orient(adj, sep_xy, sep_bits, priority=2)
    if priority not in (3, 4):
        raise NotImplementedError(f"uc_priority={priority}: priorities 2, 3 and 4 are built")
    if ci is None:
        raise ValueError("priority 3/4 orientation needs a CITester")
    R0 = uc_candidates(adj, sep_xy, sep_bits)
    nbrs = [np.flatnonzero(adj[i]) for i in range(adj.shape[0])]
    with_mid = priority == 4
    spans, tests = [], []
    for (x, y, z) in R0.tolist():
        cond = [S for S in list_union(powerset(nbrs[x]), powerset(nbrs[z])) if (y in S) == with_mid]
        spans.append((len(tests), len(tests) + len(cond)))
        tests.extend((x, z, S) for S in cond)
        if len(tests) > MAX_UC_TESTS:
            raise NotImplementedError(f"uc_priority={priority}: more than {MAX_UC_TESTS} conditioning sets "
                                      "(neighbourhood power sets) — graph too dense")
    p = ci.pvalues(tests)
    score = [max(p[a:b]) for (a, b) in spans]
    order = sorted(range(len(score)), key=lambda q: score[q], reverse=with_mid)   # stable, like sorted(dict)
    if knowledge is not None:
        return orient_bk(adj, sep_xy, sep_bits, *knowledge, priority=priority, triples=R0, scores=score)
    return orient_triples(adj, R0[order] if len(order) else R0)


__all__ = ["CITester", "uc_orient", "powerset", "list_union", "MAX_UC_TESTS"]
