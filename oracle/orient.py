"""Orientation oracle — UCSepset(priority 2/3/4) + Meek [U], literal restatement (tests only).

Follows the vendored enumerations in ``lib/causallearn/graph/GraphClass.py``:
``find_tails``/``find_arrow_heads`` (:108-116), ``find_adj`` (:145-147),
``find_unshielded_triples`` (:157-165), ``find_triangles`` (:167-176), ``find_kites``
(:178-188) — computed with ``itertools.permutations`` exactly as written there — and the
causal-learn 0.1.3.3 GeneralGraph edge semantics [U] (add_edge no-op on an existing edge,
dpath ancestry via adjust_dpath / reconstitute_dpath on removal of a directed edge).
Quadratic in the number of edges: small graphs only. The C++ ``pcg_orient`` is checked
against this.

Background knowledge [U] (``knowledge=(forbidden, required)`` n x n masks, [i, j] = rule for
i -> j): ``orient_by_background_knowledge`` over ``get_graph_edges`` before uc_sepset, the
collider skip (x->y or z->y forbidden, y->x or y->z required) in every priority, and the
per-rule skip in Meek (orienting a->b forbidden, or b->a required), as causal-learn 0.1.3.3
publishes them (PC.py / BackGroundKnowledgeOrientUtils.py / UCSepset.py / Meek.py, not vendored).
"""
from __future__ import annotations

from itertools import chain, combinations, permutations

import numpy as np


class _G:
    def __init__(self, graph: np.ndarray):
        self.graph = graph.astype(int).copy()
        n = len(graph)
        self.n = n
        self.dpath = np.zeros((n, n), int)
        for i in range(n):
            self.adjust_dpath(i, i)

    def adjust_dpath(self, i, j):
        dp = self.dpath
        dp[j, i] = 1
        for k in range(self.n):
            if dp[i, k] == 1:
                dp[j, k] = 1
            if dp[k, j] == 1:
                dp[k, i] = 1

    def get_graph_edges(self):
        edges = []
        g = self.graph
        for i in range(self.n):
            for j in range(i + 1, self.n):
                if g[i, j] == 0 and g[j, i] == 0:
                    continue
                if g[i, j] == 1 and g[j, i] == -1:   # i <- j : Edge normalised j -> i
                    edges.append((j, i))
                else:
                    edges.append((i, j))
        return edges

    def reconstitute_dpath(self):
        for i in range(self.n):
            self.adjust_dpath(i, i)
        edges = self.get_graph_edges()
        while edges:
            i, j = edges.pop()
            self.adjust_dpath(i, j)

    def is_fully_directed(self, i, j):
        return self.graph[i, j] == -1 and self.graph[j, i] == 1

    def is_undirected(self, i, j):
        return self.graph[i, j] == -1 and self.graph[j, i] == -1

    def is_ancestor_of(self, a, b):
        return self.dpath[b, a] == 1

    def remove_edge(self, i, j):
        directed = self.is_fully_directed(i, j) or self.is_fully_directed(j, i)
        self.graph[i, j] = self.graph[j, i] = 0
        if directed:
            self.reconstitute_dpath()

    def add_directed(self, i, j):
        e1, e2 = self.graph[i, j], self.graph[j, i]
        bidirected = e1 == 1 and e2 == 1
        if (not bidirected and (e1 != 0 or e2 != 0)) or bidirected:
            return
        self.graph[j, i] = 1
        self.graph[i, j] = -1
        self.adjust_dpath(i, j)

    # GraphClass.py enumerations
    def find_adj(self):
        T = np.where(self.graph == -1)
        A = np.where(self.graph == 1)
        return list(zip(T[1], T[0])) + list(zip(A[1], A[0]))

    def find_unshielded_triples(self):
        return [(p[0][0], p[0][1], p[1][1]) for p in permutations(self.find_adj(), 2)
                if p[0][1] == p[1][0] and p[0][0] != p[1][1] and self.graph[p[0][0], p[1][1]] == 0]

    def find_triangles(self):
        Adj = self.find_adj()
        return [(p[0][0], p[0][1], p[1][1]) for p in permutations(Adj, 2)
                if p[0][1] == p[1][0] and p[0][0] != p[1][1] and (p[0][0], p[1][1]) in Adj]

    def find_kites(self):
        return [(p[0][0], p[0][1], p[1][1], p[0][2]) for p in permutations(self.find_triangles(), 2)
                if p[0][0] == p[1][0] and p[0][2] == p[1][2] and p[0][1] < p[1][1]
                and self.graph[p[0][1], p[1][1]] == 0]


class _NoKnowledge:
    def forbidden(self, i, j):
        return False

    def required(self, i, j):
        return False


class _Knowledge:
    def __init__(self, forbidden, required):
        self.F, self.R = np.asarray(forbidden, bool), np.asarray(required, bool)

    def forbidden(self, i, j):
        return bool(self.F[i, j])

    def required(self, i, j):
        return bool(self.R[i, j])


def orient_by_background_knowledge(G: _G, bk) -> None:
    for (a, b) in G.get_graph_edges():
        if not G.is_undirected(a, b):
            continue
        if bk.forbidden(b, a):
            G.remove_edge(a, b)
            G.add_directed(a, b)
        elif bk.forbidden(a, b):
            G.remove_edge(a, b)
            G.add_directed(b, a)
        elif bk.required(b, a):
            G.remove_edge(a, b)
            G.add_directed(b, a)
        elif bk.required(a, b):
            G.remove_edge(a, b)
            G.add_directed(a, b)


def _collider_blocked(bk, x, y, z):
    return bk.forbidden(x, y) or bk.forbidden(z, y) or bk.required(y, x) or bk.required(y, z)


def uc_sepset_priority2(G: _G, sepset_has, bk=_NoKnowledge()) -> None:
    UT = [(i, j, k) for (i, j, k) in G.find_unshielded_triples() if i < k]
    for (x, y, z) in UT:
        if sepset_has(x, z, y):
            continue
        if _collider_blocked(bk, x, y, z):
            continue
        if (not G.is_fully_directed(y, x)) and (not G.is_fully_directed(y, z)):
            if G.graph[x, y] != 0:
                G.remove_edge(x, y)
            G.add_directed(x, y)
            if G.graph[z, y] != 0:
                G.remove_edge(z, y)
            G.add_directed(z, y)


def powerset(L):
    """causal-learn ``PCUtils.Helper.powerset`` [U]: all subsets, by size, combinations order."""
    s = list(L)
    return list(chain.from_iterable(combinations(s, r) for r in range(len(s) + 1)))


def list_union(L1, L2):
    """``Helper.list_union`` [U]: L1 followed by the members of L2 not in L1."""
    return L1 + [x for x in L2 if x not in L1]


def find_cond_sets(G: _G, i, j):
    """``GraphClass.find_cond_sets`` (:190-196): power sets of both neighbourhoods."""
    ni = np.where(G.graph[i, :] != 0)[0]
    nj = np.where(G.graph[j, :] != 0)[0]
    return list_union(powerset(ni), powerset(nj))


def uc_sepset_priority34(G: _G, sepset_has, ci_test, priority: int, bk=_NoKnowledge()) -> None:
    """uc_sepset(priority=3 | 4) [U]: R0 = candidates in UT order; score each by the max
    p-value of ``ci_test(x, z, S)`` over ``find_cond_sets_without_mid`` (3) or
    ``_with_mid`` (4) (GraphClass.py:198-204); stable sort ascending (3) / descending (4);
    then the collider step in that order."""
    UT = [(i, j, k) for (i, j, k) in G.find_unshielded_triples() if i < k]
    R0 = [(x, y, z) for (x, y, z) in UT if not sepset_has(x, z, y)]
    UC = {}
    for (x, y, z) in R0:
        cond = [S for S in find_cond_sets(G, x, z) if (y in S) == (priority == 4)]
        UC[(x, y, z)] = max([ci_test(x, z, S) for S in cond])
    UC = dict(sorted(UC.items(), key=lambda item: item[1], reverse=(priority == 4)))
    for (x, y, z) in UC.keys():
        if _collider_blocked(bk, x, y, z):
            continue
        if (not G.is_fully_directed(y, x)) and (not G.is_fully_directed(y, z)):
            if G.graph[x, y] != 0:
                G.remove_edge(x, y)
            G.add_directed(x, y)
            if G.graph[z, y] != 0:
                G.remove_edge(z, y)
            G.add_directed(z, y)


def meek(G: _G, bk=_NoKnowledge()) -> None:
    UT, Tri, Kite = G.find_unshielded_triples(), G.find_triangles(), G.find_kites()
    loop = True
    while loop:
        loop = False
        for (i, j, k) in UT:
            if G.is_fully_directed(i, j) and G.is_undirected(j, k):
                if bk.forbidden(j, k) or bk.required(k, j):
                    continue
                if G.is_ancestor_of(k, j):
                    continue
                G.remove_edge(j, k)
                G.add_directed(j, k)
                loop = True
        for (i, j, k) in Tri:
            if G.is_fully_directed(i, j) and G.is_fully_directed(j, k) and G.is_undirected(i, k):
                if bk.forbidden(i, k) or bk.required(k, i):
                    continue
                if G.is_ancestor_of(k, i):
                    continue
                G.remove_edge(i, k)
                G.add_directed(i, k)
                loop = True
        for (i, j, k, l) in Kite:
            if (G.is_undirected(i, j) and G.is_undirected(i, k) and G.is_fully_directed(j, l)
                    and G.is_fully_directed(k, l) and G.is_undirected(i, l)):
                if bk.forbidden(i, l) or bk.required(l, i):
                    continue
                if G.is_ancestor_of(l, i):
                    continue
                G.remove_edge(i, l)
                G.add_directed(i, l)
                loop = True


def orient(skeleton_adj: np.ndarray, sepset, priority: int = 2, ci_test=None, knowledge=None) -> np.ndarray:
    """``sepset``: n x n object array of lists of tuples (reference layout);
    ``ci_test(x, z, S) -> p`` is needed for priority 3 / 4; ``knowledge=(forbidden, required)``."""
    G = _G(np.where(skeleton_adj, -1, 0))
    bk = _NoKnowledge() if knowledge is None else _Knowledge(*knowledge)

    def has(x, z, y):
        return not all(y not in S for S in sepset[x, z])

    # uc_sepset's candidate list comes from its deepcopy of the graph after the background
    # orientation; the triples depend on adjacency only, which that orientation keeps
    if knowledge is not None:
        orient_by_background_knowledge(G, bk)
    if priority == 2:
        uc_sepset_priority2(G, has, bk)
    else:
        uc_sepset_priority34(G, has, ci_test, priority, bk)
    meek(G, bk)
    return G.graph
