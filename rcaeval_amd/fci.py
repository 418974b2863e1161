"""FCI on the MI355X engine — ``fci(dataset, fisherz, alpha=0.05, ...)`` as RCAEval calls it.

Caller: ``RCAEval/graph_construction/fci.py:5-14`` (``fci_default``), used by
``RCAEval/e2e/fci_pagerank.py:7-20`` and ``RCAEval/e2e/pc_randomwalk.py:53-72``
(``fci_randomwalk``). The reference resolves ``fci`` to causal-learn 0.1.3.3 [U] (not on disk);
the on-disk spec restated here is the vendored copy ``lib/causallearn/search/ConstraintBased/
FCI.py:992-1180`` + ``lib/causallearn/utils/Fas.py:391-534`` — every place where 0.1.3.3 is
known or suspected to differ is **parity-unpinned** (DESIGN.md §2).

Pipeline (vendored semantics):

* FAS (``Fas.py:474-520``, ``searchAtDepth`` ``:134-259``): per depth, node i ascending tests
  (i, y | S) for every S of the depth-start adjacency of i (``adjacencies_completed``) and
  removes the edge at once (``:203-207``); y's own turn only sees the live adjacency, so a pair
  a < b is decided from a's side and, only if a found no independent S, from b's side. The
  removal set equals the stable PC skeleton's (same tests, same snapshot neighbourhoods, same
  ``freeDegree > depth`` stopping rule ``:259`` = ``max_degree - 1 > depth``), so FAS runs on
  the device level engine (``pcg_skeleton``). ``sep_sets`` keeps FAS's one-sided keys: depth 0
  → ``(a, b)`` = set() (``:124``); depth >= 1 → ``(a, b)`` = a's union if a's side found an
  independent S, else ``(b, a)`` = b's union (``:209-215``).
* Possible-D-Sep removal (``FCI.py:1095-1125``): in the vendored ``getPossibleDsep``
  (``:117-211``) the ``previous`` map is never written (``:139``/``:171`` are commented out),
  so Possible-D-Sep(x, y) = adj(x) minus y, and ``get_cond_set`` (``:227-282``) tests subsets
  of it by size. Every such subset of size <= the last FAS depth was already tested dependent
  by FAS from x's side (it is a subset of x's depth-start neighbourhood), and no node has more
  neighbours than that depth + 1 when FAS stops — so with the default ``depth=-1`` the step
  removes nothing and issues only cache hits. Only the sizes FAS did not reach (possible when
  ``depth`` caps FAS) are evaluated, on the device.
* ``rule0`` (``:349-406``), then ``rulesR1R2cycle`` (``:480-501``), ``ruleR3`` (``:509-564``,
  including its ``not adj(A, D) or adj(C, D)`` test and the one-sided ``sep_sets[(A, C)]``
  lookup, which raises ``KeyError`` like the reference), ``ruleR4B`` / ``ddpOrient`` /
  ``doDdpOrientation`` (``:579-841``; CI tests on the device through ``CITester``) until no
  rule changes the graph.

PAG encoding (causal-learn ``GeneralGraph.graph`` [U], ``FCI.py:1025-1028``):
``g[a, b]`` = the mark at a on edge a - b: TAIL -1, ARROW 1, CIRCLE 2; 0 = no edge.
"""
from __future__ import annotations

import time
import warnings
from collections import deque
from itertools import combinations

import numpy as np

from .causal import GeneralGraph, _check_supported, fisherz, skeleton_from_data
from .citest import CITester

TAIL, ARROW, CIRCLE = -1, 1, 2


class PAG:
    """Endpoint-mark matrix with the GeneralGraph queries the FCI rules use [U]."""

    def __init__(self, adj: np.ndarray):
        self.g = np.where(adj, CIRCLE, 0).astype(np.int64)
        self.n = adj.shape[0]

    def adjacent(self, a: int, b: int) -> bool:
        return self.g[a, b] != 0 and self.g[b, a] != 0

    def endpoint(self, x: int, y: int) -> int:
        """``get_endpoint(x, y)``: the mark at y on edge x - y (0 if none)."""
        return int(self.g[y, x]) if self.adjacent(x, y) else 0

    def set_edge(self, x: int, y: int, mark_x: int, mark_y: int) -> None:
        """``add_edge(Edge(x, y, mark_x, mark_y))`` after ``remove_edge``."""
        self.g[x, y] = mark_x
        self.g[y, x] = mark_y

    def adjacent_nodes(self, b: int) -> list:
        return [int(j) for j in np.flatnonzero((self.g[b] != 0) & (self.g[:, b] != 0))]

    def nodes_into(self, b: int, mark: int) -> list:
        """``get_nodes_into(b, mark)``: j with the mark at b on edge b - j."""
        return [int(j) for j in np.flatnonzero(self.g[b] == mark)]

    def nodes_out_of(self, b: int, mark: int) -> list:
        """``get_nodes_out_of(b, mark)``: j with the mark at j on edge b - j."""
        return [int(j) for j in np.flatnonzero(self.g[:, b] == mark)]

    def is_def_collider(self, a: int, b: int, c: int) -> bool:
        return (self.adjacent(a, b) and self.adjacent(b, c) and self.g[b, a] == ARROW
                and self.g[b, c] == ARROW)

    def is_parent_of(self, a: int, c: int) -> bool:
        """a --> c."""
        return self.g[a, c] == TAIL and self.g[c, a] == ARROW

    def parents(self, c: int) -> list:
        return [int(p) for p in np.flatnonzero((self.g[:, c] == TAIL) & (self.g[c, :] == ARROW))]

    def reorient_all(self, mark: int) -> None:
        self.g[self.g != 0] = mark


def is_arrow_point_allowed(G: PAG, x: int, y: int) -> bool:
    """``FCI.py:335-346`` without background knowledge."""
    e = G.endpoint(x, y)
    if e == ARROW:
        return True
    if e == TAIL:
        return False
    return e == CIRCLE


def rule0(G: PAG, sep_sets: dict) -> None:
    """``FCI.py:349-406``: unshielded colliders from the one-sided sep_sets keys."""
    G.reorient_all(CIRCLE)
    for b in range(G.n):
        adj = G.adjacent_nodes(b)
        if len(adj) < 2:
            continue
        for ia, ic in combinations(range(len(adj)), 2):
            a, c = adj[ia], adj[ic]
            if G.adjacent(a, c) or G.is_def_collider(a, b, c):
                continue
            sep = sep_sets.get((a, c))
            if sep is not None and b not in sep:
                if not is_arrow_point_allowed(G, a, b) or not is_arrow_point_allowed(G, c, b):
                    continue
                G.set_edge(a, b, G.g[a, b], ARROW)
                G.set_edge(c, b, G.g[c, b], ARROW)


def rule_r1(G: PAG, a: int, b: int, c: int, change: bool) -> bool:
    """``FCI.py:419-442``: a *-> b o-* c, a, c non-adjacent => b --> c."""
    if G.adjacent(a, c):
        return change
    if G.endpoint(a, b) == ARROW and G.endpoint(c, b) == CIRCLE:
        if not is_arrow_point_allowed(G, b, c):
            return change
        G.set_edge(c, b, ARROW, TAIL)
        change = True
    return change


def rule_r2(G: PAG, a: int, b: int, c: int, change: bool) -> bool:
    """``FCI.py:445-477``."""
    if G.adjacent(a, c) and G.endpoint(a, c) == CIRCLE:
        if (G.endpoint(a, b) == ARROW and G.endpoint(b, c) == ARROW
                and (G.endpoint(b, a) == TAIL or G.endpoint(c, b) == TAIL)):
            if not is_arrow_point_allowed(G, a, c):
                return change
            G.set_edge(a, c, G.g[a, c], ARROW)
            change = True
    return change


def rules_r1r2_cycle(G: PAG, change: bool) -> bool:
    """``FCI.py:480-501``: every pair (A, C) of B's neighbours, in place."""
    for b in range(G.n):
        adj = G.adjacent_nodes(b)
        if len(adj) < 2:
            continue
        for ia, ic in combinations(range(len(adj)), 2):
            a, c = adj[ia], adj[ic]
            change = rule_r1(G, a, b, c, change)
            change = rule_r1(G, c, b, a, change)
            change = rule_r2(G, a, b, c, change)
            change = rule_r2(G, c, b, a, change)
    return change


def rule_r3(G: PAG, sep_sets: dict, change: bool) -> bool:
    """``FCI.py:509-564`` (its adjacency test and one-sided sepset lookup kept as written)."""
    for b in range(G.n):
        into_arrows = G.nodes_into(b, ARROW)
        into_circles = G.nodes_into(b, CIRCLE)
        for d in into_circles:
            if len(into_arrows) < 2:
                continue
            for ia, ic in combinations(range(len(into_arrows)), 2):
                a, c = into_arrows[ia], into_arrows[ic]
                if G.adjacent(a, c):
                    continue
                if not G.adjacent(a, d) or G.adjacent(c, d):
                    continue
                sep = sep_sets[(a, c)]                       # isNoncollider :504-506 (KeyError as upstream)
                if not (sep is not None and d in sep):
                    continue
                if G.endpoint(a, d) != CIRCLE or G.endpoint(c, d) != CIRCLE:
                    continue
                if not is_arrow_point_allowed(G, d, b):
                    continue
                G.set_edge(d, b, G.g[d, b], ARROW)
                change = True
    return change


def _get_path(c: int, previous: dict) -> list:
    """``FCI.py:567-576``."""
    out = []
    p = previous[c]
    if p is not None:
        out.append(p)
    while p is not None:
        p = previous.get(p)
        if p is not None:
            out.append(p)
    return out


def _ddp_orientation(G: PAG, d: int, a: int, b: int, c: int, previous: dict, ci: CITester, alpha: float,
                     sep_sets: dict, change: bool):
    """``FCI.py:579-717``."""
    if G.adjacent(d, c):
        raise Exception("illegal argument!")
    path = _get_path(d, previous)
    ind = ci(d, c, tuple(path)) > alpha
    path2 = list(path)
    path2.remove(b)
    ind2 = ci(d, c, tuple(path2)) > alpha
    if not ind and not ind2:
        sep = sep_sets.get((d, c))
        if sep is None:
            return False, change
        ind = b in sep
    if ind:
        G.set_edge(c, b, G.g[c, b], TAIL)
        return True, True
    if not is_arrow_point_allowed(G, a, b) or not is_arrow_point_allowed(G, c, b):
        return False, change
    G.set_edge(a, b, G.g[a, b], ARROW)
    G.set_edge(c, b, G.g[c, b], ARROW)
    return True, True


def _ddp_orient(G: PAG, a: int, b: int, c: int, max_path_length: int, ci: CITester, alpha: float,
                sep_sets: dict, change: bool) -> bool:
    """``FCI.py:720-797``: breadth-first search for a discriminating path for b."""
    Q = deque([a])
    V = {a, b}
    e = None
    distance = 0
    previous = {a: b}
    c_parents = set(G.parents(c))
    bound = 1000 if max_path_length == -1 else max_path_length
    while Q:
        t = Q.popleft()
        if e is None or e == t:
            e = t
            distance += 1
            if distance > 0 and distance > bound:
                return change
        for d in G.nodes_into(t, ARROW):
            if d in V:
                continue
            previous[d] = t
            p = previous[t]
            if not G.is_def_collider(d, t, p):
                continue
            previous[d] = t
            if not G.adjacent(d, c) and d != c:
                res, change = _ddp_orientation(G, d, a, b, c, previous, ci, alpha, sep_sets, change)
                if res:
                    return change
            if d in c_parents:
                Q.append(d)
                V.add(d)
    return change


def rule_r4b(G: PAG, max_path_length: int, ci: CITester, alpha: float, sep_sets: dict, change: bool) -> bool:
    """``FCI.py:800-841``."""
    for b in range(G.n):
        poss_a = G.nodes_out_of(b, ARROW)
        poss_c = G.nodes_into(b, CIRCLE)
        for a in poss_a:
            for c in poss_c:
                if not G.is_parent_of(a, c):
                    continue
                if G.endpoint(b, c) != ARROW:
                    continue
                change = _ddp_orient(G, a, b, c, max_path_length, ci, alpha, sep_sets, change)
    return change


def fas_sep_sets(out) -> dict:
    """FAS's one-sided ``sep_sets`` from the device skeleton (see the module docstring)."""
    rl = out.removed_level
    sides = {}
    for (x, y), bits in zip(out.sep_xy.tolist(), out.sep_bits):
        mem = set()
        for w, v in enumerate(bits.tolist()):
            v = int(v)
            while v:
                low = v & -v
                mem.add(w * 64 + low.bit_length() - 1)
                v ^= low
        sides.setdefault((int(x), int(y)), set()).update(mem)
    sep_sets = {}
    for a, b in zip(*np.nonzero(np.triu(rl >= 0, 1))):
        a, b = int(a), int(b)
        if rl[a, b] == 0:
            sep_sets[(a, b)] = set()
        elif (a, b) in sides:
            sep_sets[(a, b)] = sides[(a, b)]
        else:
            sep_sets[(b, a)] = sides.get((b, a), set())
    return sep_sets


def _cond_set(G: PAG, u: int, v: int, ci: CITester, alpha: float, depth: int, fas_last: int):
    """``SepsetsPossibleDsep.get_cond_set`` (``FCI.py:227-282``) with Possible-D-Sep(u, v) =
    adj(u) minus v (the vendored ``getPossibleDsep``, module docstring). Sizes <= the last FAS
    depth were all tested dependent by FAS from u's side (cache hits in the reference) and are
    skipped; larger sizes (only reachable when ``depth`` capped FAS) go to the device."""
    pd = [w for w in G.adjacent_nodes(u) if w != v]
    top = min(1000 if depth == -1 else depth, len(pd))
    for s in range(0, top + 1):
        if s <= fas_last:
            continue
        subsets = list(combinations(pd, s))
        p = ci.pvalues([(u, v, S) for S in subsets])
        hit = [S for S, pv in zip(subsets, p) if pv > alpha]
        if hit:
            return set(w for S in hit for w in S)
    return None


def possible_dsep_removal(G: PAG, sep_sets: dict, ci: CITester, alpha: float, depth: int, fas_last: int) -> None:
    """``FCI.py:1109-1125``: edges in ``get_graph_edges`` order (i < j), removals deferred."""
    waiting = []
    for x in range(G.n):
        for y in range(x + 1, G.n):
            if not G.adjacent(x, y):
                continue
            sep = _cond_set(G, x, y, ci, alpha, depth, fas_last)
            if sep is None:
                sep = _cond_set(G, y, x, ci, alpha, depth, fas_last)
            if sep is not None:
                waiting.append((x, y, sep))
    for x, y, sep in waiting:
        G.g[x, y] = G.g[y, x] = 0
        sep_sets[(x, y)] = sep


def fci_orient(adj: np.ndarray, sep_sets: dict, ci: CITester, alpha: float = 0.05, depth: int = -1,
               max_path_length: int = -1, fas_last: int = 1 << 30) -> np.ndarray:
    """FCI after FAS (``FCI.py:1087-1176``): rule0, Possible-D-Sep removal, rule0, then R1-R3 and
    R4B until nothing changes; returns the PAG matrix. ``sep_sets`` is updated in place."""
    G = PAG(adj)
    rule0(G, sep_sets)
    possible_dsep_removal(G, sep_sets, ci, alpha, depth, fas_last)
    G.reorient_all(CIRCLE)
    rule0(G, sep_sets)
    change = True
    while change:
        change = False
        change = rules_r1r2_cycle(G, change)
        change = rule_r3(G, sep_sets, change)
        if change:
            change = rule_r4b(G, max_path_length, ci, alpha, sep_sets, change)
    return G.g


class FciGraph(GeneralGraph):
    """``fci(...)[0]``: the PAG (``.graph``) with the FAS ``sep_sets`` kept for inspection."""

    def __init__(self, graph, names, sep_sets):
        super().__init__(graph, names)
        self.sep_sets = sep_sets
        self.pag = True


def fci(dataset: np.ndarray, independence_test_method=fisherz, alpha: float = 0.05, depth: int = -1,
        max_path_length: int = -1, verbose: bool = False, background_knowledge=None, node_names=None,
        device: int | None = None, **kwargs):
    """``fci`` (``FCI.py:992-1180``) with fisherz on the GPU; returns ``(graph, edges)``."""
    if dataset.shape[0] < dataset.shape[1]:
        warnings.warn("The number of features is much larger than the sample size!")
    if depth is None or type(depth) != int:
        raise TypeError("'depth' must be 'int' type!")
    if max_path_length is not None and type(max_path_length) != int:
        raise TypeError("'max_path_length' must be 'int' type!")
    _check_supported(independence_test_method, True, 0, 2, False, background_knowledge)
    X = np.asarray(dataset, dtype=np.float64)
    assert not np.isnan(X).any(), "Input data contains NaN. Please check."
    assert not np.isinf(X).any(), "Input data contains Inf. Please check."
    n = X.shape[1]
    names = node_names if node_names is not None else [f"X{i + 1}" for i in range(n)]
    t0 = time.time()
    if n < 2:
        g = np.zeros((n, n), int)
        return FciGraph(g, names, {}), []
    # FAS runs depths 0 .. depth-1 (Fas.py:449-450,474: range(depth), -1 -> 1000); with depth 0
    # it runs none, and since depth 0 is where adjacencies are first added (:126-128) the
    # skeleton is empty
    if depth == 0:
        from .engine import get_engine
        C = get_engine(device).corr(X)
        adj = np.zeros((n, n), dtype=bool)
        sep_sets, fas_last = {}, -1
    else:
        out, C = skeleton_from_data(X, alpha=alpha, max_depth=depth - 1 if depth > 0 else -1, device=device)
        adj, sep_sets, fas_last = out.adj, fas_sep_sets(out), out.levels - 1
    ci = CITester(C, X.shape[0], device=device)
    g = fci_orient(adj, sep_sets, ci, alpha=alpha, depth=depth, max_path_length=max_path_length, fas_last=fas_last)
    G = FciGraph(g.astype(int), names, sep_sets)
    G.elapsed = time.time() - t0
    return G, []


__all__ = ["fci", "fci_orient", "fas_sep_sets", "PAG", "TAIL", "ARROW", "CIRCLE"]
