"""FCI (vendored causal-learn) — CPU oracle, TEST INFRASTRUCTURE ONLY (parity unpinned).

A literal, object-style restatement of the on-disk spec, for checking ``rcaeval_amd.fci``:

* ``fas``: ``lib/causallearn/utils/Fas.py:391-534`` with ``searchAtDepth0`` (``:55-131``) and
  the stable ``searchAtDepth`` (``:134-259``): adjacencies are sets of node objects, removal is
  immediate, conditioning sets come from the depth-start copy, ``sep_sets`` keys are
  ``(processing node, y)``.
* ``fci``: ``lib/causallearn/search/ConstraintBased/FCI.py:992-1180`` with ``rule0`` (``:349``),
  ``SepsetsPossibleDsep`` (``:14-288``, including the BFS whose ``previous`` map is never
  written), ``rulesR1R2cycle`` (``:480``), ``ruleR3`` (``:509``), ``ruleR4B`` / ``ddpOrient`` /
  ``doDdpOrientation`` (``:579-841``).
* ``GeneralGraph`` / ``Edge`` semantics [U] (causal-learn is not on disk): ``graph[i, j]`` is
  the mark at i of edge i - j (TAIL -1, ARROW 1, CIRCLE 2), ``get_endpoint(a, b)`` the mark at
  b, node lists in index order.

The CI test is ``oracle.fisherz.pvalue`` (numpy/scipy restatement of FisherZ [U]) behind the
module-level cache of ``Fas.py:10`` keyed like ``:164-170``. causal-learn 0.1.3.3 (what the
reference imports) is not on disk, so nothing here is pinned by reference outputs.
"""
from __future__ import annotations

from collections import deque
from itertools import combinations

import numpy as np

from . import fisherz as fz

TAIL, ARROW, CIRCLE = -1, 1, 2


class Node:
    def __init__(self, name: str, idx: int):
        self.name, self.idx = name, idx

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, Node) and other.name == self.name

    def __repr__(self):
        return self.name


class Edge:
    def __init__(self, node1, node2, end1, end2):
        self.node1, self.node2, self.end1, self.end2 = node1, node2, end1, end2

    def get_proximal_endpoint(self, node):
        return self.end1 if node == self.node1 else self.end2


class Graph:
    def __init__(self, nodes):
        self.nodes = list(nodes)
        self.node_map = {nd: i for i, nd in enumerate(self.nodes)}
        self.graph = np.zeros((len(nodes), len(nodes)), int)

    def add_edge(self, e: Edge):
        i, j = self.node_map[e.node1], self.node_map[e.node2]
        self.graph[i, j] = e.end1
        self.graph[j, i] = e.end2

    def remove_edge(self, e: Edge):
        i, j = self.node_map[e.node1], self.node_map[e.node2]
        self.graph[i, j] = self.graph[j, i] = 0

    def get_edge(self, a, b):
        i, j = self.node_map[a], self.node_map[b]
        if self.graph[i, j] == 0 or self.graph[j, i] == 0:
            return None
        return Edge(a, b, int(self.graph[i, j]), int(self.graph[j, i]))

    def get_endpoint(self, a, b):
        e = self.get_edge(a, b)
        return e.get_proximal_endpoint(b) if e else None

    def is_adjacent_to(self, a, b):
        return self.get_edge(a, b) is not None

    def get_adjacent_nodes(self, a):
        i = self.node_map[a]
        return [self.nodes[j] for j in range(len(self.nodes)) if self.graph[i, j] != 0 and self.graph[j, i] != 0]

    def get_nodes_into(self, a, endpoint):
        i = self.node_map[a]
        return [self.nodes[j] for j in range(len(self.nodes)) if self.graph[i, j] == endpoint]

    def get_nodes_out_of(self, a, endpoint):
        i = self.node_map[a]
        return [self.nodes[j] for j in range(len(self.nodes)) if self.graph[j, i] == endpoint]

    def is_def_collider(self, a, b, c):
        e1, e2 = self.get_edge(a, b), self.get_edge(b, c)
        if e1 is None or e2 is None:
            return False
        return e1.get_proximal_endpoint(b) == ARROW and e2.get_proximal_endpoint(b) == ARROW

    def is_parent_of(self, a, b):
        i, j = self.node_map[a], self.node_map[b]
        return self.graph[j, i] == ARROW and self.graph[i, j] == TAIL

    def get_parents(self, a):
        return [p for p in self.nodes if self.is_parent_of(p, a)]

    def get_graph_edges(self):
        out = []
        for i in range(len(self.nodes)):
            for j in range(i + 1, len(self.nodes)):
                if self.graph[i, j] != 0:
                    out.append(self.get_edge(self.nodes[i], self.nodes[j]))
        return out

    def get_nodes(self):
        return self.nodes


class CITest:
    """Module-level cache of Fas.py:10 in front of the FisherZ restatement."""

    def __init__(self, C, N):
        self.C, self.N, self.cache = C, N, {}

    def __call__(self, X, Y, cond):
        X, Y = (X, Y) if X < Y else (Y, X)
        key = (X, Y, frozenset(cond))
        if key not in self.cache:
            self.cache[key] = fz.pvalue(self.C, self.N, X, Y, tuple(sorted(cond)))
        return self.cache[key]


def _free_degree(nodes, adjacencies):
    mx = 0
    for x in nodes:
        for y in adjacencies[x]:
            mx = max(mx, len(adjacencies[x]) - 1)
    return mx


def fas(nodes, ci: CITest, alpha=0.05, depth=-1):
    """``Fas.py:391-534`` (knowledge None, stable)."""
    sep_sets = {}
    adjacencies = {nd: set() for nd in nodes}
    if depth is None or depth < 0:
        depth = 1000
    for d in range(depth):
        if d == 0:
            for i in range(len(nodes)):
                for j in range(i + 1, len(nodes)):
                    if ci(i, j, ()) > alpha:
                        sep_sets[(i, j)] = set()
                    else:
                        adjacencies[nodes[i]].add(nodes[j])
                        adjacencies[nodes[j]].add(nodes[i])
            more = _free_degree(nodes, adjacencies) > 0
        else:
            completed = {k: set(v) for k, v in adjacencies.items()}

            def edge(adjx, i):
                for node_y in adjx:
                    _adjx = list(completed[nodes[i]])
                    _adjx.remove(node_y)
                    if len(_adjx) >= d:
                        flag = False
                        for choice in combinations(range(len(_adjx)), d):
                            cond = [_adjx[k].idx for k in choice]
                            if ci(i, node_y.idx, cond) > alpha:
                                adjacencies[nodes[i]].discard(node_y)
                                adjacencies[node_y].discard(nodes[i])
                                key = (i, node_y.idx)
                                if key in sep_sets:
                                    sep_sets[key].update(cond)
                                else:
                                    sep_sets[key] = set(cond)
                                flag = True
                        if flag:
                            return False
                return True

            for i in range(len(nodes)):
                adjx = list(adjacencies[nodes[i]])
                while not edge(adjx, i):
                    adjx = list(adjacencies[nodes[i]])
            more = _free_degree(nodes, adjacencies) > d
        if not more:
            break
    g = Graph(nodes)
    for i in range(len(nodes)):
        for j in range(i + 1, len(nodes)):
            if nodes[j] in adjacencies[nodes[i]]:
                g.add_edge(Edge(nodes[i], nodes[j], TAIL, TAIL))
    return g, sep_sets


def _allowed(x, y, g):
    """``is_arrow_point_allowed`` (``FCI.py:335-346``), knowledge None."""
    if g.get_endpoint(x, y) == ARROW:
        return True
    if g.get_endpoint(x, y) == TAIL:
        return False
    return g.get_endpoint(x, y) == CIRCLE


def _reorient_all(g, endpoint):
    for e in g.get_graph_edges():
        g.remove_edge(e)
        e.end1 = e.end2 = endpoint
        g.add_edge(e)


def rule0(g, nodes, sep_sets):
    _reorient_all(g, CIRCLE)
    for b in nodes:
        adj = g.get_adjacent_nodes(b)
        if len(adj) < 2:
            continue
        for ia, ic in combinations(range(len(adj)), 2):
            a, c = adj[ia], adj[ic]
            if g.is_adjacent_to(a, c) or g.is_def_collider(a, b, c):
                continue
            sep = sep_sets.get((g.node_map[a], g.node_map[c]))
            if sep is not None and g.node_map[b] not in sep:
                if not _allowed(a, b, g) or not _allowed(c, b, g):
                    continue
                e1 = g.get_edge(a, b)
                g.remove_edge(e1)
                g.add_edge(Edge(a, b, e1.get_proximal_endpoint(a), ARROW))
                e2 = g.get_edge(c, b)
                g.remove_edge(e2)
                g.add_edge(Edge(c, b, e2.get_proximal_endpoint(c), ARROW))


def _r1(a, b, c, g, flag):
    if g.is_adjacent_to(a, c):
        return flag
    if g.get_endpoint(a, b) == ARROW and g.get_endpoint(c, b) == CIRCLE:
        if not _allowed(b, c, g):
            return flag
        e = g.get_edge(c, b)
        g.remove_edge(e)
        g.add_edge(Edge(c, b, ARROW, TAIL))
        flag = True
    return flag


def _r2(a, b, c, g, flag):
    if g.is_adjacent_to(a, c) and g.get_endpoint(a, c) == CIRCLE:
        if (g.get_endpoint(a, b) == ARROW and g.get_endpoint(b, c) == ARROW
                and (g.get_endpoint(b, a) == TAIL or g.get_endpoint(c, b) == TAIL)):
            if not _allowed(a, c, g):
                return flag
            e = g.get_edge(a, c)
            g.remove_edge(e)
            g.add_edge(Edge(a, c, e.get_proximal_endpoint(a), ARROW))
            flag = True
    return flag


def rules_r1r2(g, flag):
    for b in g.get_nodes():
        adj = g.get_adjacent_nodes(b)
        if len(adj) < 2:
            continue
        for ia, ic in combinations(range(len(adj)), 2):
            a, c = adj[ia], adj[ic]
            flag = _r1(a, b, c, g, flag)
            flag = _r1(c, b, a, g, flag)
            flag = _r2(a, b, c, g, flag)
            flag = _r2(c, b, a, g, flag)
    return flag


def rule_r3(g, sep_sets, flag):
    for b in g.get_nodes():
        arrows = g.get_nodes_into(b, ARROW)
        circles = g.get_nodes_into(b, CIRCLE)
        for d in circles:
            if len(arrows) < 2:
                continue
            for ia, ic in combinations(range(len(arrows)), 2):
                a, c = arrows[ia], arrows[ic]
                if g.is_adjacent_to(a, c):
                    continue
                if not g.is_adjacent_to(a, d) or g.is_adjacent_to(c, d):
                    continue
                sep = sep_sets[(g.node_map[a], g.node_map[c])]
                if not (sep is not None and g.node_map[d] in sep):
                    continue
                if g.get_endpoint(a, d) != CIRCLE or g.get_endpoint(c, d) != CIRCLE:
                    continue
                if not _allowed(d, b, g):
                    continue
                e = g.get_edge(d, b)
                g.remove_edge(e)
                g.add_edge(Edge(d, b, e.get_proximal_endpoint(d), ARROW))
                flag = True
    return flag


def _get_path(c, previous):
    out = []
    p = previous[c]
    if p is not None:
        out.append(p)
    while p is not None:
        p = previous.get(p)
        if p is not None:
            out.append(p)
    return out


def _do_ddp(d, a, b, c, previous, g, ci, alpha, sep_sets, flag):
    if g.is_adjacent_to(d, c):
        raise Exception("illegal argument!")
    path = _get_path(d, previous)
    ind = ci(g.node_map[d], g.node_map[c], [g.node_map[x] for x in path]) > alpha
    path2 = list(path)
    path2.remove(b)
    ind2 = ci(g.node_map[d], g.node_map[c], [g.node_map[x] for x in path2]) > alpha
    if not ind and not ind2:
        sep = sep_sets.get((g.node_map[d], g.node_map[c]))
        if sep is None:
            return False, flag
        ind = g.node_map[b] in sep
    if ind:
        e = g.get_edge(c, b)
        g.remove_edge(e)
        g.add_edge(Edge(c, b, e.get_proximal_endpoint(c), TAIL))
        return True, True
    if not _allowed(a, b, g) or not _allowed(c, b, g):
        return False, flag
    e1 = g.get_edge(a, b)
    g.remove_edge(e1)
    g.add_edge(Edge(a, b, e1.get_proximal_endpoint(a), ARROW))
    e2 = g.get_edge(c, b)
    g.remove_edge(e2)
    g.add_edge(Edge(c, b, e2.get_proximal_endpoint(c), ARROW))
    return True, True


def _ddp_orient(a, b, c, g, max_path_length, ci, alpha, sep_sets, flag):
    Q = deque([a])
    V = {a, b}
    e = None
    distance = 0
    previous = {a: b}
    c_parents = g.get_parents(c)
    while Q:
        t = Q.popleft()
        if e is None or e == t:
            e = t
            distance += 1
            if distance > 0 and distance > (1000 if max_path_length == -1 else max_path_length):
                return flag
        for d in g.get_nodes_into(t, ARROW):
            if d in V:
                continue
            previous[d] = t
            p = previous[t]
            if not g.is_def_collider(d, t, p):
                continue
            previous[d] = t
            if not g.is_adjacent_to(d, c) and d != c:
                res, flag = _do_ddp(d, a, b, c, previous, g, ci, alpha, sep_sets, flag)
                if res:
                    return flag
            if d in c_parents:
                Q.append(d)
                V.add(d)
    return flag


def rule_r4b(g, max_path_length, ci, alpha, sep_sets, flag):
    for b in g.get_nodes():
        for a in g.get_nodes_out_of(b, ARROW):
            for c in g.get_nodes_into(b, CIRCLE):
                if not g.is_parent_of(a, c):
                    continue
                if g.get_endpoint(b, c) != ARROW:
                    continue
                flag = _ddp_orient(a, b, c, g, max_path_length, ci, alpha, sep_sets, flag)
    return flag


def _possible_dsep(g, x, y):
    """``getPossibleDsep`` (``FCI.py:117-211``) with its BFS; ``previous`` stays {x: None}."""
    dsep = set()
    Q = deque()
    V = set()
    previous = {x: None}
    for b in g.get_adjacent_nodes(x):
        if b == y:
            continue
        Q.append((x, b))
        V.add((x, b))
        dsep.add(b)
    while Q:
        a, b = Q.popleft()
        if b == x:                               # existOnePathWithPossibleParents(previous, b, x, ...)
            dsep.add(b)
        elif previous.get(b) is not None:        # never: previous holds only x
            dsep.add(b)
        for c in g.get_adjacent_nodes(b):
            if c in (a, x, y):
                continue
            e1, e2 = g.get_edge(a, b), g.get_edge(b, c)
            coll = (e1 is not None and e2 is not None and e1.get_proximal_endpoint(b) == ARROW
                    and e2.get_proximal_endpoint(b) == ARROW)
            if coll or g.is_adjacent_to(a, c):
                u = (a, c)
                if u in V:
                    continue
                V.add(u)
                Q.append(u)
    dsep.discard(x)
    dsep.discard(y)
    return dsep


def _get_cond_set(g, n1, n2, ci, alpha, depth):
    pd = list(_possible_dsep(g, n1, n2))
    top = 1000 if depth == -1 else depth
    for d in range(1 + min(top, len(pd))):
        union, flag = set(), False
        for choice in combinations(range(len(pd)), d):
            cond = [g.node_map[pd[k]] for k in choice]
            if ci(g.node_map[n1], g.node_map[n2], cond) > alpha:
                union.update(cond)
                flag = True
        if flag:
            return union
    return None


def fci(C: np.ndarray, N: int, alpha=0.05, depth=-1, max_path_length=-1):
    """``FCI.py:992-1180`` on a correlation matrix; returns (PAG matrix, sep_sets, ci)."""
    n = C.shape[0]
    nodes = [Node(f"X{i + 1}", i) for i in range(n)]
    ci = CITest(C, N)
    g, sep_sets = fas(nodes, ci, alpha=alpha, depth=depth)
    _reorient_all(g, CIRCLE)
    rule0(g, nodes, sep_sets)
    waiting = []
    for e in g.get_graph_edges():
        x, y = e.node1, e.node2
        sep = _get_cond_set(g, x, y, ci, alpha, depth)
        if sep is None:
            sep = _get_cond_set(g, y, x, ci, alpha, depth)
        if sep is not None:
            waiting.append((x, y, sep))
    for x, y, sep in waiting:
        g.remove_edge(g.get_edge(x, y))
        sep_sets[(g.node_map[x], g.node_map[y])] = sep
    _reorient_all(g, CIRCLE)
    rule0(g, nodes, sep_sets)
    flag = True
    while flag:
        flag = False
        flag = rules_r1r2(g, flag)
        flag = rule_r3(g, sep_sets, flag)
        if flag:
            flag = rule_r4b(g, max_path_length, ci, alpha, sep_sets, flag)
    return g.graph.copy(), sep_sets, ci
