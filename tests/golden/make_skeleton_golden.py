"""Golden vectors for the PC skeleton loop and for FCI, produced by EXECUTING the reference's own
vendored causal-learn code.

MANUAL, SANDBOXED STEP. This script loads and runs Python files from /root/reference (untrusted
public content) as modules, so it is kept out of every automated path: no test, build, smoke or
bench imports or runs it (the tests import the case definitions from ``skeleton_cases.py``), and
the committed ``skeleton_ref.json`` is the only artefact they read. A maintainer regenerates the
goldens by hand, in a throwaway container with no credentials and no network:

  python tests/golden/make_skeleton_golden.py

What runs is the reference text itself, loaded from /root/reference as modules:

* ``lib/causallearn/graph/GraphClass.py`` (``CausalGraph``: complete start graph, ``ci_test``
  memo, ``neighbors``, ``max_degree``, ``find_unshielded_triples`` / ``find_triangles`` /
  ``find_kites``);
* ``lib/causallearn/utils/PCUtils/SkeletonDiscovery.py`` (``skeleton_discovery``: stable and
  non-stable, background knowledge);
* ``lib/causallearn/utils/Fas.py`` and ``lib/causallearn/search/ConstraintBased/FCI.py``
  (``fas`` + ``fci``).

Those files import causal-learn modules that are not vendored (causal-learn 0.1.3.3 is not on
disk). Stage B installs minimal stand-ins for exactly those names before loading them (see
``_install_standins``): ``Endpoint`` / ``GraphNode`` / ``Edge`` / ``Edges`` / ``GeneralGraph``
with the endpoint-matrix semantics SURVEY Appendix A.6 states ([U], as ``oracle/fci.py`` restates
them), ``ChoiceGenerator`` (lexicographic combinations), ``PCUtils.Helper.append_value``,
``BackgroundKnowledge`` (name-keyed forbidden/required pairs) and ``cit.fisherz`` bound to
``oracle.fisherz.pvalue`` — the library-call expression of causal-learn's FisherZ [U] on
``np.corrcoef(data.T)``. The loop structure, memo keys, visit order, sepset/p_values appends,
deferred removal and the FCI rule sequence are the reference's own code, executed.

Stage B also counts, per depth, what the reference loop did: ``CausalGraph.max_degree`` is wrapped
(after loading, the file is not edited) to snapshot the adjacency, the memo size and
``no_ci_tests`` each time the ``while`` condition (``SkeletonDiscovery.py:72``) is evaluated.

Only outputs are stored (``tests/golden/skeleton_ref.json``): graphs, sepset / p_values lists,
counts, triple / triangle / kite lists, FCI PAGs and sep_sets, and sha256 digests of the inputs
(tests rebuild the inputs from the seeds below and check the digest). Stage B runs under
/opt/conda/bin/python3.9 with PYTHONHASHSEED fixed, and FCI is run under two hash seeds to show
its output does not depend on set iteration order. No reference text is copied into the repo.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
LIB = os.path.join(REF, "lib")
PY39 = "/opt/conda/bin/python3.9"
OUT = os.path.join(HERE, "skeleton_ref.json")
sys.path.insert(0, ROOT)

from tests.golden.skeleton_cases import FCI_CASES, PC_CASES, digest, fci_input, pc_input  # noqa: E402,F401


def stage_a(tmp):
    spec = {"pc": {}, "fci": {}}
    for name, case in PC_CASES.items():
        X = pc_input(name)
        np.save(os.path.join(tmp, name + ".npy"), X)
        spec["pc"][name] = {"opt": case[6], "digest": digest(X)}
    for name, case in FCI_CASES.items():
        X = fci_input(name)
        np.save(os.path.join(tmp, name + ".npy"), X)
        spec["fci"][name] = {"depth": case[6], "digest": digest(X)}
    with open(os.path.join(tmp, "spec.json"), "w") as f:
        json.dump(spec, f)


# --------------------------------------------------------------------------------------------
# stage B (python3.9): stand-ins for the causal-learn names the vendored files import
# --------------------------------------------------------------------------------------------

def _install_standins():
    """Register minimal causal-learn modules the vendored files import ([U] semantics)."""
    import enum
    import itertools
    import math
    import types

    from oracle import fisherz as ofz

    def module(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class Endpoint(enum.Enum):
        TAIL = -1
        NULL = 0
        ARROW = 1
        CIRCLE = 2

    class GraphNode:
        def __init__(self, name):
            self.name = name
            self.attributes = {}

        def get_name(self):
            return self.name

        def add_attribute(self, key, value):
            self.attributes[key] = value

        def __hash__(self):
            return hash(self.name)

        def __eq__(self, other):
            return isinstance(other, GraphNode) and other.name == self.name

        def __repr__(self):
            return self.name

    class EdgeProperty(enum.Enum):
        dd = 1
        nl = 2
        pd = 3
        pl = 4

    class Edge:
        Property = EdgeProperty

        def __init__(self, node1, node2, end1, end2):
            # an edge pointing left (node1 <-- node2) is stored as node2 --> node1
            if end1 == Endpoint.ARROW and end2 == Endpoint.TAIL:
                node1, node2, end1, end2 = node2, node1, end2, end1
            self.node1, self.node2, self.endpoint1, self.endpoint2 = node1, node2, end1, end2
            self.properties = []

        def get_node1(self):
            return self.node1

        def get_node2(self):
            return self.node2

        def get_endpoint1(self):
            return self.endpoint1

        def get_endpoint2(self):
            return self.endpoint2

        def set_endpoint1(self, e):
            self.endpoint1 = e

        def set_endpoint2(self, e):
            self.endpoint2 = e

        def get_proximal_endpoint(self, node):
            if self.node1 == node:
                return self.endpoint1
            if self.node2 == node:
                return self.endpoint2
            return None

        def __str__(self):
            return f"{self.node1} {self.endpoint1.name} {self.endpoint2.name} {self.node2}"

    class Edges:
        def undirected_edge(self, a, b):
            return Edge(a, b, Endpoint.TAIL, Endpoint.TAIL)

    class GeneralGraph:
        """graph[i, j] = the mark at node i of edge i - j (TAIL -1, ARROW 1, CIRCLE 2)."""

        def __init__(self, nodes):
            self.nodes = list(nodes)
            self.num_vars = len(self.nodes)
            self.node_map = {nd: i for i, nd in enumerate(self.nodes)}
            self.graph = np.zeros((self.num_vars, self.num_vars), np.dtype(int))
            self.pag = False

        def add_edge(self, edge):
            i, j = self.node_map[edge.node1], self.node_map[edge.node2]
            self.graph[i, j] = edge.endpoint1.value
            self.graph[j, i] = edge.endpoint2.value

        def add_directed_edge(self, a, b):
            self.add_edge(Edge(a, b, Endpoint.TAIL, Endpoint.ARROW))

        def remove_edge(self, edge):
            i, j = self.node_map[edge.node1], self.node_map[edge.node2]
            self.graph[i, j] = self.graph[j, i] = 0

        def get_edge(self, a, b):
            i, j = self.node_map[a], self.node_map[b]
            if self.graph[i, j] == 0:
                return None
            return Edge(a, b, Endpoint(int(self.graph[i, j])), Endpoint(int(self.graph[j, i])))

        def contains_edge(self, edge):
            e = self.get_edge(edge.node1, edge.node2)
            return e is not None and e.get_proximal_endpoint(edge.node1) == edge.get_proximal_endpoint(edge.node1) \
                and e.get_proximal_endpoint(edge.node2) == edge.get_proximal_endpoint(edge.node2)

        def get_endpoint(self, a, b):
            e = self.get_edge(a, b)
            return e.get_proximal_endpoint(b) if e is not None else None

        def is_adjacent_to(self, a, b):
            return self.graph[self.node_map[a], self.node_map[b]] != 0

        def get_adjacent_nodes(self, a):
            i = self.node_map[a]
            return [self.nodes[j] for j in range(self.num_vars) if self.graph[j, i] != 0]

        def get_nodes_into(self, a, endpoint):
            i = self.node_map[a]
            return [self.nodes[j] for j in range(self.num_vars) if self.graph[i, j] == endpoint.value]

        def get_nodes_out_of(self, a, endpoint):
            i = self.node_map[a]
            return [self.nodes[j] for j in range(self.num_vars) if self.graph[j, i] == endpoint.value]

        def is_def_collider(self, a, b, c):
            e1, e2 = self.get_edge(a, b), self.get_edge(b, c)
            return e1 is not None and e2 is not None and e1.get_proximal_endpoint(b) == Endpoint.ARROW \
                and e2.get_proximal_endpoint(b) == Endpoint.ARROW

        def is_parent_of(self, a, b):
            i, j = self.node_map[a], self.node_map[b]
            return self.graph[j, i] == Endpoint.ARROW.value and self.graph[i, j] == Endpoint.TAIL.value

        def get_parents(self, a):
            return [p for p in self.nodes if self.is_parent_of(p, a)]

        def get_graph_edges(self):
            return [self.get_edge(self.nodes[i], self.nodes[j]) for i in range(self.num_vars)
                    for j in range(i + 1, self.num_vars) if self.graph[i, j] != 0]

        def get_nodes(self):
            return self.nodes

        def set_pag(self, pag):
            self.pag = pag

    class ChoiceGenerator:
        """Tetrad's ChoiceGenerator: the b-subsets of range(a) in lexicographic order, then None."""

        def __init__(self, a, b):
            self._all = [list(c) for c in itertools.combinations(range(a), b)]
            self._k = 0

        def next(self):
            if self._k == len(self._all):
                return None
            self._k += 1
            return self._all[self._k - 1]

    class BackgroundKnowledge:
        """Name-keyed forbidden / required pairs ([U] PCUtils/BackgroundKnowledge.py)."""

        def __init__(self):
            self.forbidden_rules_specs = set()
            self.required_rules_specs = set()
            self.tier_map = {}

        def add_forbidden_by_node(self, a, b):
            self.forbidden_rules_specs.add((a.get_name(), b.get_name()))
            return self

        def is_forbidden(self, a, b):
            return (a.get_name(), b.get_name()) in self.forbidden_rules_specs

        def is_required(self, a, b):
            return (a.get_name(), b.get_name()) in self.required_rules_specs

    corr_cache = {}

    def fisherz(data, X, Y, condition_set, *unused):
        """causal-learn FisherZ [U]: np.corrcoef(data.T) once per data set, then the library-call
        expression of oracle/fisherz.pvalue (inv of the (|S|+2)^2 sub-matrix, math.log, norm.cdf)."""
        key = id(data)
        if key not in corr_cache:
            with np.errstate(invalid="ignore", divide="ignore"):
                corr_cache[key] = (data, np.corrcoef(data.T))
        C = corr_cache[key][1]
        with np.errstate(invalid="ignore", divide="ignore"):
            return ofz.pvalue(C, data.shape[0], X, Y, condition_set)

    def chisq(*a, **k):
        raise NotImplementedError

    def gsq(*a, **k):
        raise NotImplementedError

    def append_value(array, i, j, value):
        if array[i, j] is None:
            array[i, j] = [value]
        else:
            array[i, j].append(value)

    def powerset(L):
        return [list(c) for r in range(len(L) + 1) for c in itertools.combinations(L, r)]

    def list_union(a, b):
        return a + [x for x in b if x not in a]

    class GraphUtils:
        pass

    for pkg in ("causallearn", "causallearn.graph", "causallearn.utils", "causallearn.utils.PCUtils",
                "causallearn.search", "causallearn.search.ConstraintBased"):
        module(pkg, __path__=[])
    module("causallearn.graph.Endpoint", Endpoint=Endpoint)
    module("causallearn.graph.GraphNode", GraphNode=GraphNode)
    module("causallearn.graph.Edge", Edge=Edge)
    module("causallearn.graph.Edges", Edges=Edges)
    module("causallearn.graph.GeneralGraph", GeneralGraph=GeneralGraph)
    module("causallearn.utils.ChoiceGenerator", ChoiceGenerator=ChoiceGenerator)
    module("causallearn.utils.GraphUtils", GraphUtils=GraphUtils)
    module("causallearn.utils.cit", fisherz=fisherz, chisq=chisq, gsq=gsq, np=np, math=math,
           __all__=["fisherz", "chisq", "gsq", "np"])
    module("causallearn.utils.PCUtils.Helper", append_value=append_value, powerset=powerset, list_union=list_union)
    module("causallearn.utils.PCUtils.BackgroundKnowledge", BackgroundKnowledge=BackgroundKnowledge)
    return fisherz, BackgroundKnowledge, corr_cache


def _load(modname, relpath):
    """Load one vendored reference file as the module it is imported as."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(modname, os.path.join(LIB, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _ints(t):
    return [int(v) for v in t]


def _obj_lists(arr, conv):
    """n x n object array of lists (or None) -> {"i,j": [...]} for the non-empty cells."""
    out = {}
    n = arr.shape[0]
    for i in range(n):
        for j in range(n):
            if arr[i, j] is not None:
                out[f"{i},{j}"] = [conv(v) for v in arr[i, j]]
    return out


def stage_b(tmp):
    import warnings
    warnings.simplefilter("ignore")
    fisherz, BackgroundKnowledge, corr_cache = _install_standins()
    GC = _load("causallearn.graph.GraphClass", "causallearn/graph/GraphClass.py")
    SD = _load("causallearn.utils.PCUtils.SkeletonDiscovery", "causallearn/utils/PCUtils/SkeletonDiscovery.py")
    FAS = _load("causallearn.utils.Fas", "causallearn/utils/Fas.py")
    FCI = _load("causallearn.search.ConstraintBased.FCI", "causallearn/search/ConstraintBased/FCI.py")

    levels = []
    orig_max_degree = GC.CausalGraph.max_degree

    def max_degree(self):                      # the loop's while test, SkeletonDiscovery.py:72
        levels.append({"adj": (self.G.graph != 0).astype(np.uint8), "unique": len(self.citest_cache),
                       "calls": int(self.no_ci_tests)})
        return orig_max_degree(self)

    GC.CausalGraph.max_degree = max_degree

    spec = json.load(open(os.path.join(tmp, "spec.json")))
    out = {"pc": {}, "fci": {}}
    for name, c in spec["pc"].items():
        X = np.load(os.path.join(tmp, name + ".npy"))
        opt = c["opt"]
        n = X.shape[1]
        levels.clear()
        corr_cache.clear()
        bk = None
        if "forbid" in opt:
            bk = BackgroundKnowledge()
            from causallearn.graph.GraphNode import GraphNode
            for i, j in opt["forbid"]:
                bk.add_forbidden_by_node(GraphNode(f"X{i + 1}"), GraphNode(f"X{j + 1}"))
        rec = {"digest": c["digest"], "opt": opt, "n": n, "N": int(X.shape[0])}
        try:
            cg = SD.skeleton_discovery(X, 0.05, fisherz, stable=opt.get("stable", True), background_knowledge=bk,
                                       show_progress=False)
        except ValueError as e:
            rec["error"] = {"type": "ValueError", "message": str(e), "levels_started": len(levels)}
            out["pc"][name] = rec
            print(name, "ValueError", flush=True)
            continue
        g = cg.G.graph
        rec["graph"] = np.asarray(g, dtype=int).tolist()
        rec["sepset"] = _obj_lists(cg.sepset, _ints)
        rec["p_values"] = _obj_lists(cg.p_values, float)
        rec["no_ci_tests"] = int(cg.no_ci_tests)
        rec["unique_tests"] = len(cg.citest_cache)
        # one snapshot per evaluation of the while condition: [k] = state after depth k-1
        rec["levels"] = [{"adj_bits": np.packbits(s["adj"], axis=None).tobytes().hex(), "unique": s["unique"],
                          "calls": s["calls"]} for s in levels]
        rec["unshielded_triples"] = [_ints(t) for t in cg.find_unshielded_triples()]
        rec["triangles"] = [_ints(t) for t in cg.find_triangles()]
        rec["kites"] = [_ints(t) for t in cg.find_kites()]
        out["pc"][name] = rec
        print(name, "depths", len(levels) - 1, "tests", rec["unique_tests"], "calls", rec["no_ci_tests"], flush=True)

    for name, c in spec["fci"].items():
        X = np.load(os.path.join(tmp, name + ".npy"))
        FAS.citest_cache.clear()
        corr_cache.clear()
        G, edges = FCI.fci(X, fisherz, 0.05, depth=int(c["depth"]))
        out["fci"][name] = {"digest": c["digest"], "depth": c["depth"], "graph": np.asarray(G.graph, int).tolist(),
                            "unique_tests": len(FAS.citest_cache)}
        print(name, "fci edges", int((G.graph != 0).sum() // 2), flush=True)

    # FAS separately, for its sep_sets (fci's local sep_sets dict is not returned)
    for name, c in spec["fci"].items():
        X = np.load(os.path.join(tmp, name + ".npy"))
        FAS.citest_cache.clear()
        corr_cache.clear()
        from causallearn.graph.GraphNode import GraphNode
        nodes = [GraphNode(f"X{i + 1}") for i in range(X.shape[1])]
        depth = int(c["depth"])
        g, sep_sets = FAS.fas(X, nodes, fisherz, 0.05, None, depth, False, True, False)
        out["fci"][name]["fas_graph"] = np.asarray(g.graph, int).tolist()
        out["fci"][name]["fas_sep_sets"] = sorted([[int(k[0]), int(k[1]), sorted(int(v) for v in s)]
                                                   for k, s in sep_sets.items()])
    json.dump(out, open(os.path.join(tmp, "out.json"), "w"))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--stage-b":
        return stage_b(sys.argv[2])
    with tempfile.TemporaryDirectory() as tmp:
        stage_a(tmp)
        results = []
        for seed in ("0", "12345"):
            env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED=seed,
                       OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
            subprocess.check_call([PY39, os.path.abspath(__file__), "--stage-b", tmp], env=env)
            results.append(json.load(open(os.path.join(tmp, "out.json"))))
        a, b = results
        assert a == b, "reference outputs depend on the hash seed (set iteration order)"
    with open(OUT, "w") as f:
        json.dump(a, f, separators=(",", ":"))
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
