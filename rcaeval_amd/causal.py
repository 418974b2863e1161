"""Drop-in for causal-learn's ``pc(...)`` on the MI355X engine.

Mirrors causal-learn 0.1.3.3 ``search/ConstraintBased/PC.py`` ``pc`` / ``pc_alg`` [U] as
called by RCAEval (``RCAEval/e2e/pc_pagerank.py:19``, ``RCAEval/graph_construction/pc.py:15-20,
46-56``): same arguments, same ``CausalGraph`` surface (``.G.graph`` endpoint codes,
``.sepset`` n x n lists of tuples, ``.p_values``, ``.PC_elapsed``, ``.no_ci_tests``), same
error behaviour (``ValueError`` on a singular sub-correlation matrix or a math domain error,
``AssertionError`` on NaN/inf input).

Pipeline: host → HBM once (X), K1 correlation (fp64 MFMA), K2/K3 level-synchronous
skeleton on the device, sepset unions + removal depths back to the host, orientation
(UCSepset priority 2 + Meek) in host C++ (``pcg_orient``); priorities 3/4 score their
collider candidates with batched device CI tests (``rcaeval_amd.citest``).
"""
from __future__ import annotations

import time
import warnings
from itertools import combinations

import numpy as np

from . import _lib
from .background import BackgroundKnowledge, banned_pairs
from .citest import CITester, uc_orient
from .engine import SkeletonOut, get_engine, orient
from .phases import phase
from .skeleton_seq import skeleton_unstable

fisherz = "fisherz"
chisq = "chisq"
gsq = "gsq"
kci = "kci"
mv_fisherz = "mv_fisherz"


class GraphNode:
    def __init__(self, name: str):
        self.name = name

    def get_name(self) -> str:
        return self.name

    def __repr__(self) -> str:
        return self.name


class GeneralGraph:
    """Endpoint-code matrix holder (causal-learn ``GeneralGraph`` [U] subset)."""

    def __init__(self, graph: np.ndarray, names):
        self.graph = graph
        self.nodes = [GraphNode(str(nm)) for nm in names]
        self.num_vars = len(self.nodes)

    def get_nodes(self):
        return self.nodes

    def get_node_names(self):
        return [nd.get_name() for nd in self.nodes]

    def get_num_edges(self) -> int:
        return int(np.count_nonzero(np.triu((self.graph != 0) | (self.graph.T != 0), 1)))


class SepsetArray:
    """``cg.sepset`` (n x n object array of lists of tuples), materialised per entry.

    Entry [a, b] follows ``SkeletonDiscovery.py:135-136``: for every depth at which the pair
    was adjacent, one tuple from a's visit then one from b's visit (each visit skipped when
    that node had fewer than depth-1 neighbours, ``:83``); the tuple is the union of all
    independent S from that side (``:129-130``), empty unless the edge was removed there.

    The tuple is ``tuple(sepsets)`` of the reference's ``set`` of ``np.int64``, so its order is
    CPython's set order for the reference's insertion sequence: the members of each
    independent S, S in ``combinations`` order (``:109,129-130``). A union of exactly d
    members came from one S (inserted ascending); a larger union is ordered by deciding the
    d-subsets of the union in ``combinations`` order on the device (``pcg_fisherz_batch``,
    LU path) — all of them at once, on first access of such an entry.
    """

    def __init__(self, out: SkeletonOut, ci=None, alpha: float = 0.05):
        """``ci``: a CITester, or a zero-argument callable that builds one on first need."""
        self.shape = (out.n, out.n)
        self._out = out
        self._levels = out.levels
        n = out.n
        self._rl = out.removed_level
        self._deg = out.deg_levels
        self._ci = ci
        self._alpha = float(alpha)
        self._rows_built: dict | None = None       # decoded on first access (pc_pagerank never reads them)
        self._order: dict | None = None

    @property
    def _rows(self) -> dict:
        """(x, y) -> ascending members of x's side union at the removal depth (export rows)."""
        if self._rows_built is None:
            out = self._out
            rows: dict = {}
            xy = np.asarray(out.sep_xy)
            if len(xy):
                bits = np.ascontiguousarray(out.sep_bits).view(np.uint64)
                # little-endian bit order: member w * 64 + b <-> bit b of word w
                flags = np.unpackbits(bits.view(np.uint8).reshape(len(xy), -1), axis=1, bitorder="little")
                rr, cc = np.nonzero(flags)
                starts = np.searchsorted(rr, np.arange(len(xy) + 1))
                for r in range(len(xy)):
                    x, y = int(xy[r, 0]), int(xy[r, 1])
                    members = cc[starts[r]:starts[r + 1]].tolist()
                    prev = rows.get((x, y))          # several rows per pair when edge-sharded: OR
                    rows[(x, y)] = sorted(set(prev) | set(members)) if prev else members
            self._rows_built = rows
        return self._rows_built

    def _resolve_order(self) -> dict:
        """First-insertion order of every union with more members than its depth."""
        order: dict = {}
        todo = []
        for (x, y), mem in self._rows.items():
            a, b = (x, y) if x < y else (y, x)
            d = int(self._rl[a, b])
            if 0 < d < len(mem):
                todo.append((x, y, d, mem))
        if not todo:
            return order
        if self._ci is None:
            raise RuntimeError("sepset insertion order needs the CI tester of the run "
                               "(CausalGraph.release() dropped it)")
        if not isinstance(self._ci, CITester):
            self._ci = self._ci()
        tests, spans = [], []
        for (x, y, d, mem) in todo:
            subs = list(combinations(mem, d))
            spans.append((len(tests), subs))
            tests.extend((x, y, S) for S in subs)
        p, _ = self._ci.pvalues_status(tests)
        for (x, y, d, mem), (lo, subs) in zip(todo, spans):
            seq: list = []
            for q, S in enumerate(subs):
                if p[lo + q] > self._alpha:
                    seq.extend(s for s in S if s not in seq)
            seq.extend(s for s in mem if s not in seq)    # decisions within the LU band: ascending
            order[(x, y)] = seq
        return order

    def _side(self, x: int, y: int) -> tuple:
        mem = self._rows.get((x, y))
        if not mem:
            return ()
        a, b = (x, y) if x < y else (y, x)
        if len(mem) > max(int(self._rl[a, b]), 0):
            if self._order is None:
                self._order = self._resolve_order()
            mem = self._order.get((x, y), mem)
        return tuple(set(np.int64(m) for m in mem))    # CPython set order for this insertion order

    def __getitem__(self, key):
        if isinstance(key, tuple) and len(key) == 2:
            i, j = int(key[0]), int(key[1])
            if i == j:
                return None
            a, b = (i, j) if i < j else (j, i)
            rl = int(self._rl[a, b])
            last = rl if rl >= 0 else self._levels - 1
            out = []
            for d in range(0, last + 1):
                for v, w in ((a, b), (b, a)):
                    if self._deg[d, v] < d - 1:
                        continue
                    out.append(self._side(v, w) if d == rl else ())
            return out if out else None
        if isinstance(key, (int, np.integer)):
            return [self[int(key), j] for j in range(self.shape[1])]
        raise TypeError("SepsetArray supports [i, j] indexing")

    def to_numpy(self) -> np.ndarray:
        n = self.shape[0]
        arr = np.empty((n, n), object)
        for i in range(n):
            for j in range(n):
                arr[i, j] = self[i, j]
        return arr


# p_values materialises one float per reference ci_test call that returned p <= alpha; past
# this many calls (RCAEval graphs are far below it) the lists would not fit a host anyway
MAX_P_VALUE_CALLS = 20_000_000


def p_values_from_run(out: SkeletonOut, C, N: int, alpha: float, device: int | None = None,
                      banned=None) -> np.ndarray:
    """``cg.p_values`` of a stable run (``SkeletonDiscovery.py:131-132``): for every visit of
    x -> y at every depth, the p of each dependent S in ``combinations`` order.

    The p-values come from a ``PCG_FLAG_FULL_P | PCG_FLAG_RECORD`` rerun of the skeleton on the
    same C (every unique test recorded with the reference's p); the enumeration replays the
    reference loop on the recorded adjacency of each depth (``removed_level``), so cache hits
    repeat the cached p exactly as ``GraphClass.py:89-90`` returns it. Tests deeper than the
    record depth (degenerate graphs) are evaluated by ``pcg_fisherz_batch``.
    """
    n = out.n
    calls = int(sum(out.stats["calls"]))
    if calls > MAX_P_VALUE_CALLS:
        raise NotImplementedError(f"cg.p_values of {calls} ci_test calls (> {MAX_P_VALUE_CALLS}): "
                                  "use the record path (Engine.skeleton(..., flags=PCG_FLAG_RECORD))")
    eng = get_engine(device)
    L = out.levels
    rer = eng.skeleton(C, N, alpha=alpha, max_depth=L - 1,
                       flags=_lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD,
                       record_capacity=max(int(sum(out.stats["tests"])), 1), banned=banned)
    cache: dict = {}
    for r in rer.records:
        d = int(r["d"])
        cache[(int(r["a"]), int(r["b"]), tuple(int(s) for s in r["s"][:d]))] = float(r["p"])
    rl = out.removed_level
    pv = np.empty((n, n), object)
    ci = None
    for d in range(L):
        A = (rl == -1) | (rl >= d)
        np.fill_diagonal(A, False)
        nbrs = [np.flatnonzero(A[x]).tolist() for x in range(n)]
        miss = []
        for x in range(n):
            Nx = nbrs[x]
            if len(Nx) < d - 1:
                continue
            for y in Nx:
                a, b = (x, y) if x < y else (y, x)
                for S in combinations([v for v in Nx if v != y], d):
                    if (a, b, S) not in cache:
                        miss.append((a, b, S))
        if miss:
            if ci is None:
                ci = CITester(C, N, device=device)
            p, _ = ci.pvalues_status(miss)
            cache.update(zip(miss, p))
        for x in range(n):
            Nx = nbrs[x]
            if len(Nx) < d - 1:
                continue
            for y in Nx:
                a, b = (x, y) if x < y else (y, x)
                for S in combinations([v for v in Nx if v != y], d):
                    p = cache[(a, b, S)]
                    if not p > alpha:
                        if pv[x, y] is None:
                            pv[x, y] = [p]
                        else:
                            pv[x, y].append(p)
    return pv


class CausalGraph:
    """causal-learn ``CausalGraph`` result surface [U] (``lib/causallearn/graph/GraphClass.py:19-60``).

    ``p_values`` is built on first access (``p_values_from_run``) for stable runs."""

    def __init__(self, graph: np.ndarray, names, skeleton: SkeletonOut | None, C=None, N: int = 0,
                 alpha: float = 0.05, device: int | None = None, banned=None):
        self.G = GeneralGraph(graph, names)
        self.skeleton = skeleton
        self._run = (C, int(N), float(alpha), device, banned)
        # the device correlation stays referenced only for what may still need it (the lazy
        # p_values rerun and the sepset insertion order); the CI tester is built on first use
        ci = (lambda: CITester(self._run[0], self._run[1], device=self._run[3])) \
            if (skeleton is not None and C is not None) else None
        self.sepset = (SepsetArray(skeleton, ci, alpha) if skeleton is not None
                       else np.empty(graph.shape, object))
        self._p_values = None if (skeleton is not None and C is not None) else np.empty(graph.shape, object)
        self.PC_elapsed = -1
        self.no_ci_tests = int(sum(skeleton.stats["calls"])) if skeleton is not None else 0
        self.stats = skeleton.stats if skeleton is not None else {}

    @property
    def p_values(self) -> np.ndarray:
        if self._p_values is None:
            C, N, alpha, device, banned = self._run
            if C is None:
                raise RuntimeError("p_values needs the run's correlation matrix (CausalGraph.release() dropped it)")
            self._p_values = p_values_from_run(self.skeleton, C, N, alpha, device, banned)
        return self._p_values

    @p_values.setter
    def p_values(self, value) -> None:
        self._p_values = value

    def release(self) -> None:
        """Drop the run's device correlation (n x n fp64) once ``G`` is all that is needed:
        afterwards ``p_values`` (if not yet read) and large-union ``sepset`` orders raise."""
        C, N, alpha, device, banned = self._run
        self._run = (None, N, alpha, device, banned)
        if isinstance(self.sepset, SepsetArray):
            self.sepset._ci = None


def _check_supported(indep_test, stable, uc_rule, uc_priority, mvpc, background_knowledge):
    name = indep_test if isinstance(indep_test, str) else getattr(indep_test, "__name__", str(indep_test))
    if name != fisherz:
        raise NotImplementedError(f"indep_test={name!r}: only fisherz runs on the MI355X engine")
    if mvpc:
        raise NotImplementedError("mvpc=True (missing-value PC) is not on the engine's path")
    if uc_rule != 0:
        raise NotImplementedError("uc_rule != 0 is not on the pc_pagerank / pc_randomwalk path")
    if uc_priority not in (-1, 2, 3, 4):
        raise NotImplementedError(f"uc_priority={uc_priority}: priorities 2, 3 (= -1, the default) and 4 are built")
    if background_knowledge is not None and not isinstance(background_knowledge, BackgroundKnowledge):
        raise TypeError("'background_knowledge' must be 'BackgroundKnowledge' type!")
    if background_knowledge is not None and not stable:
        raise NotImplementedError("background_knowledge with stable=False is not on the RCAEval path "
                                  "(pc_default passes it to the stable run only)")


def skeleton_from_data(data: np.ndarray, alpha: float = 0.05, max_depth: int = -1, flags: int = 0,
                       device: int | None = None, record_capacity: int = 0, banned=None):
    """Correlation + stable skeleton on the GPU; returns (SkeletonOut, C tensor)."""
    eng = get_engine(device)
    X = np.asarray(data, dtype=np.float64)
    return eng.corr_skeleton(X, alpha=alpha, max_depth=max_depth, flags=flags, record_capacity=record_capacity,
                             banned=banned)


def pc(data: np.ndarray, alpha: float = 0.05, indep_test=fisherz, stable: bool = True, uc_rule: int = 0,
       uc_priority: int = 2, mvpc: bool = False, correction_name: str = "MV_Crtn_Fisher_Z",
       background_knowledge=None, verbose: bool = False, show_progress: bool = True, node_names=None,
       max_depth: int = -1, device: int | None = None, full_p: bool = False, **kwargs) -> CausalGraph:
    """causal-learn ``pc`` [U] on the GPU (fisherz, stable, uc_rule 0, uc_priority 2/3/4; -1 means
    uc_sepset's default priority 3, as ``pc_alg`` [U] calls ``uc_sepset(cg_1)`` then)."""
    assert type(data) == np.ndarray  # SkeletonDiscovery.py:47
    assert 0 < alpha < 1
    _check_supported(indep_test, stable, uc_rule, uc_priority, mvpc, background_knowledge)
    if data.shape[0] < data.shape[1]:
        warnings.warn("The number of features is much larger than the sample size!")
    X = np.asarray(data, dtype=np.float64)
    # CIT_Base.assert_input_data_is_valid [U]
    assert not np.isnan(X).any(), "Input data contains NaN. Please check."
    assert not np.isinf(X).any(), "Input data contains Inf. Please check."
    n = X.shape[1]
    names = node_names if node_names is not None else [f"X{i + 1}" for i in range(n)]
    start = time.time()
    if n == 0:
        raise ValueError("max() arg is an empty sequence")
    if n == 1:
        cg = CausalGraph(np.zeros((1, 1), int), names, None)
        cg.PC_elapsed = time.time() - start
        return cg
    priority = 3 if uc_priority == -1 else uc_priority
    if not stable:
        eng = get_engine(device)
        ci = CITester(eng.corr(X), X.shape[0], device=device)
        sk = skeleton_unstable(ci, alpha=alpha, max_depth=max_depth)
        xy, bits = sk.sep_rows()
        graph = uc_orient(sk.adj.astype(np.uint8), xy, bits, priority, ci).astype(int)
        cg = CausalGraph(graph, names, None)
        cg.sepset = sk.sepset
        cg.p_values = sk.p_values
        cg.no_ci_tests = int(sum(sk.calls))
        cg.stats = {"levels": sk.levels, "calls": sk.calls}
        cg.PC_elapsed = time.time() - start
        return cg
    flags = _lib.PCG_FLAG_FULL_P if full_p else 0
    knowledge = background_knowledge.masks(names) if background_knowledge is not None else None
    banned = None if knowledge is None else banned_pairs(knowledge[0])
    with phase("K1 + skeleton"):
        out, C = skeleton_from_data(X, alpha=alpha, max_depth=max_depth, flags=flags, device=device, banned=banned)
    with phase("orientation"):
        if priority == 2 and knowledge is None:
            graph = orient(out.adj, out.sep_xy, out.sep_bits, priority=2).astype(int)
        else:
            ci = CITester(C, X.shape[0], device=device) if priority != 2 else None
            graph = uc_orient(out.adj, out.sep_xy, out.sep_bits, priority, ci, knowledge=knowledge).astype(int)
    cg = CausalGraph(graph, names, out, C=C, N=X.shape[0], alpha=alpha, device=device, banned=banned)
    cg.PC_elapsed = time.time() - start
    return cg
