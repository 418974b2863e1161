"""CPU: the C-ABI library loads and exports exactly what include/pcgpu.h declares; host-only
entry points (pcg_orient) run without a GPU; the product path has no CPU fallback."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    text = open(os.path.join(ROOT, "include", "pcgpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*\*?\s*(pcg_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    from rcaeval_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert bound == set(syms), (set(syms) - bound, bound - set(syms))


def test_library_abi_matches_bindings():
    """pcg_abi_info: struct sizes / version of the built library equal the ctypes structs."""
    from rcaeval_amd import _lib
    lib = _lib.load()
    sb, rb, ver = _lib.abi_info(lib)
    assert (sb, rb, ver) == (ctypes.sizeof(_lib.PcgStats), ctypes.sizeof(_lib.PcgRecord), _lib.PCG_ABI_VERSION)
    hdr = open(os.path.join(ROOT, "include", "pcgpu.h")).read()
    assert int(re.search(r"#define PCG_ABI_VERSION (\d+)", hdr).group(1)) == ver

    class Short(ctypes.Structure):       # a binding that missed a field must be refused
        _fields_ = [("tests", ctypes.c_int64 * 32)]
    with pytest.raises(_lib.EngineUnavailable, match="ABI mismatch"):
        _lib.check_abi(lib, stats_cls=Short)


def test_integration_stub_matches_library_abi():
    """INTEGRATION.md's ctypes stub: its Stats struct and its ABI assertion, executed against
    the built library (the stub's own `lib` line is replaced by the in-tree library path)."""
    from rcaeval_amd import _lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(# RCAEval/graph_construction/pc_mi355x.py.*?)```", text, re.S).group(1)
    head = block.split("lib.pcg_create.argtypes")[0]          # struct + ABI check, before any GPU call
    head = head.replace("import ctypes, numpy as np, torch", "import ctypes")
    head = re.sub(r'lib = ctypes.CDLL\("[^"]+"\)', "lib = ctypes.CDLL(LIB_PATH)", head)
    ns = {"LIB_PATH": _lib.LIB_PATH}
    exec(compile(head, "INTEGRATION.md", "exec"), ns)      # asserts inside the stub
    assert ctypes.sizeof(ns["Stats"]) == ctypes.sizeof(_lib.PcgStats)
    assert [f[0] for f in ns["Stats"]._fields_] == [f[0] for f in _lib.PcgStats._fields_]


def test_comm_group_lifecycle_host_only():
    """The in-process transport's group object (pcg_comm_group_*) is host-only: create, stats,
    destroy; bad arguments are refused; a NULL handle cannot join."""
    from rcaeval_amd import _lib
    from rcaeval_amd.dist import LocalGroup
    lib = _lib.load()
    g = ctypes.c_void_p()
    assert lib.pcg_comm_group_create(0, 10.0, ctypes.byref(g)) == _lib.PCG_ERR_INVALID
    grp = LocalGroup(4, timeout_s=5.0)
    assert grp.stats() == {"collectives": 0, "bytes": 0, "broken": False}
    assert lib.pcg_comm_init_group(None, grp.g, 0) == _lib.PCG_ERR_INVALID
    grp.close()
    assert grp.g is None


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from rcaeval_amd import _lib
    from rcaeval_amd.engine import Engine
    with pytest.raises(_lib.EngineUnavailable):
        Engine(0)
    h = ctypes.c_void_p()
    assert _lib.load().pcg_create(0, ctypes.byref(h)) != 0


def test_rca_wrapper_does_not_swallow_missing_engine():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from rcaeval_amd import _lib, synth
    from rcaeval_amd.e2e import pc_pagerank, pc_randomwalk
    df = synth.telemetry_frame(10, 100, seed=1)
    for fn in (pc_pagerank, pc_randomwalk):
        with pytest.raises(_lib.EngineUnavailable):
            fn(df, 0, dataset="online-boutique")


def test_rca_wrapper_dummy_ranks_on_method_error():
    from rcaeval_amd.e2e import rca
    from rcaeval_amd import synth

    @rca
    def broken(data, inject_time=None, dataset=None, **kw):
        raise ValueError("singular")
    df = synth.telemetry_frame(8, 60, n_constant=2, seed=2)
    out = broken(df, 0, dataset="online-boutique")
    from rcaeval_amd.io.time_series import preprocess
    cols = preprocess(df, dataset="online-boutique").columns.to_list()
    assert out == {"adj": [], "node_names": cols, "ranks": cols}


@pytest.mark.parametrize("code", [-1, -2, -3, -6, -8])
def test_rca_wrapper_propagates_engine_faults(code):
    """Engine faults (INVALID, OOM, HIP, RCCL, PEER) must not become dummy rankings: a sticky
    device fault would otherwise score every later RQ2 case as a dummy silently."""
    from rcaeval_amd import _lib, synth
    from rcaeval_amd.e2e import rca

    @rca
    def broken(data, inject_time=None, dataset=None, **kw):
        raise _lib.PcgError(code, "fault")
    df = synth.telemetry_frame(8, 60, seed=2)
    with pytest.raises(_lib.PcgError):
        broken(df, 0, dataset="online-boutique")


def test_rca_wrapper_dummy_ranks_on_data_errors():
    """Data-driven engine outcomes keep the reference's dummy-rank fallback: singular / domain
    (ValueError, as causal-learn raises) and an overflow that survived its reruns."""
    from rcaeval_amd import _lib, synth
    from rcaeval_amd.e2e import rca
    from rcaeval_amd.io.time_series import preprocess
    df = synth.telemetry_frame(8, 60, seed=2)
    cols = preprocess(df, dataset="online-boutique").columns.to_list()
    for exc in (ValueError("singular"), _lib.PcgError(_lib.PCG_ERR_OVERFLOW, "list overflow")):
        @rca
        def broken(data, inject_time=None, dataset=None, **kw):
            raise exc
        with pytest.warns(UserWarning) if isinstance(exc, _lib.PcgError) else _nullctx():
            out = broken(df, 0, dataset="online-boutique")
        assert out == {"adj": [], "node_names": cols, "ranks": cols}


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_orient_cpp_matches_python_oracle_golden():
    from rcaeval_amd.engine import orient
    g = np.load(os.path.join(GOLD, "orient.npz"))
    for i in range(4):
        got = orient(g[f"adj{i}"], g[f"xy{i}"], g[f"bits{i}"])
        np.testing.assert_array_equal(got, g[f"graph{i}"])


@pytest.mark.parametrize("seed", range(5))
def test_orient_cpp_matches_python_oracle_random(seed):
    from oracle import orient as oor
    from oracle import skeleton as osk
    from rcaeval_amd import synth
    from rcaeval_amd.engine import orient
    n = 12 + seed
    X = synth.gaussian_sem(n, 700, seed=300 + seed, w_low=0.4, w_high=0.9, edge_prob=0.28)
    r = osk.skeleton_discovery(np.corrcoef(X.T), 700)
    xy, bits = [], []
    for x in range(n):
        for y in range(n):
            if x != y and r.removed_level[x, y] >= 1:
                lst = r.sepset[x, y]
                side = set(lst[-2]) if x < y else set(lst[-1])
                if side:
                    xy.append((x, y))
                    bits.append([sum(1 << int(s) for s in side)])
    got = orient(r.adj, np.array(xy, np.int32).reshape(-1, 2), np.array(bits, np.uint64).reshape(-1, 1))
    np.testing.assert_array_equal(got, oor.orient(r.adj, r.sepset))


def test_page_rank_preprocess_pair_rules():
    from rcaeval_amd.graph_heads.page_rank import page_rank_preprocess
    adj = np.array([[0, -1, 1, 0], [-1, 0, 0, -1], [-1, 0, 0, 2], [0, 1, 1, 0]])
    out = page_rank_preprocess(adj)
    assert out[0, 1] == out[1, 0] == 1          # undirected
    assert out[0, 2] == 1 and out[2, 0] == 0    # page_rank.py:21-23 (effect -> cause)
    assert out[2, 3] == 1 and out[3, 2] == 0    # (2, 1): FCI o-> treated as ->
    with pytest.raises(ValueError):
        page_rank_preprocess(np.array([[0, 3], [0, 0]]))


def test_digraph_matrix_matches_networkx_semantics():
    """pc_pagerank.py:20-29 with networkx: edges from endpoint codes, sorted non-isolated nodes."""
    import networkx as nx
    from rcaeval_amd.e2e.pc_pagerank import digraph_matrix
    rng = np.random.default_rng(0)
    for _ in range(10):
        n = 12
        g = np.zeros((n, n), int)
        for i in range(n):
            for j in range(i + 1, n):
                r = rng.random()
                if r < 0.15:
                    g[i, j] = g[j, i] = -1
                elif r < 0.25:
                    g[i, j], g[j, i] = -1, 1
                elif r < 0.35:
                    g[i, j], g[j, i] = 1, -1
        G = nx.DiGraph()
        for i in range(n):
            for j in range(n):
                if g[i, j] == -1:
                    G.add_edge(i, j)
                if g[i, j] == 1:
                    G.add_edge(j, i)
        nodes = sorted(G.nodes())
        ref = nx.to_numpy_array(G, nodelist=nodes)
        M, mine = digraph_matrix(g)
        assert mine == nodes
        np.testing.assert_array_equal(M, ref)


class _OracleCI:
    """CPU stand-in for CITester (tests only): oracle Fisher-z p-values, same call surface."""

    def __init__(self, C, N):
        self.C, self.N = C, N

    def pvalues(self, tests):
        from oracle import fisherz as ofz
        return [ofz.pvalue(self.C, self.N, i, j, S) for (i, j, S) in tests]

    def __call__(self, i, j, S):
        return self.pvalues([(i, j, S)])[0]


@pytest.mark.parametrize("priority,seed", [(3, 0), (3, 1), (3, 2), (4, 0), (4, 1)])
def test_uc_priority34_host_matches_python_oracle(priority, seed):
    """UCSepset priority 3/4 [U]: C++ R0 candidates + ordered collider step + Meek against the
    literal Python restatement, both scored with the oracle's Fisher-z p-values."""
    from oracle import orient as oor
    from oracle import skeleton as osk
    from rcaeval_amd import synth
    from rcaeval_amd.citest import uc_orient
    n = 9 + seed
    X = synth.gaussian_sem(n, 500, seed=900 + seed, w_low=0.4, w_high=0.9, edge_prob=0.3)
    C = np.corrcoef(X.T)
    r = osk.skeleton_discovery(C, 500)
    xy, bits = [], []
    for x in range(n):
        for y in range(n):
            if x != y and r.removed_level[x, y] >= 1:
                lst = r.sepset[x, y]
                side = set(lst[-2]) if x < y else set(lst[-1])
                if side:
                    xy.append((x, y))
                    bits.append([sum(1 << int(s) for s in side)])
    ci = _OracleCI(C, 500)
    got = uc_orient(r.adj, np.array(xy, np.int32).reshape(-1, 2), np.array(bits, np.uint64).reshape(-1, 1),
                    priority, ci)
    want = oor.orient(r.adj, r.sepset, priority=priority, ci_test=ci)
    np.testing.assert_array_equal(got, want)


def test_uc_candidates_match_priority2_order():
    """Priority 2 == the collider step over R0 in find_unshielded_triples order."""
    from rcaeval_amd.engine import orient, orient_triples, uc_candidates
    g = np.load(os.path.join(GOLD, "orient.npz"))
    for i in range(4):
        R0 = uc_candidates(g[f"adj{i}"], g[f"xy{i}"], g[f"bits{i}"])
        np.testing.assert_array_equal(orient_triples(g[f"adj{i}"], R0), g[f"graph{i}"])
        np.testing.assert_array_equal(orient(g[f"adj{i}"], g[f"xy{i}"], g[f"bits{i}"]), g[f"graph{i}"])


@pytest.mark.parametrize("seed", range(6))
def test_transition_matrix_array_form_equals_loop(seed):
    from rcaeval_amd.graph_heads.random_walk import transition_matrix
    rng = np.random.default_rng(seed)
    m = int(rng.integers(2, 40))
    codes = rng.choice([0, 0, 0, -1, 1], size=(m, m))
    adj = codes.copy()
    for a in range(m):                       # keep pairs valid: (x, y) in the accepted set
        for b in range(a + 1, m):
            pair = [(0, 0), (-1, -1), (1, -1), (-1, 1), (0, 1), (1, 0), (1, 1)][rng.integers(0, 7)]
            adj[a, b], adj[b, a] = pair
        adj[a, a] = [0, -1, 1][rng.integers(0, 3)] if seed % 2 else 0
    names = [f"n{int(v)}" for v in rng.integers(0, max(2, m - seed), size=m)]   # duplicates merge by name
    uniq = list(dict.fromkeys(names))
    scores = None if seed < 2 else rng.normal(size=len(uniq))
    from tests_support import loop_transition_matrix
    np.testing.assert_array_equal(transition_matrix(adj, names, uniq, scores),
                                  loop_transition_matrix(adj, names, uniq, scores))


def test_random_walk_codes_error_first_cell():
    from rcaeval_amd.graph_heads.random_walk import edge_matrix
    adj = np.zeros((4, 4), int)
    adj[2, 1], adj[1, 2] = 2, 1
    adj[0, 3] = 5
    with pytest.raises(ValueError, match="Unexpected value: 5, 0"):
        edge_matrix(adj)


def test_page_rank_preprocess_table_equals_visit_loop():
    from rcaeval_amd.graph_heads.page_rank import _PAIR_RULES, page_rank_preprocess
    rng = np.random.default_rng(3)
    keys = list(_PAIR_RULES)
    for m in (1, 2, 7, 30):
        adj = np.zeros((m, m), int)
        for a in range(m):
            for b in range(a, m):
                u, v = keys[rng.integers(0, len(keys))]
                if a == b:
                    u = v = [0, -1, 1, 2][rng.integers(0, 4)]
                adj[a, b], adj[b, a] = u, v
        ref = np.zeros_like(adj)
        for a in range(m):
            for b in range(m):
                rule = _PAIR_RULES[(int(adj[a, b]), int(adj[b, a]))]
                if rule is None:
                    continue
                if rule[0] is not None:
                    ref[a, b] = rule[0]
                if rule[1] is not None:
                    ref[b, a] = rule[1]
        np.testing.assert_array_equal(page_rank_preprocess(adj), ref)


def _crt_units_host(n, N):
    """corr.hip crt_plan restated: (moduli k, split-K slabs ks) of the CRT K1, or None."""
    import bench
    km = bench.k1_crt_moduli(n, N, {"K1_I8": 1, "K1_CRT": 1, "K1_CRT_MINN": 256, "K1_CRT_BITS": 53})
    if km is None:
        return None
    k = km[0]
    T = (n + 255) // 256
    ntiles = T * (T + 1) // 2
    TB = (N + 63) // 64 * 2
    best, cost_best = 1, None
    for ks in range(1, 17):
        kb = -(-TB // ks)
        kb = -(-kb // 4) * 4
        if -(-TB // kb) != ks or kb > 4095:
            continue
        U = ntiles * k * ks
        cost = ((U + 255) // 256) * kb * 0.3 + U * 0.026
        if cost_best is None or cost < cost_best:
            best, cost_best = ks, cost
    return k, best, ntiles


@pytest.mark.parametrize("n,N,world", [(2000, 10000, 1), (2000, 10000, 8), (300, 1200, 3), (256, 40000, 2),
                                       (100, 5000, 2), (255, 1000, 1)])
def test_corr_shard_bytes_follow_the_k1_plan(n, N, world):
    """pcg_corr_shard_bytes (host-only): the CRT path (n >= 256) shares (tile, modulus, slab)
    residue units of 64 KiB; below it, the digit path's packed rows x n doubles."""
    from rcaeval_amd import _lib
    lib = _lib.load()
    got = ctypes.c_int64()
    assert lib.pcg_corr_shard_bytes(None, n, N, world, ctypes.byref(got)) == 0
    plan = _crt_units_host(n, N)
    if plan is None:
        rows = ctypes.c_int64()
        assert lib.pcg_corr_shard_rows(n, world, ctypes.byref(rows)) == 0
        assert got.value == rows.value * n * 8
    else:
        k, ks, ntiles = plan
        units = ntiles * k * ks
        assert got.value == -(-units // world) * 65536
    if (n, N) == (2000, 10000):
        assert plan[:2] == (16, 2)          # the headline: 16 moduli (b = 55), 2 slabs


def test_corr_crt_path_switch(monkeypatch):
    """PCG_K1_CRT=0 (the environment default of PCG_TUNE_K1_CRT; a NULL handle reads the defaults)
    routes n >= 256 back to the digit path's row share, with another plan signature."""
    from rcaeval_amd import _lib
    lib = _lib.load()
    got, rows = ctypes.c_int64(), ctypes.c_int64()
    monkeypatch.setenv("PCG_K1_CRT", "0")
    assert lib.pcg_corr_shard_bytes(None, 2000, 10000, 4, ctypes.byref(got)) == 0
    assert lib.pcg_corr_shard_rows(2000, 4, ctypes.byref(rows)) == 0
    assert got.value == rows.value * 2000 * 8
    sig_digit = ctypes.c_int64()
    assert lib.pcg_k1_plan_signature(None, 2000, 10000, ctypes.byref(sig_digit)) == 0
    monkeypatch.delenv("PCG_K1_CRT")
    sig_crt = ctypes.c_int64()
    assert lib.pcg_k1_plan_signature(None, 2000, 10000, ctypes.byref(sig_crt)) == 0
    assert sig_crt.value != sig_digit.value and sig_crt.value >> 62 == 1
