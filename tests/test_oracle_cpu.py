"""CPU: the oracle pinned against golden vectors and against itself (numpy vs C restatement).

No GPU needed. These establish what the GPU parity tests compare against.
"""
import json
import os

import numpy as np
import pytest

from oracle import cpc, fisherz
from oracle import orient as oor
from oracle import pagerank as opr
from oracle import random_walk as orw
from oracle import skeleton as osk
from rcaeval_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_fisherz_golden_library_arithmetic():
    """oracle FisherZ == the committed causal-learn-expression p-values (numpy/scipy calls)."""
    g = np.load(os.path.join(GOLD, "fisherz.npz"))
    C = fisherz.corrcoef(g["X"])
    np.testing.assert_array_equal(C, g["C"])
    for key, p in zip(g["keys"][::7], g["p"][::7]):
        x, y, S = int(key[0]), int(key[1]), [int(v) for v in key[2:] if v >= 0]
        assert fisherz.p_close(fisherz.pvalue(C, 500, x, y, S), p)


def test_c_oracle_matches_fisherz_golden():
    """C restatement (LU per test, cephes ndtr branches) within the north-star tolerance."""
    g = np.load(os.path.join(GOLD, "fisherz.npz"))
    C = g["C"]
    import ctypes
    lib = cpc.lib()
    keys, ps = g["keys"], g["p"]
    for d in range(4):
        sel = np.nonzero((keys[:, 2:] >= 0).sum(1) == d)[0]
        ab = np.ascontiguousarray(keys[sel, :2], np.int32)
        S = np.ascontiguousarray(keys[sel, 2:2 + max(d, 1)], np.int32)
        out = np.zeros(len(sel))
        err = np.zeros(len(sel), np.int32)
        P = ctypes.c_void_p
        lib.orc_fisherz_batch(C.ctypes.data_as(P), 12, 500, ab.ctypes.data_as(P), S.ctypes.data_as(P), d,
                              len(sel), out.ctypes.data_as(P), err.ctypes.data_as(P))
        assert not err.any()
        assert fisherz.p_close(out, ps[sel]).all()


def test_p_value_cancellation_replicated():
    """p = 2*(1 - norm.cdf(X)) reaches exactly 0 for large X, like the reference."""
    assert fisherz.pvalue_from_r(0.999999, 10000, 0) == 0.0
    p = fisherz.pvalue_from_r(0.3, 100, 1)
    assert 0 < p < 0.01


@pytest.mark.parametrize("n,N,seed", [(8, 300, 0), (12, 500, 1), (20, 300, 2), (15, 1000, 3), (25, 400, 4)])
def test_skeleton_numpy_vs_c_oracle(n, N, seed):
    X = synth.gaussian_sem(n, N, seed=seed, w_low=0.3, w_high=0.9)
    C = np.corrcoef(X.T)
    r = osk.skeleton_discovery(C, N)
    c = cpc.skeleton(C, N, record_cap=10 ** 6)
    np.testing.assert_array_equal(c.removed_level, r.removed_level)
    assert c.tests == r.tests_per_level and c.calls == r.calls_per_level
    got = {(int(a), int(b), tuple(int(v) for v in s[:dd])): p for a, b, dd, s, p in c.records}
    assert set(got) == set(r.cache)
    keys = sorted(got)
    assert fisherz.p_close([got[k] for k in keys], [r.cache[k] for k in keys]).all()
    # x-side unions at the removal depth
    for x in range(n):
        for y in range(n):
            if x != y and r.removed_level[x, y] >= 1:
                lst = r.sepset[x, y]
                side = set(int(v) for v in (lst[-2] if x < y else lst[-1]))
                bits = c.side_union[x, y]
                mine = {j for j in range(n) if (int(bits[j >> 6]) >> (j & 63)) & 1}
                assert mine == side


def test_max_depth_and_node_skip_rule():
    X = synth.gaussian_sem(18, 400, seed=5, w_low=0.3, w_high=0.9, edge_prob=0.3)
    C = np.corrcoef(X.T)
    for md in (0, 1, 2):
        r = osk.skeleton_discovery(C, 400, max_depth=md)
        c = cpc.skeleton(C, 400, max_depth=md)
        np.testing.assert_array_equal(c.removed_level, r.removed_level)
        assert r.max_depth_run <= md


def test_pairwise_sum_model_matches_numpy():
    """The GPU PageRank reduction reproduces numpy's pairwise summation bit for bit."""
    from tests_support import pairwise_sum
    rng = np.random.default_rng(3)
    for _ in range(200):
        m = int(rng.integers(1, 3000))
        a = rng.random(m) * 10.0 ** rng.uniform(-6, 6, m)
        assert pairwise_sum(list(a)) == np.sum(a)
        assert pairwise_sum(list(np.abs(a - 0.5))) == np.linalg.norm(a - 0.5, ord=1)


def test_pagerank_kernel_algorithm_matches_golden():
    """A line-by-line replica of k_pagerank's arithmetic equals the scipy/numpy oracle bitwise."""
    from tests_support import kernel_pagerank
    g = np.load(os.path.join(GOLD, "pagerank.npz"))
    for i in range(12):
        A, s = g[f"A{i}"], g[f"s{i}"]
        np.testing.assert_array_equal(opr.pagerank(A), s)
        np.testing.assert_array_equal(kernel_pagerank(A.tolist()), s)


def test_pcg64_replica_matches_numpy():
    st = np.random.default_rng(0).bit_generator.state["state"]
    mine = orw.pcg64_doubles(st["state"], st["inc"], 50)
    np.testing.assert_array_equal(np.array(mine), np.random.default_rng(0).random(50))


def test_random_walk_oracle_matches_reference_golden():
    """oracle/random_walk + the drop-in's transition matrix reproduce the reference outputs."""
    from rcaeval_amd.graph_heads.random_walk import transition_matrix
    cases = json.load(open(os.path.join(GOLD, "random_walk.json")))
    for c in cases:
        adj = np.array(c["adj"])
        names = c["names"]
        uniq = list(dict.fromkeys(names))
        P = transition_matrix(adj, names, uniq)
        num_loop = c["num_loop"] if c["num_loop"] is not None else 10 * len(uniq)
        counts = orw.walk_counts(P, 0, num_loop)
        res = sorted([(nm, counts[i] / num_loop) for i, nm in enumerate(uniq)], key=lambda t: t[1], reverse=True)
        assert [r[0] for r in res] == c["ranks"]
        np.testing.assert_array_equal([r[1] for r in res], c["scores"])


def test_preprocess_matches_reference_golden():
    import pandas as pd
    from rcaeval_amd.io.time_series import preprocess
    g = np.load(os.path.join(GOLD, "preprocess.npz"))
    for key in g["keys"]:
        i, dataset, dk = str(key).split("_")
        dataset = None if dataset == "None" else dataset
        df = pd.DataFrame(g[f"in{i}_values"], columns=list(g[f"in{i}_cols"]))
        out = preprocess(data=df, dataset=dataset, dk_select_useful=(dk == "True"))
        assert out.columns.to_list() == list(g[f"out{key}_cols"])
        np.testing.assert_array_equal(out.to_numpy(dtype=float), g[f"out{key}_values"])


def test_orient_oracle_golden():
    g = np.load(os.path.join(GOLD, "orient.npz"))
    for i in range(4):
        adj = g[f"adj{i}"].astype(bool)
        n = adj.shape[0]
        sep = np.empty((n, n), object)
        rows = {}
        for (x, y), b in zip(g[f"xy{i}"], g[f"bits{i}"]):
            rows.setdefault((min(x, y), max(x, y)), set()).update(
                j for j in range(n) if (int(b[j >> 6]) >> (j & 63)) & 1)
        for a in range(n):
            for b in range(n):
                sep[a, b] = [tuple(rows.get((min(a, b), max(a, b)), ()))]
        np.testing.assert_array_equal(oor.orient(adj, sep), g[f"graph{i}"])
