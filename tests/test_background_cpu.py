"""Background knowledge (pc_default(with_bg=True), RCAEval/graph_construction/pc.py:6-9,19) on CPU:
the BackgroundKnowledge rule semantics and masks, the C-restated skeleton's banned pairs against
the literal Python restatement of SkeletonDiscovery.py:86-106, and the host C++ orientation
(pcg_orient_bk) against the Python restatement of orient_by_background_knowledge + uc_sepset +
meek. causal-learn is not importable here and the reference holds no with_bg fixture, so these
are parity UNPINNED [U]: the restatements follow causal-learn 0.1.3.3's published source."""
import numpy as np
import pytest

from rcaeval_amd import synth
from rcaeval_amd.background import BackgroundKnowledge, banned_pairs


def _names(n, seed):
    rng = np.random.default_rng(seed)
    kinds = ["cpu", "mem", "lat50", "lat90", "latency"]
    svcs = ["frontend", "cart", "frontend-x", "ad", "xfrontend"]
    return [f"{svcs[rng.integers(len(svcs))]}{i}_{kinds[rng.integers(len(kinds))]}" for i in range(n)]


def _knowledge(names, seed):
    rng = np.random.default_rng(seed)
    bk = BackgroundKnowledge()
    bk.add_forbidden_by_pattern(".*mem$", ".*lat50$")
    bk.add_forbidden_by_pattern(".*cpu$", ".*lat50$")
    bk.add_forbidden_by_pattern(".*", "frontend.*")
    bk.add_required_by_pattern("cart.*", ".*lat90$")
    for _ in range(3):
        a, b = rng.choice(len(names), 2, replace=False)
        bk.add_forbidden_by_node(names[a], names[b])
        a, b = rng.choice(len(names), 2, replace=False)
        bk.add_required_by_node(names[a], names[b])
    for i in rng.choice(len(names), 4, replace=False):
        bk.add_node_to_tier(names[i], int(rng.integers(0, 3)))
    return bk


@pytest.mark.parametrize("seed", range(3))
def test_masks_equal_pairwise_queries(seed):
    names = _names(17, seed)
    bk = _knowledge(names, seed)
    F, R = bk.masks(names)
    for i, a in enumerate(names):
        for j, b in enumerate(names):
            assert F[i, j] == bk.is_forbidden(a, b)
            assert R[i, j] == bk.is_required(a, b)
    B = banned_pairs(F)
    assert (B == B.T).all() and not B.diagonal().any()
    assert ((B != 0) == ((F != 0) & (F.T != 0) & ~np.eye(len(names), dtype=bool))).all()


def test_reference_patterns_match_at_the_start_only():
    from rcaeval_amd.graph_construction.pc import background_knowledge as bk
    assert bk.is_forbidden("cart_mem", "cart_lat50")
    assert bk.is_forbidden("cart_cpu", "ad_lat50")
    assert not bk.is_forbidden("cart_lat50", "cart_mem")
    assert not bk.is_forbidden("cart_mem", "cart_lat50x")       # '$' anchors the end
    assert bk.is_forbidden("anything", "frontend_cpu")
    assert not bk.is_forbidden("anything", "xfrontend_cpu")     # re.match: start-anchored
    assert bk.is_forbidden("frontend_cpu", "frontend_mem") and bk.is_forbidden("frontend_mem", "frontend_cpu")


def test_rule_api_types_and_removal():
    bk = BackgroundKnowledge()
    with pytest.raises(TypeError):
        bk.add_forbidden_by_pattern(1, "a")
    with pytest.raises(TypeError):
        bk.add_node_to_tier("a", -1)
    assert bk.add_forbidden_by_node("a", "b") is bk
    assert bk.is_forbidden("a", "b") and not bk.is_forbidden("b", "a")
    bk.remove_forbidden_by_node("a", "b")
    assert not bk.is_forbidden("a", "b")
    bk.add_node_to_tier("late", 2).add_node_to_tier("early", 1)
    assert bk.is_forbidden("late", "early") and not bk.is_forbidden("early", "late")
    assert bk.is_in_which_tier("late") == 2 and bk.is_in_which_tier("none") == -1


def test_pc_rejects_unsupported_knowledge_combinations():
    from rcaeval_amd.causal import pc
    X = np.random.default_rng(0).standard_normal((50, 4))
    with pytest.raises(TypeError):
        pc(X, background_knowledge=object())
    with pytest.raises(NotImplementedError):
        pc(X, stable=False, background_knowledge=BackgroundKnowledge())


def _frame_C(m, rows, seed):
    X = synth.gaussian_sem(m, rows, w_low=0.4, w_high=0.9, edge_prob=0.3, seed=seed)
    return np.corrcoef(X.T)


@pytest.mark.parametrize("seed", range(4))
def test_c_oracle_banned_pairs_match_python_restatement(seed):
    """pc_oracle.c's banned pairs == SkeletonDiscovery.py:86-106 restated literally."""
    from oracle import cpc
    from oracle import skeleton as osk
    n = 14 + seed
    names = _names(n, 40 + seed)
    F, _ = _knowledge(names, 40 + seed).masks(names)
    C = _frame_C(n, 600, 500 + seed)
    r = osk.skeleton_discovery(C, 600, forbidden=F.astype(bool))
    c = cpc.skeleton(C, 600, banned=banned_pairs(F))
    np.testing.assert_array_equal(c.removed_level, r.removed_level.astype(np.int8))
    assert c.tests == r.tests_per_level and c.calls == r.calls_per_level
    B = banned_pairs(F).astype(bool)
    assert B.any() and (r.removed_level[B] == 0).all()


def _sep_rows(r, n):
    xy, bits = [], []
    for x in range(n):
        for y in range(n):
            if x != y and r.removed_level[x, y] >= 1:
                lst = r.sepset[x, y]
                side = set(lst[-2]) if x < y else set(lst[-1])
                if side:
                    xy.append((x, y))
                    bits.append([sum(1 << int(s) for s in side)])
    return np.array(xy, np.int32).reshape(-1, 2), np.array(bits, np.uint64).reshape(-1, 1)


class _OracleCI:
    def __init__(self, C, N):
        self.C, self.N = C, N

    def pvalues(self, tests):
        from oracle import fisherz as ofz
        return [ofz.pvalue(self.C, self.N, i, j, S) for (i, j, S) in tests]

    def __call__(self, i, j, S):
        return self.pvalues([(i, j, S)])[0]


@pytest.mark.parametrize("priority,seed", [(2, 0), (2, 1), (2, 2), (2, 3), (2, 4), (3, 0), (3, 1), (4, 0)])
def test_orient_bk_host_matches_python_restatement(priority, seed):
    from oracle import orient as oor
    from oracle import skeleton as osk
    from rcaeval_amd.citest import uc_orient
    n = 12 + seed
    names = _names(n, 70 + seed)
    F, R = _knowledge(names, 70 + seed).masks(names)
    C = _frame_C(n, 500, 800 + seed)
    r = osk.skeleton_discovery(C, 500, forbidden=F.astype(bool))
    xy, bits = _sep_rows(r, n)
    ci = _OracleCI(C, 500)
    got = uc_orient(r.adj.astype(np.uint8), xy, bits, priority, ci if priority != 2 else None, knowledge=(F, R))
    want = oor.orient(r.adj, r.sepset, priority=priority, ci_test=ci, knowledge=(F, R))
    np.testing.assert_array_equal(got, want)
    # the knowledge changed something (else the test would not pin it)
    plain = oor.orient(r.adj, r.sepset, priority=priority, ci_test=ci)
    assert seed > 0 or priority != 2 or not np.array_equal(plain, want)


def test_orient_bk_required_only_and_empty_knowledge():
    """Required edges alone orient the skeleton; empty masks reproduce pcg_orient exactly."""
    from oracle import orient as oor
    from oracle import skeleton as osk
    from rcaeval_amd.engine import orient, orient_bk
    n = 13
    C = _frame_C(n, 600, 901)
    r = osk.skeleton_discovery(C, 600)
    xy, bits = _sep_rows(r, n)
    Z = np.zeros((n, n), np.uint8)
    np.testing.assert_array_equal(orient_bk(r.adj, xy, bits, Z, Z), orient(r.adj, xy, bits))
    Rq = np.zeros((n, n), np.uint8)
    a, b = np.argwhere(np.triu(r.adj, 1))[0]
    Rq[b, a] = 1
    got = orient_bk(r.adj, xy, bits, Z, Rq)
    np.testing.assert_array_equal(got, oor.orient(r.adj, r.sepset, knowledge=(Z, Rq)))
    assert got[b, a] == -1 and got[a, b] == 1
