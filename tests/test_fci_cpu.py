"""CPU: FCI — the vendored-spec oracle (oracle/fci.py) against the PC
oracle and against the drop-in's matrix-form rules (rcaeval_amd.fci) driven by the same CPU
CI test. Parity with causal-learn 0.1.3.3 itself is unpinned (the package is absent)."""
import numpy as np
import pytest

from oracle import fci as ofci
from oracle import fisherz
from oracle import skeleton as osk
from rcaeval_amd import synth

CASES = [(12, 500, 1, .3, .9, .3), (20, 800, 2, .2, .8, .2), (30, 600, 3, .3, .9, .15), (25, 300, 9, .1, .5, .3),
         (40, 2000, 5, .2, .6, .1), (18, 250, 11, .4, .9, .35)]


class CpuCI:
    """CITester stand-in (test only): the oracle FisherZ behind the cache-key memo."""

    def __init__(self, C, N):
        self.C, self.N, self.cache = C, N, {}

    def pvalues(self, tests):
        out = []
        for i, j, S in tests:
            a, b = (int(i), int(j)) if i < j else (int(j), int(i))
            key = (a, b, frozenset(int(s) for s in S))
            if key not in self.cache:
                self.cache[key] = fisherz.pvalue(self.C, self.N, a, b, tuple(sorted(key[2])))
            out.append(self.cache[key])
        return out

    def __call__(self, i, j, S):
        return self.pvalues([(i, j, S)])[0]


class FakeOut:
    """SkeletonOut stand-in built from the PC oracle's per-side unions (test only)."""

    def __init__(self, ref, n):
        self.removed_level = ref.removed_level
        W = (n + 63) // 64
        xy, bits = [], []
        for x in range(n):
            for y in range(n):
                if x == y or ref.removed_level[x, y] < 1:
                    continue
                lst = ref.sepset[x, y]
                # entries at the removal depth: x's visit then y's visit (a < b order of appends)
                side = set(int(v) for v in (lst[-2] if x < y else lst[-1]))
                if side:
                    row = np.zeros(W, np.uint64)
                    for v in side:
                        row[v >> 6] |= np.uint64(1 << (v & 63))
                    xy.append((x, y))
                    bits.append(row)
        self.sep_xy = np.array(xy, np.int32).reshape(-1, 2)
        self.sep_bits = np.array(bits, np.uint64).reshape(-1, W)
        adj = ref.removed_level == -1
        np.fill_diagonal(adj, False)
        self.adj = adj


def _data(n, N, seed, wl, wh, ep):
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    return np.corrcoef(X.T), N


@pytest.mark.parametrize("case", CASES)
def test_fas_equals_stable_pc_skeleton_and_sep_sets_rule(case):
    from rcaeval_amd.fci import fas_sep_sets
    C, N = _data(*case)
    n = C.shape[0]
    nodes = [ofci.Node(f"X{i + 1}", i) for i in range(n)]
    g, sep = ofci.fas(nodes, ofci.CITest(C, N))
    ref = osk.skeleton_discovery(C, N)
    np.testing.assert_array_equal(g.graph != 0, ref.adj)
    assert fas_sep_sets(FakeOut(ref, n)) == sep


@pytest.mark.parametrize("case", CASES)
def test_fci_orientation_matches_vendored_restatement(case):
    from rcaeval_amd.fci import fas_sep_sets, fci_orient
    C, N = _data(*case)
    n = C.shape[0]
    want, sep_ref, _ = ofci.fci(C, N)
    ref = osk.skeleton_discovery(C, N)
    out = FakeOut(ref, n)
    got = fci_orient(out.adj, fas_sep_sets(out), CpuCI(C, N), fas_last=ref.max_depth_run)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_fci_depth_cap_evaluates_possible_dsep_sizes(depth):
    """fci(depth=k): FAS runs depths 0..k-1 and Possible-D-Sep tests the size k it left."""
    from rcaeval_amd.fci import fas_sep_sets, fci_orient
    C, N = _data(20, 800, 2, .2, .8, .2)
    n = C.shape[0]
    want, _, _ = ofci.fci(C, N, depth=depth)
    if depth == 0:
        adj, sep, last = np.zeros((n, n), dtype=bool), {}, -1   # FAS ran no depth: no edges
    else:
        ref = osk.skeleton_discovery(C, N, max_depth=depth - 1)
        out = FakeOut(ref, n)
        adj, sep, last = out.adj, fas_sep_sets(out), ref.max_depth_run
    got = fci_orient(adj, sep, CpuCI(C, N), depth=depth, fas_last=last)
    np.testing.assert_array_equal(got, want)
