"""CPU: the oracles pinned to the REFERENCE's own skeleton loop and FCI, executed.

``tests/golden/skeleton_ref.json`` holds outputs of the vendored causal-learn code run under
python3.9 (``tests/golden/make_skeleton_golden.py``: ``SkeletonDiscovery.skeleton_discovery``
with the vendored ``CausalGraph``, ``Fas.fas`` and ``FCI.fci``; the absent causal-learn names
replaced by stand-ins, FisherZ as the numpy/scipy library-call expression). Here the numpy
restatement (``oracle/skeleton.py``), the C restatement (``oracle/pc_oracle.c``), the orientation
oracle's triple / triangle / kite enumerations (``oracle/orient.py``) and the FCI restatement
(``oracle/fci.py``) are checked against those outputs: graph, every sepset list, every p_values
list, the memo size and call count per depth, and the reference's ValueError on a singular
sub-matrix.
"""
import json
import os

import numpy as np
import pytest

from oracle import cpc
from oracle import fci as ofci
from oracle import fisherz
from oracle import orient as oor
from oracle import skeleton as osk
from tests.golden import skeleton_cases as mk

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "skeleton_ref.json")))
PC = GOLD["pc"]
FCI = GOLD["fci"]


def _input(name):
    X = mk.pc_input(name)
    assert mk.digest(X) == PC[name]["digest"], "input generator drifted from the golden's"
    with np.errstate(invalid="ignore", divide="ignore"):
        return X, np.corrcoef(X.T)


def _forbidden(name, n):
    f = np.zeros((n, n), dtype=bool)
    for i, j in PC[name]["opt"].get("forbid", []):
        f[i, j] = True
    return f


def _levels(rec):
    """Adjacency after each depth from the golden's while-condition snapshots."""
    n = rec["n"]
    out = []
    for s in rec["levels"]:
        bits = np.unpackbits(np.frombuffer(bytes.fromhex(s["adj_bits"]), np.uint8))[: n * n]
        out.append(bits.reshape(n, n).astype(bool))
    return out


def _same_p(a, b):
    """The north-star p tolerance (|dp| <= 1e-9 |p| + 2^-51): the golden ran numpy 1.26's LAPACK
    under python3.9, this interpreter numpy 2.x's; the inverses differ in the last bits."""
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and bool(np.all(fisherz.p_close(a, b)))


OK_CASES = [k for k, v in PC.items() if "error" not in v]


def test_golden_covers_the_reference_options():
    opts = [v["opt"] for v in PC.values()]
    assert any(o.get("stable") is False for o in opts)
    assert any("forbid" in o for o in opts) and any("const" in o for o in opts)
    assert any("error" in v for v in PC.values())
    assert max(len(v["levels"]) for v in PC.values() if "levels" in v) >= 10      # deep unlimited runs
    # unions from several independent S at one visit (|union| > depth of that visit)
    rec = PC["p32multi"]
    assert any(len(t) > 1 for lst in rec["sepset"].values() for t in lst)


@pytest.mark.parametrize("name", OK_CASES)
def test_numpy_oracle_equals_reference_loop(name):
    rec = PC[name]
    X, C = _input(name)
    n, N = rec["n"], rec["N"]
    stable = rec["opt"].get("stable", True)
    forb = _forbidden(name, n) if "forbid" in rec["opt"] else None
    with np.errstate(invalid="ignore", divide="ignore"):
        r = osk.skeleton_discovery(C, N, stable=stable, forbidden=forb)
    g = np.asarray(rec["graph"])
    np.testing.assert_array_equal(r.adj, g != 0)
    np.testing.assert_array_equal(osk.endpoint_graph(r.adj), g)
    for i in range(n):
        for j in range(n):
            key = f"{i},{j}"
            want = rec["sepset"].get(key)
            got = r.sepset[i, j]
            assert (got is None) == (want is None), key
            if want is not None:
                assert [list(map(int, t)) for t in got] == want, key
            want_p = rec["p_values"].get(key)
            got_p = r.p_values[i, j]
            assert (got_p is None) == (want_p is None), key
            if want_p is not None:
                assert _same_p(got_p, want_p), key
    assert len(r.cache) == rec["unique_tests"]
    assert sum(r.calls_per_level) == rec["no_ci_tests"]
    # per depth: the memo growth and call count, and the adjacency each depth left
    lv = rec["levels"]
    assert len(r.tests_per_level) == len(lv) - 1
    for d in range(len(lv) - 1):
        assert r.tests_per_level[d] == lv[d + 1]["unique"] - lv[d]["unique"], d
        assert r.calls_per_level[d] == lv[d + 1]["calls"] - lv[d]["calls"], d


@pytest.mark.parametrize("name", [k for k in OK_CASES if PC[k]["opt"].get("stable", True)])
def test_numpy_oracle_depth_caps_equal_reference_snapshots(name):
    """max_depth = k stops where the reference's loop stood after depth k."""
    rec = PC[name]
    X, C = _input(name)
    forb = _forbidden(name, rec["n"]) if "forbid" in rec["opt"] else None
    snaps = _levels(rec)
    for k in range(len(snaps) - 1):
        with np.errstate(invalid="ignore", divide="ignore"):
            r = osk.skeleton_discovery(C, rec["N"], max_depth=k, forbidden=forb)
        np.testing.assert_array_equal(r.adj, snaps[k + 1], err_msg=f"depth {k}")


@pytest.mark.parametrize("name", [k for k in OK_CASES if PC[k]["opt"].get("stable", True)])
def test_c_oracle_equals_reference_loop(name):
    """pc_oracle.c: removal depths from the snapshots, unique tests and calls per depth, and the
    per-side unions (the last sepset entry each side appended) of every removed pair."""
    rec = PC[name]
    X, C = _input(name)
    n = rec["n"]
    banned = None
    if "forbid" in rec["opt"]:
        f = _forbidden(name, n)
        banned = f & f.T
    with np.errstate(invalid="ignore", divide="ignore"):
        r = cpc.skeleton(C, rec["N"], banned=banned)
    assert r.error == 0
    snaps = _levels(rec)
    lv = rec["levels"]
    assert r.levels == len(lv) - 1
    want_rl = np.full((n, n), -1)
    for d in range(len(snaps) - 1):
        want_rl[snaps[d] & ~snaps[d + 1]] = d
        assert r.tests[d] == lv[d + 1]["unique"] - lv[d]["unique"], d
        assert r.calls[d] == lv[d + 1]["calls"] - lv[d]["calls"], d
    np.testing.assert_array_equal(r.removed_level, want_rl)
    for x in range(n):
        for y in range(n):
            d = want_rl[x, y]
            if x == y or d < 1:
                continue
            # x's visit of y at depth d is x's last append to sepset[x, y]; y's visit of x is the
            # last append to sepset[y, x]: entry -2 / -1 of the list by visit order (x < y first)
            lst = rec["sepset"][f"{x},{y}"]
            side = lst[-2] if x < y else lst[-1]
            bits = r.side_union[x, y]
            got = sorted(j for j in range(n) if (int(bits[j >> 6]) >> (j & 63)) & 1)
            assert got == sorted(side), (x, y)


def test_reference_raises_on_singular_submatrix_and_oracles_agree():
    rec = PC["dup12"]
    assert rec["error"]["type"] == "ValueError" and "singular" in rec["error"]["message"]
    X, C = _input("dup12")
    with pytest.raises(ValueError, match="singular"):
        osk.skeleton_discovery(C, rec["N"])
    with np.errstate(invalid="ignore", divide="ignore"):
        r = cpc.skeleton(C, rec["N"])
    assert r.error != 0
    # the reference raised during the depth its loop had started
    assert r.levels == rec["error"]["levels_started"] or r.levels + 1 == rec["error"]["levels_started"]


@pytest.mark.parametrize("name", OK_CASES)
def test_orientation_enumerations_equal_reference(name):
    """oracle/orient.py's triple / triangle / kite lists (the order UCSepset and Meek consume
    them in) equal the vendored CausalGraph's on the reference's own skeleton."""
    rec = PC[name]
    G = oor._G(np.asarray(rec["graph"]))
    assert [list(map(int, t)) for t in G.find_unshielded_triples()] == rec["unshielded_triples"]
    assert [list(map(int, t)) for t in G.find_triangles()] == rec["triangles"]
    assert [list(map(int, t)) for t in G.find_kites()] == rec["kites"]


def _fci_input(name):
    X = mk.fci_input(name)
    assert mk.digest(X) == FCI[name]["digest"]
    return X, np.corrcoef(X.T)


@pytest.mark.parametrize("name", list(FCI))
def test_fas_oracle_equals_reference(name):
    rec = FCI[name]
    X, C = _fci_input(name)
    n = C.shape[0]
    nodes = [ofci.Node(f"X{i + 1}", i) for i in range(n)]
    g, sep = ofci.fas(nodes, ofci.CITest(C, X.shape[0]), depth=rec["depth"])
    np.testing.assert_array_equal(g.graph, np.asarray(rec["fas_graph"]))
    assert sorted([int(a), int(b), sorted(map(int, s))] for (a, b), s in sep.items()) == rec["fas_sep_sets"]


@pytest.mark.parametrize("name", list(FCI))
def test_fci_oracle_equals_reference(name):
    rec = FCI[name]
    X, C = _fci_input(name)
    want, _, _ = ofci.fci(C, X.shape[0], depth=rec["depth"])
    np.testing.assert_array_equal(want, np.asarray(rec["graph"]))
