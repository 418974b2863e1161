"""The PC / FCI golden cases: seeded inputs and their digests. Shared by the tests (which rebuild
each input and check its digest against ``skeleton_ref.json``) and by the manual generator
``make_skeleton_golden.py``; the tests import only this module, never the generator."""
from __future__ import annotations

import hashlib

import numpy as np

# name: (n, N, seed, w_low, w_high, edge_prob, options)
#   stable      SkeletonDiscovery(stable=...)
#   const       column index set to a constant (NaN correlations, never separated)
#   dup         (a, b): column b := column a (exactly singular sub-matrices -> ValueError)
#   forbid      [(i, j), ...] background knowledge: i -> j forbidden (pairs listed both ways are
#               banned edges, SkeletonDiscovery.py:88-106)
PC_CASES = {
    "p12": (12, 500, 1, .3, .9, .3, {}),
    "p20": (20, 800, 2, .2, .8, .2, {}),
    "p30": (30, 600, 3, .3, .9, .15, {}),
    "p25": (25, 300, 9, .1, .5, .3, {}),
    "p18": (18, 250, 11, .4, .9, .35, {}),
    "p15deep": (15, 3000, 4, .5, 1.0, .45, {}),
    "p32multi": (32, 400, 3, .1, .3, .3, {}),
    "u20": (20, 800, 2, .2, .8, .2, {"stable": False}),
    "u30": (30, 600, 3, .3, .9, .15, {"stable": False}),
    "u18": (18, 250, 11, .4, .9, .35, {"stable": False}),
    "const11": (11, 400, 31, .3, .9, .3, {"const": 4}),
    "bk20": (20, 800, 2, .2, .8, .2, {"forbid": [(0, 1), (1, 0), (3, 7), (7, 3), (5, 6), (2, 9), (9, 2)]}),
    "dup12": (12, 500, 1, .3, .9, .3, {"dup": (2, 7)}),
}
# name: (n, N, seed, w_low, w_high, edge_prob, depth)
FCI_CASES = {
    "f12": (12, 500, 1, .3, .9, .3, -1),
    "f20": (20, 800, 2, .2, .8, .2, -1),
    "f30": (30, 600, 3, .3, .9, .15, -1),
    "f25": (25, 300, 9, .1, .5, .3, -1),
    "f18": (18, 250, 11, .4, .9, .35, -1),
    "f20d1": (20, 800, 2, .2, .8, .2, 1),
    "f20d2": (20, 800, 2, .2, .8, .2, 2),
}


def pc_input(name):
    """The seeded N x n input of one PC case (tests rebuild it the same way)."""
    from rcaeval_amd import synth
    n, N, seed, wl, wh, ep, opt = PC_CASES[name]
    X = synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)
    if "const" in opt:
        X[:, opt["const"]] = 1.0
    if "dup" in opt:
        a, b = opt["dup"]
        X[:, b] = X[:, a]
    return np.ascontiguousarray(X)


def fci_input(name):
    from rcaeval_amd import synth
    n, N, seed, wl, wh, ep, _ = FCI_CASES[name]
    return synth.gaussian_sem(n, N, seed=seed, w_low=wl, w_high=wh, edge_prob=ep)


def digest(a) -> str:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return hashlib.sha256(a.tobytes() + str(a.shape).encode()).hexdigest()
