"""CloudRanger's second-order random walk head — ``relaToRank`` / ``guiyi`` /
``secondorder_randomwalk`` of ``RCAEval/e2e/cloudranger.py:69-148`` restated without the
O(n³) Python loops.

Transition tensor ``M[k, i, j]`` = probability of stepping i → j having arrived at i from k:
forward edges of the dependency graph ``access`` weighted ``(1−β)·P[k, i] + β·P[i, j]``
(``:113-122``), backward edges ``ρ·((1−β)·P[k, i] + β·P[j, i])`` normalised over the in-nodes
(``:124-133``), a self edge ``max(0, S[i] − max_{j≠i} M[k, i, j])`` where none exists
(``:135-140``), then every row normalised (``:142-146``). ``P`` is ``|S[j]|`` on the access
pattern, row-normalised by ``guiyi`` (``:91-101``), with ``S = rela[frontend − 1]`` — the row
*before* the SLI's (index −1, i.e. the last row, when the SLI is column 0), as in the reference.

Bitwise parity with the loops: every sum the reference takes (``np.sum`` of a row, of a
row's gathered in-node entries) is taken here over the same contiguous elements in the same
order, so numpy's pairwise reduction tree is identical; the per-row ``max`` keeps Python's
first-maximum / NaN semantics. The walk draws from numpy's global legacy ``RandomState`` like
the reference (``np.random.choice(range(n), p=row)``): the first visit of each ``(previous,
current)`` row goes through ``np.random.choice`` itself (numpy's own validation and one draw),
later visits reuse that row's normalised cdf with one ``random_sample()`` each — the same stream
consumption and the same index (``cdf.searchsorted(u, 'right')``).
"""
from __future__ import annotations

import numpy as np


def guiyi(p) -> np.ndarray:
    """``cloudranger.py:91-101``: row-normalise; rows summing to 0 stay 0."""
    p = np.asarray(p, dtype=float)
    s = np.sum(p, axis=1)
    out = np.zeros_like(p)
    live = ~(s == 0)
    out[live] = p[live] / s[live, None]
    return out


def _builtin_max_excluding_diag(M: np.ndarray) -> np.ndarray:
    """``max(M[k, i, j] for j != i)`` with Python's ``max`` semantics (first maximum wins,
    NaN never replaced / never replacing) for every (k, i)."""
    n = M.shape[0]
    if n < 2:
        raise ValueError("max() arg is an empty sequence")
    first = np.where(np.arange(n) == 0, 1, 0)               # first j != i
    res = np.take_along_axis(M, np.broadcast_to(first[None, :, None], (n, n, 1)), axis=2)[:, :, 0].copy()
    for j in range(n):
        col = M[:, :, j]
        upd = (col > res)
        upd[:, j] = False                                    # j == i is excluded
        res = np.where(upd, col, res)
    return res


def transition_tensor(rela, access, frontend: int, beta: float = 0.1, rho: float = 0.3):
    """``relaToRank`` (``cloudranger.py:104-146``) up to the walk: returns (P, M)."""
    access = np.asarray(access)
    n = len(access)
    rela = np.asarray(rela, dtype=float)
    S = rela[frontend - 1]
    P = guiyi(np.where(access != 0, np.abs(S)[None, :], 0.0))
    # forward edges, normalised over out-nodes
    fwd = access > 0
    M = np.where(fwd[None, :, :], (1 - beta) * P[:, :, None] + beta * P[None, :, :], 0.0)
    s = M.sum(axis=2)
    M = np.where((s > 0)[:, :, None], M / np.where(s > 0, s, 1.0)[:, :, None], M)
    # backward edges, normalised over in-nodes (gathered in ascending j, like in_inds)
    back = (access == 0) & (access.T != 0)
    for i in range(n):
        ins = np.nonzero(back[i])[0]
        if ins.size == 0:
            continue
        B = rho * ((1 - beta) * P[:, i][:, None] + beta * P[ins, i][None, :])
        bs = B.sum(axis=1)
        M[:, i, ins] = np.where((bs > 0)[:, None], B / np.where(bs > 0, bs, 1.0)[:, None], B)
    # self edges where none exists
    diag = M[:, np.arange(n), np.arange(n)]                  # (k, i)
    need = diag == 0
    if need.any():
        x = S[None, :] - _builtin_max_excluding_diag(M)
        val = np.where(x > 0, x, 0.0)
        kk, ii = np.nonzero(need)
        M[kk, ii, ii] = val[kk, ii]
    s = M.sum(axis=2)
    M = np.where((s > 0)[:, :, None], M / np.where(s > 0, s, 1.0)[:, :, None], M)
    return P, M


def secondorder_randomwalk(M: np.ndarray, epochs: int, start_node: int, label=(), walk_step: int = 1000,
                           print_trace: bool = False):
    """``cloudranger.py:69-88`` on numpy's global RandomState (see module docstring);
    ``print_trace`` is accepted and ignored (debug output only)."""
    n = M.shape[0]
    score = np.zeros([n])
    cdfs = {}
    for _ in range(epochs):
        previous = current = start_node - 1
        for _ in range(walk_step):
            row = M[previous, current]
            if np.sum(row) == 0:
                break
            key = (previous % n, current % n)
            cdf = cdfs.get(key)
            if cdf is None:
                nxt = int(np.random.choice(range(n), p=row))
                cdf = row.cumsum()
                cdf /= cdf[-1]
                cdfs[key] = cdf
            else:
                nxt = int(cdf.searchsorted(np.random.random_sample(), side="right"))
            score[nxt] += 1
            previous, current = current, nxt
    out = list(zip(label, score))
    out.sort(key=lambda x: x[1], reverse=True)
    return out


def relaToRank(rela, access, rankPaces, frontend, beta=0.1, rho=0.3, print_trace=False):
    """``cloudranger.py:104-148``: (ranked [(label, visits)], P, M)."""
    P, M = transition_tensor(rela, access, frontend, beta=beta, rho=rho)
    label = list(range(1, len(access) + 1))
    return secondorder_randomwalk(M, rankPaces, frontend, label), P, M


__all__ = ["guiyi", "transition_tensor", "secondorder_randomwalk", "relaToRank"]
