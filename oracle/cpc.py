"""ctypes binding of ``pc_oracle.c`` (C restatement of the stable PC-fisherz skeleton).

TEST INFRASTRUCTURE ONLY — used by tests/, smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OrcStats(ctypes.Structure):
    _fields_ = [("tests", ctypes.c_int64 * 32), ("calls", ctypes.c_int64 * 32),
                ("indep", ctypes.c_int64 * 32), ("levels", ctypes.c_int32),
                ("error", ctypes.c_int32), ("secs", ctypes.c_double * 32)]


REC_DTYPE = np.dtype([("a", np.int32), ("b", np.int32), ("d", np.int32),
                      ("s", np.int32, 12), ("p", np.float64)], align=True)


def build() -> str:
    path = os.path.join(_HERE, "liborc.so")
    src = os.path.join(_HERE, "pc_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liborc.so"])
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        P = ctypes.c_void_p
        _LIB.orc_skeleton.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                      P, P, P, P, ctypes.c_int64, P, P, ctypes.c_int64, P, P, ctypes.c_int]
        _LIB.orc_skeleton.restype = ctypes.c_int
        _LIB.orc_skeleton_bk.argtypes = _LIB.orc_skeleton.argtypes + [P]
        _LIB.orc_skeleton_bk.restype = ctypes.c_int
        _LIB.orc_fisherz_batch.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int,
                                           ctypes.c_int64, P, P]
        _LIB.orc_corrcoef.argtypes = [P, ctypes.c_int64, ctypes.c_int, P]
        _LIB.orc_level_sample.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
        _LIB.orc_level_sample.restype = ctypes.c_int
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


@dataclass
class CSkeleton:
    removed_level: np.ndarray    # n x n int8
    deg_at_level: np.ndarray     # levels x n int32
    side_union: np.ndarray       # n x n x W uint64 or None
    records: np.ndarray          # REC_DTYPE or None
    near_alpha: np.ndarray       # REC_DTYPE: every unique test with |p - alpha| < 1e-9
    tests: list
    calls: list
    indep: list
    levels: int
    error: int
    secs: list = None            # wall seconds per depth

    @property
    def adj(self) -> np.ndarray:
        n = self.removed_level.shape[0]
        return (self.removed_level == -1) & ~np.eye(n, dtype=bool)


def skeleton(C: np.ndarray, N: int, alpha: float = 0.05, max_depth: int = -1,
             want_union: bool = True, record_cap: int = 0, nthreads: int = 0, banned=None) -> CSkeleton:
    """``banned``: n x n pairs forbidden both ways by background knowledge (removed at depth 0)."""
    C = np.ascontiguousarray(C, dtype=np.float64)
    bn = None if banned is None else np.ascontiguousarray(banned, dtype=np.uint8)
    n = C.shape[0]
    W = (n + 63) // 64
    rl = np.empty((n, n), np.int8)
    deg = np.zeros((32, n), np.int32)
    su = np.empty((n, n, W), np.uint64) if want_union else None
    rec = np.empty(record_cap, REC_DTYPE) if record_cap else None
    cnt = np.zeros(1, np.int64)
    near_cap = 1 << 16
    near = np.empty(near_cap, REC_DTYPE)
    ncnt = np.zeros(1, np.int64)
    st = OrcStats()
    lib().orc_skeleton_bk(_p(C), n, int(N), float(alpha), int(max_depth), _p(rl), _p(deg), _p(su),
                          _p(rec), int(record_cap), _p(cnt), _p(near), near_cap, _p(ncnt),
                          ctypes.byref(st), int(nthreads), _p(bn))
    L = st.levels
    if rec is not None:
        if cnt[0] > record_cap:
            raise RuntimeError(f"record buffer overflow: {cnt[0]} > {record_cap}")
        rec = rec[: cnt[0]]
    if ncnt[0] > near_cap:
        raise RuntimeError(f"near-alpha buffer overflow: {ncnt[0]} > {near_cap}")
    return CSkeleton(rl, deg[:L].copy(), su, rec, near[: ncnt[0]].copy(), list(st.tests[:L]),
                     list(st.calls[:L]), list(st.indep[:L]), L, st.error, list(st.secs[:L]))


def level_sample(C: np.ndarray, N: int, removed_level: np.ndarray, d: int, x0: int = 0, xstep: int = 1,
                 alpha: float = 0.05, nthreads: int = 0):
    """Time depth ``d``'s visits of nodes x0, x0+xstep, ... on the graph at the start of
    depth d (pairs with removed_level -1 or >= d): (unique tests, seconds)."""
    C = np.ascontiguousarray(C, dtype=np.float64)
    rl = np.ascontiguousarray(removed_level, dtype=np.int8)
    tests = np.zeros(1, np.int64)
    secs = np.zeros(1, np.float64)
    err = lib().orc_level_sample(_p(C), C.shape[0], int(N), float(alpha), _p(rl), int(d), int(x0), int(xstep),
                                 int(nthreads), _p(tests), _p(secs))
    if err:
        raise RuntimeError(f"orc_level_sample error {err}")
    return int(tests[0]), float(secs[0])


def corrcoef(data: np.ndarray) -> np.ndarray:
    X = np.ascontiguousarray(data, dtype=np.float64)
    N, n = X.shape
    C = np.empty((n, n), np.float64)
    lib().orc_corrcoef(_p(X), N, n, _p(C))
    return C


def fisherz_batch(C: np.ndarray, N: int, ab: np.ndarray, S: np.ndarray, d: int):
    """FisherZ p of explicit canonical tests (a < b, S sorted, all of size d): (p, err)."""
    C = np.ascontiguousarray(C, dtype=np.float64)
    ab = np.ascontiguousarray(ab, dtype=np.int32).reshape(-1, 2)
    count = len(ab)
    S = np.ascontiguousarray(S, dtype=np.int32).reshape(count, max(d, 1))
    p = np.empty(count, np.float64)
    err = np.empty(count, np.int32)
    lib().orc_fisherz_batch(_p(C), C.shape[0], int(N), _p(ab), _p(S), int(d), count, _p(p), _p(err))
    return p, err
