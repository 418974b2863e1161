"""Per-phase wall-clock accounting for the RQ2 loop (off unless enabled; no effect on results).

``enable()`` turns it on for the calling thread; ``phase("name")`` brackets a region and adds its
wall time to that thread's totals; ``take()`` returns and clears them. Used by ``rq2.run`` /
``bench.py --workload rq2`` to split a case into read_csv + window, preprocess, K1 + skeleton,
orientation, PageRank, glue and JSON.
"""
from __future__ import annotations

import threading
import time
from contextlib import contextmanager

_tls = threading.local()


def enable(on: bool = True) -> None:
    _tls.on = on
    _tls.acc = {}
    _tls.cnt = {}


def enabled() -> bool:
    return getattr(_tls, "on", False)


@contextmanager
def phase(name: str):
    if not getattr(_tls, "on", False):
        yield
        return
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        _tls.acc[name] = _tls.acc.get(name, 0.0) + dt
        _tls.cnt[name] = _tls.cnt.get(name, 0) + 1


def add(name: str, seconds: float) -> None:
    if getattr(_tls, "on", False):
        _tls.acc[name] = _tls.acc.get(name, 0.0) + seconds
        _tls.cnt[name] = _tls.cnt.get(name, 0) + 1


def take() -> dict:
    """{name: (seconds, count)} accumulated on this thread since enable() / the last take()."""
    out = {k: (v, getattr(_tls, "cnt", {}).get(k, 0)) for k, v in getattr(_tls, "acc", {}).items()}
    _tls.acc = {}
    _tls.cnt = {}
    return out
