"""Random-walk head restatement + PCG64 replica — tests only.

``walk_counts`` restates ``RandomWalkScorer._walk`` (RCAEval/graph_heads/random_walk.py:179-186)
with numpy's own Generator (the reference draws from ``default_rng(0)``, :148);
``pcg64_doubles`` is a pure-Python PCG64 (XSL-RR 128/64) replica used to check the HIP
kernel's jump-ahead arithmetic against numpy's bit generator.
"""
from __future__ import annotations

import numpy as np

MULT = 0x2360ED051FC65DA44385DF649FCCF645
MASK128 = (1 << 128) - 1


def walk_counts(P: np.ndarray, start: int, num_loop: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    m = P.shape[0]
    counts = np.zeros(m, np.int64)
    idx = np.arange(m)
    node = start
    for _ in range(num_loop):
        node = int(rng.choice(idx, p=P[:, node]))
        counts[node] += 1
    return counts


def pcg64_doubles(state: int, inc: int, k: int) -> list:
    out = []
    for _ in range(k):
        state = (state * MULT + inc) & MASK128
        rot = state >> 122
        xs = ((state >> 64) ^ state) & ((1 << 64) - 1)
        v = ((xs >> rot) | (xs << ((64 - rot) & 63))) & ((1 << 64) - 1)
        out.append((v >> 11) * (1.0 / 9007199254740992.0))
    return out
