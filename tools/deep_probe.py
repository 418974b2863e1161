"""Probe the reference's default (unlimited depth) on a config-5-family SEM: run the skeleton with
max_depth = 4, 5, ... while the next depth's work fits a budget, and print per-depth stats plus the
work the next depth would need on the graph the last run left (GPU tool, not a test).

  python tools/deep_probe.py --n 2000 --samples 10000 --budget 2e11 > gpurun_out/.../probe.jsonl

For every capped run: tests / calls / max degree / edges / level_ms per depth. For the graph after
depth k: calls(k+1) = sum_x deg(x) * C(deg(x) - 1, k + 1) (the reference's ci_test invocations at
depth k + 1 if nothing more were removed: an upper bound of that depth, and of every deeper depth
once the graph stops changing), the degree histogram's tail, and 2^(D-1) for the largest degree
D (every subset of one node's other neighbours, tested once per depth d = 0..D-1 as long as one of
its edges survives: the floor of what an unlimited run has to do on that node alone).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--start", type=int, default=4)
    ap.add_argument("--budget", type=float, default=2e11, help="stop before a depth whose calls bound exceeds this")
    ap.add_argument("--max-depth", type=int, default=40)
    a = ap.parse_args()
    import torch
    from rcaeval_amd import synth
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    X = synth.gaussian_sem(a.n, a.samples, seed=a.seed)
    Xd = eng.to_device(X)
    torch.cuda.synchronize()
    k = a.start
    while k <= a.max_depth:
        t0 = time.perf_counter()
        out = eng.corr_skeleton(Xd, alpha=0.05, max_depth=k)[0]
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        st = out.stats
        rl = out.removed_level
        adj = (rl == -1)
        np.fill_diagonal(adj, False)
        deg = adj.sum(axis=1)
        nxt = k + 1
        calls_next = int(sum(int(d) * math.comb(int(d) - 1, nxt) for d in deg if d - 1 >= nxt))
        D = int(deg.max())
        line = {"n": a.n, "N": a.samples, "seed": a.seed, "max_depth": k, "levels": st["levels"], "wall_s": wall,
                "tests": st["tests"], "calls": st["calls"], "max_degree_at_start": st["max_degree"],
                "edges_after": st["edges_after"], "level_ms": [round(v, 3) for v in st["level_ms"]],
                "kernel_ms": [round(v, 3) for v in st["kernel_ms"]],
                "degree_top": sorted((int(v) for v in deg), reverse=True)[:16],
                "degree_hist": np.bincount(deg).tolist(),
                "next_depth_calls_bound": calls_next, "floor_largest_node_2^(D-1)": 2 ** max(D - 1, 0)}
        print(json.dumps(line), flush=True)
        if st["levels"] <= k:        # the loop ended by itself: this was the unlimited run
            print(json.dumps({"done": True, "unlimited_levels": st["levels"], "total_tests": int(sum(st["tests"]))}),
                  flush=True)
            return
        if calls_next > a.budget:
            print(json.dumps({"stopped": True, "reason": f"depth {nxt} bound {calls_next:.3e} calls > budget"}),
                  flush=True)
            return
        k += 1


if __name__ == "__main__":
    main()
