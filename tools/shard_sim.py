"""Estimate edge-sharded scaling on ONE GPU: per depth, run every rank's chunk range of the
work split back to back (so the skeleton is complete and identical), time each range with
HIP events, and report sum over depths of max-over-ranks kernel time per world size.

usage: python tools/shard_sim.py [n] [samples]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from rcaeval_amd import synth
from rcaeval_amd._lib import PcgStats, check
from rcaeval_amd.dist import split_by_work
from rcaeval_amd.engine import get_engine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
eng = get_engine(0)
lib, h = eng.lib, eng.h
X = synth.gaussian_sem(n, N, seed=0)
C = eng.corr(X)
torch.cuda.synchronize()
for world in (1, 2, 4, 8):
    rl = torch.empty((n, n), dtype=torch.int8, device=eng.device)
    check(h, lib.pcg_skeleton_init(h, ctypes.c_void_p(C.data_ptr()), n, n, N, 0.05, 0,
                                   ctypes.c_void_p(rl.data_ptr())), "init")
    st = PcgStats()
    per_level = []
    for depth in range(5):
        total, md, rmp = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_void_p()
        rc = lib.pcg_level_begin(h, depth, ctypes.byref(total), ctypes.byref(md), ctypes.byref(rmp))
        if rc == 1:
            break
        check(h, rc, "begin")
        prefix = np.zeros(total.value + 1, np.int64)
        check(h, lib.pcg_level_chunk_work(h, prefix.ctypes.data_as(ctypes.c_void_p), len(prefix)), "work")
        ts = []
        for r in range(world):
            lo, hi = split_by_work(prefix, r, world)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            check(h, lib.pcg_level_run(h, lo, hi), "run")
            torch.cuda.synchronize()
            ts.append(1000 * (time.perf_counter() - t0))
        check(h, lib.pcg_level_end(h, ctypes.byref(st)), "end")
        per_level.append((max(ts), min(ts), sum(ts)))
    tot_max = sum(p[0] for p in per_level)
    print(f"world {world}: sum_depth max_rank run ms = {tot_max:.2f}  per depth (max/min/sum) = "
          + " ".join(f"{a:.2f}/{b:.2f}/{c:.2f}" for a, b, c in per_level), flush=True)
