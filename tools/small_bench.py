"""Time one RQ2-shaped case on the engine (GPU tool): K1 alone, the skeleton alone (small-graph
kernel vs the level loop, PCG_SMALL), K1 + skeleton in one call, and pc() end to end.

  python tools/small_bench.py [n] [N] [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 44
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    import torch
    from rcaeval_amd import synth
    from rcaeval_amd.causal import pc
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    X = synth.gaussian_sem(n, N, seed=1, w_low=0.2, w_high=0.8, edge_prob=0.1)
    Xd = eng.to_device(X)
    C = eng.corr(Xd)

    def t(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / reps

    res = {"n": n, "N": N, "corr_ms": t(lambda: eng.corr(Xd))}
    for small in (1, 0):
        # the knob is read once per handle (pcg_create): set it on the live handle
        with eng.tuned(SMALL=small):
            res[f"skeleton_ms_small{small}"] = t(lambda: eng.skeleton(C, N))
            res[f"corr_skeleton_ms_small{small}"] = t(lambda: eng.corr_skeleton(Xd))
            res[f"pc_ms_small{small}"] = t(lambda: pc(X))
            out = eng.skeleton(C, N)
        res[f"levels_small{small}"] = out.stats["levels"]
        res[f"driver_small{small}"] = out.stats["driver"]
        res[f"kernel_ms_small{small}"] = [round(v, 4) for v in out.stats["kernel_ms"]]
    print(res, flush=True)




def profile_pc(n=44, N=600, reps=300):
    """cProfile of pc() on one RQ2-shaped case (where the host time of a small case goes)."""
    import cProfile
    import pstats
    from rcaeval_amd import synth
    from rcaeval_amd.causal import pc
    X = synth.gaussian_sem(n, N, seed=1, w_low=0.2, w_high=0.8, edge_prob=0.1)
    for _ in range(10):
        pc(X)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        pc(X)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    if "--profile" in sys.argv:
        profile_pc()
    else:
        main()
