"""Full-depth skeleton (the reference's default: no depth cap) on the config-5 SEM family at
n variables: per-level tests, level and kernel times, total GPU time (one warm-up, then the
median of --reps timed runs). Used under rocprofv3 --kernel-trace --stats for the per-kernel
breakdown of the deep levels.

usage: python tools/profile_deep.py [--n 500] [--samples 10000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--max-depth", type=int, default=-1)
    args = ap.parse_args()
    import numpy as np
    import torch
    from rcaeval_amd import synth
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    X = synth.gaussian_sem(args.n, args.samples, seed=0)
    C = np.corrcoef(X.T)
    Cd = eng.to_device(C)
    out = eng.skeleton(Cd, args.samples, max_depth=args.max_depth)
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        out = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.skeleton(Cd, args.samples, max_depth=args.max_depth)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    st = out.stats
    print(json.dumps({"n": args.n, "N": args.samples, "levels": st["levels"], "gpu_ms": 1e3 * float(np.median(times)),
                      "gpu_ms_all": [round(1e3 * t, 3) for t in times], "tests": st["tests"],
                      "unique_tests": int(sum(st["tests"])), "level_ms": [round(v, 4) for v in st["level_ms"]],
                      "kernel_ms": [round(v, 4) for v in st["kernel_ms"]], "max_degree": st["max_degree"],
                      "exact": st["exact"]}), flush=True)


if __name__ == "__main__":
    main()
