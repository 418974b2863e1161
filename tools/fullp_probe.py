"""Full-p mode (PCG_FLAG_FULL_P | PCG_FLAG_RECORD, 1-in-4099 pair sample) on config 5: per-level
times, exact-path counts and the wall time of the call (GPU tool, not a test; run it under
rocprofv3 --kernel-trace --stats for the per-kernel split).

usage: python tools/fullp_probe.py [--reps 3] [--sample 4099]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sample", type=int, default=4099)
    a = ap.parse_args()
    import torch
    from rcaeval_amd import _lib, synth
    from rcaeval_amd.engine import get_engine
    eng = get_engine(0)
    X = synth.gaussian_sem(2000, 10000, seed=0)
    C = eng.corr(X)
    fl = _lib.PCG_FLAG_FULL_P | _lib.PCG_FLAG_RECORD
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = eng.skeleton(C, 10000, max_depth=4, flags=fl, record_capacity=4_000_000, record_sample=(a.sample, 17))
        torch.cuda.synchronize()
        wall = 1000 * (time.perf_counter() - t0)
        print(json.dumps({"rep": r, "wall_ms": round(wall, 3), "device_ms": round(o.device_ms, 3),
                          "level_ms": [round(v, 3) for v in o.stats["level_ms"]],
                          "kernel_ms": [round(v, 3) for v in o.stats["kernel_ms"]],
                          "exact": o.stats["exact"], "records": int(len(o.records))}), flush=True)


if __name__ == "__main__":
    main()
