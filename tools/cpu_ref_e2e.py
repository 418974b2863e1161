"""the reference-equivalent CPU skeleton end to end at n in {50, 200, 500}.

causal-learn's stable PC is single-threaded Python doing, per unique test, an ix_ gather,
numpy.linalg.inv, math.log and scipy's norm.cdf behind a dict memo; oracle/skeleton.py is that
loop (SkeletonDiscovery.py:70-144 + the FisherZ expression) and is timed here on one core
(OMP/OpenBLAS threads = 1) on the config-5 SEM family (N = 10 000, seed 0), next to the GPU
engine on the same correlation matrix. Writes one JSON object (stdout and --out).

usage: OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python tools/cpu_ref_e2e.py [--out F] [--ns 50 200 500]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", type=int, nargs="+", default=[50, 200, 500])
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-gpu", action="store_true")
    args = ap.parse_args()
    import threading

    import numpy as np
    from oracle import skeleton as osk

    def heartbeat():      # the GPU pool kills commands silent for 3 minutes
        t0 = time.perf_counter()
        while True:
            time.sleep(20)
            print(f"[cpu_ref_e2e] {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    from rcaeval_amd import synth
    rows = []
    for n in args.ns:
        X = synth.gaussian_sem(n, args.samples, seed=0)
        C = np.corrcoef(X.T)
        t0 = time.perf_counter()
        ref = osk.skeleton_discovery(C, args.samples)
        cpu_s = time.perf_counter() - t0
        row = {"n": n, "N": args.samples, "levels": ref.max_depth_run + 1, "unique_tests": int(sum(ref.tests_per_level)),
               "calls": int(sum(ref.calls_per_level)), "cpu_seconds": cpu_s,
               "cpu_tests_per_s": sum(ref.tests_per_level) / cpu_s, "cpu_cores": 1}
        if not args.no_gpu:
            import torch
            from rcaeval_amd.engine import get_engine
            eng = get_engine(0)
            Cd = eng.to_device(C)
            eng.skeleton(Cd, args.samples)                       # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = eng.skeleton(Cd, args.samples)
            torch.cuda.synchronize()
            gpu_s = time.perf_counter() - t0
            row.update({"gpu_seconds": gpu_s, "gpu_tests_per_s": sum(out.stats["tests"]) / gpu_s,
                        "same_skeleton": bool(np.array_equal(out.removed_level, ref.removed_level)),
                        "same_tests_per_level": out.stats["tests"] == ref.tests_per_level,
                        "speedup": cpu_s / gpu_s})
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"what": "reference-equivalent single-core CPU skeleton (oracle/skeleton.py) vs the GPU engine, "
                   "config-5 SEM family, stable PC-fisherz, full depth", "rows": rows}
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
