"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_*/run_counter_collection.csv) per kernel.

usage: python tools/pmc_summary.py OUT.json [gpurun_out]
"""
import collections
import csv
import glob
import json
import os
import sys


def kname(raw: str) -> str:
    s = raw.replace("void ", "", 1)
    if "(anonymous namespace)::" in s:
        s = s.split("(anonymous namespace)::", 1)[1]
    depth, out = 0, []
    for ch in s:  # cut the argument list, keep template args
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)


def main():
    dst = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
    out = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in per.items():
            for c, vals in v.items():
                out.setdefault(k, {})[c] = {"per_dispatch_mean": sum(vals) / len(vals), "dispatches": len(vals)}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k in out:
        print(k, {c: round(v["per_dispatch_mean"]) for c, v in out[k].items() if c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU")})


if __name__ == "__main__":
    main()
