"""PMC passes of the VALU instruction-class counters over one command (rocprofv3, one pass
per group of at most 8 SQ counters, each pass under its own kill timeout), summarised per
kernel as per-dispatch means.

usage: python tools/valu_class_pmc.py COUNTERS_LIST OUTDIR OUT.json -- CMD...
COUNTERS_LIST is `rocprofv3 -L` output; only the SQ_INSTS_VALU* / SQ_INSTS_SALU counters it
names are requested (a counter the part does not have would fail the pass).
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys

WANT = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
        "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
        "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT",
        "SQ_INSTS_VALU_ADD_F16", "SQ_INSTS_VALU_MUL_F16", "SQ_INSTS_VALU_FMA_F16", "SQ_INSTS_VALU_TRANS_F16",
        "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_F32"]


def kname(raw: str) -> str:
    s = raw.replace("void ", "", 1)
    if "(anonymous namespace)::" in s:
        s = s.split("(anonymous namespace)::", 1)[1]
    depth, out = 0, []
    for ch in s:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)


def main():
    lst, outdir, dst = sys.argv[1:4]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    avail = set(re.findall(r"\b(SQ_INSTS_\w+)\b", open(lst).read()))
    have = [c for c in WANT if c in avail]
    print("class counters available:", have, flush=True)
    base = ["SQ_INSTS_VALU"]
    rest = [c for c in have if c != "SQ_INSTS_VALU"]
    groups = [base + rest[i:i + 7] for i in range(0, len(rest), 7)]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for gi, grp in enumerate(groups):
        d = os.path.join(outdir, f"vcls{gi}")
        full = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", *grp, "-d", d, "-o", "run",
                "--output-format", "csv", "--", *cmd]
        print("pass", gi, " ".join(grp), flush=True)
        with open(d + ".log", "w") as log:
            rc = subprocess.call(full, stdout=log, stderr=subprocess.STDOUT)
        if rc != 0:
            print(f"pass {gi} failed rc={rc}; see {d}.log", flush=True)
            sys.exit(rc)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: {"per_dispatch_mean": sum(v) / len(v), "dispatches": len(v)} for c, v in cs.items()}
           for k, cs in per.items()}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print("wrote", dst, len(out), "kernels", flush=True)


if __name__ == "__main__":
    main()
