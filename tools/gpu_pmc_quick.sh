#!/bin/bash
# One PMC pass per counter group over a 1-step bench; per-kernel sums of the level kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmcq$i -o run --output-format csv -- $B > gpurun_out/pmcq$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcq$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for i in (1, 2):
    for f in glob.glob(f"gpurun_out/pmcq{i}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_level" not in k: continue
            k = k.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "") + "".join(k.split("(")[1:2])[:0]
            name = r["Kernel_Name"][:60]
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    print("   ", {c: "%.3g" % x for c, x in sorted(v.items())})
PY
