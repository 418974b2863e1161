"""Timeline of the last bench step from a rocprofv3 kernel trace: per dispatch the start offset,
duration and the idle gap before it (per stream), from the last k_colsum_partial on.
usage: python tools/timeline.py run_kernel_trace.csv [ANCHOR]
(ANCHOR: the kernel that starts a step, default k_colsum_partial; k_init for skeleton-only runs)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_colsum_partial"
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]] + [len(rows)]
# the last threshold-mode step (k_level0<0>), not the full-p side run
pick = [(a, b) for a, b in zip(starts, starts[1:]) if any("k_level0<0>" in r["Kernel_Name"] for r in rows[a:b])][-1]
rows = rows[pick[0]:pick[1]]
t0 = int(rows[0]["Start_Timestamp"])
last_end = {}
busy_end = t0
idle = 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r["Queue_Id"]
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    if s > busy_end:
        idle += (s - busy_end) / 1e3
    busy_end = max(busy_end, e)
    last_end[q] = e
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{(s - t0) / 1e3:9.1f} us  q{q:>2}  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {name[:60]}")
print(f"span {(busy_end - t0) / 1e3:.1f} us, device idle (no kernel on any queue) {idle:.1f} us")
