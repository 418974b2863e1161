"""Per-kernel duration statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace` on ROCm 7): name, calls, total / average / min / max microseconds,
sorted by total time, written as CSV (the layout of rocprofv3's kernel_stats.csv).

usage: python tools/rocpd_stats.py RESULTS.db OUT.csv [NAME_SUBSTRING]
"""
import collections
import csv
import sqlite3
import sys


def stats(db_path, sub=None):
    cur = sqlite3.connect(db_path).cursor()
    names = {r[0]: r[1] for r in cur.execute("select id, display_name from rocpd_info_kernel_symbol")}
    acc = collections.defaultdict(list)
    for kid, st, en in cur.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        nm = names.get(kid, str(kid))
        if sub is None or sub in nm:
            acc[nm].append((en - st) / 1000.0)
    rows = []
    for nm, ds in acc.items():
        rows.append({"Name": nm, "Calls": len(ds), "TotalDurationUs": sum(ds), "AverageUs": sum(ds) / len(ds),
                     "MinUs": min(ds), "MaxUs": max(ds)})
    rows.sort(key=lambda r: -r["TotalDurationUs"])
    tot = sum(r["TotalDurationUs"] for r in rows) or 1.0
    for r in rows:
        r["Percentage"] = 100.0 * r["TotalDurationUs"] / tot
    return rows


def main():
    rows = stats(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 else None)
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
        w.writeheader()
        for r in rows:
            w.writerow({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()})
    for r in rows[:25]:
        print(f"{r['AverageUs']:10.1f} us x {r['Calls']:4d}  {r['Percentage']:5.1f}%  {r['Name'][:90]}")


if __name__ == "__main__":
    main()
