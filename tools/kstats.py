"""Summarise a rocprofv3 kernel_stats.csv: per-step ms, calls, average us, top-N kernels.
usage: python tools/kstats.py <run_kernel_stats.csv> <steps> [top] [filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
flt = sys.argv[4] if len(sys.argv) > 4 else ""
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms, {tot / 1e6 / steps:.2f} ms per step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    if flt and flt not in r["Name"]:
        continue
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {int(r['Calls']) / steps:7.1f} calls "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")
