"""Median duration of each run of back-to-back launches of one kernel in a rocprofv3 --kernel-trace capture
(the HIP-graph replays of tools/gemm2_bench.py / mlp_bench.py): what the kernel takes without launch gaps.
usage: python tools/kernel_runs.py <rocprof output dir> [min run length]"""
import csv
import glob
import re
import statistics
import sys


def short(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def main(d, min_run=50):
    rows = []
    for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    runs, cur = [], []
    for s, e, k in rows:
        if cur and cur[-1][2] != k:
            runs.append(cur)
            cur = []
        cur.append((s, e, k))
    if cur:
        runs.append(cur)
    i = 0
    for run in runs:
        if len(run) < min_run:
            continue
        d_us = [(e - s) / 1e3 for s, e, _ in run]
        gaps = [(run[j + 1][0] - run[j][1]) / 1e3 for j in range(len(run) - 1)]
        print(f"run {i:3d} {run[0][2][:48]:48s} n={len(run):4d} median {statistics.median(d_us):8.2f} us "
              f"(min {min(d_us):8.2f}) gap {statistics.median(gaps):6.2f} us", flush=True)
        i += 1


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 50)
