"""Host gaps inside the benched step: from a rocprofv3 --kernel-trace csv of `bench.py --profile-only --markers`,
take the kernels between consecutive marker launches (one step each), and report the idle gaps between one
kernel's end and the next kernel's start: count > 20 us, the largest ones (with the kernels around them), and the
step's busy vs wall time.  usage: python tools/trace_gaps.py <rocprof dir>"""
import csv
import glob
import re
import statistics
import sys


def short(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(d):
    rows = []
    for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "profile_marker" in r[2]]
    steps = [rows[a + 1:b] for a, b in zip(marks, marks[1:])]
    for si, st in enumerate(steps):
        if not st:
            continue
        wall = (st[-1][1] - st[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in st) / 1e3
        gaps = []
        end = st[0][1]
        for j in range(1, len(st)):
            g = (st[j][0] - end) / 1e3
            if g > 0:
                gaps.append((g, st[j - 1][2], st[j][2], j))
            end = max(end, st[j][1])
        big = sorted(gaps, reverse=True)
        n20 = sum(1 for g in gaps if g[0] > 20)
        print(f"step {si}: {len(st)} kernels, wall {wall:8.1f} us, busy {busy:8.1f} us, idle {wall - busy:7.1f} us, "
              f"gaps > 20 us: {n20}, median gap {statistics.median([g[0] for g in gaps]) if gaps else 0:.1f} us")
        for g, a, b, j in big[:8]:
            print(f"    {g:8.1f} us  after {a[:50]:50s} before {b[:50]}")


if __name__ == "__main__":
    main(sys.argv[1])
