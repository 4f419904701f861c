"""Sum rocprofv3 PMC counters (counter_collection.csv) over the dispatches of one kernel family.

python tools/pmc_traffic.py <csv> [<csv> ...] --kernel gemm_kernel --per 149
-> per-counter totals and per-`per`-dispatch (one scene) values.  FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM), so the
HBM traffic estimate is 2*FETCH_SIZE + WRITE_SIZE.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", default="gemm_kernel")
    ap.add_argument("--per", type=int, default=1, help="dispatches per unit (e.g. GEMM launches per scene)")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for path in a.csv:
        with open(path) as f:
            for row in csv.DictReader(f):
                if a.kernel not in row.get("Kernel_Name", ""):
                    continue
                name = row["Counter_Name"]
                tot[name] += float(row["Counter_Value"])
                disp[name].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for name in sorted(tot):
        n = len(disp[name])
        print(f"{name}: total {tot[name]:.1f} over {n} dispatches; per {a.per} dispatches: "
              f"{tot[name] / max(n, 1) * a.per:.1f}")
    if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        nf, nw = len(disp["FETCH_SIZE"]), len(disp["WRITE_SIZE"])
        per_unit = (2 * tot["FETCH_SIZE"] / nf + tot["WRITE_SIZE"] / nw) * a.per * 1024
        print(f"HBM traffic estimate (2*FETCH + WRITE) per unit: {per_unit / 1e9:.3f} GB")


if __name__ == "__main__":
    main()
