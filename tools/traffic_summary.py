"""Per-scene HBM traffic of the GEMM family from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs
of `bench.py --steps S --warmup W --profile-only`, i.e. S+W scenes), corrected as MI355X_MICROARCH.md prescribes
(gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads -> x2; both counters in KiB).

python tools/traffic_summary.py <fetch.csv> <write.csv> <scenes> <out.json>"""
import collections
import csv
import json
import sys


def load(path):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        k = k.replace("(anonymous namespace)::", "").replace("void ", "")
        fam = k.split("(")[0].split("<")[0]
        per[fam] += float(r["Counter_Value"]) * 1024.0
    return per


def main():
    f, w, scenes, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fe, wr = load(f), load(w)
    fams = sorted(set(fe) | set(wr), key=lambda k: -(2 * fe.get(k, 0) + wr.get(k, 0)))
    res = {"source": [f, w], "scenes": scenes, "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB->B)",
           "per_scene": {k: {"fetch_B": 2 * fe.get(k, 0) / scenes, "write_B": wr.get(k, 0) / scenes,
                             "hbm_B": (2 * fe.get(k, 0) + wr.get(k, 0)) / scenes} for k in fams[:25]}}
    json.dump(res, open(out, "w"), indent=1)
    for k in fams[:12]:
        print(f"{res['per_scene'][k]['hbm_B'] / 1e9:8.3f} GB/scene  {k}")


if __name__ == "__main__":
    main()
