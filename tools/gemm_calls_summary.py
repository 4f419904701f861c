"""Aggregate bench.py --gemm-calls output by (kind, shape): calls, total ms, TF/s.
usage: python tools/gemm_calls_summary.py <file.jsonl> [top]"""
import collections
import json
import sys

agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for line in open(sys.argv[1]):
    d = json.loads(line)
    a = agg[(d["kind"], tuple(d["shape"]))]
    a[0] += 1
    a[1] += d["ms"]
    a[2] += d["tflops"] * d["ms"]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
tot = sum(v[1] for v in agg.values())
print(f"total {tot:.3f} ms over {sum(v[0] for v in agg.values())} launches")
for (k, sh), (c, ms, tw) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{ms:8.3f} ms {c:3d}x {k:20s} {str(sh):24s} {tw / ms if ms else 0:7.1f} TF/s")
