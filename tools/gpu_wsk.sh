#!/bin/bash
# kernel-trace stats of the bench (WS on) + single-shape timings
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-wsk}
O=gpurun_out
for S in "100000 64 64 20" "90434 96 96 20" "37759 256 256 20" "37759 1024 256 20 gelu"; do
  timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1
  SFX_GEMM_WS=0 timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_prof.log 2>&1 || { tail -20 $O/${T}_prof.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$O/${T}_prof/run_kernel_stats.csv")))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print("total ms per scene", tot/7e6)
for r in rows[:25]:
    n=r['Name'].replace('(anonymous namespace)::','')[:80]
    print(f"{int(r['Calls'])/7:6.1f} {float(r['TotalDurationNs'])/7e3:9.1f}us {float(r['AverageNs'])/1e3:8.1f}  {n}")
PY
