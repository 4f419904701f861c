#!/bin/bash
# kernel-trace stats of one bench config: bash tools/gpu_prof_cfg.sh <tag> <config> [steps]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; C=$2; S=${3:-3}
O=gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 bench.py --config $C --steps $S --warmup 1 --profile-only > $O/${T}_prof.log 2>&1 || { tail -20 $O/${T}_prof.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$O/${T}_prof/run_kernel_stats.csv")))
tot=sum(float(r['TotalDurationNs']) for r in rows)
n=$S+1
print("total ms per step", tot/n/1e6)
for r in rows[:25]:
    nm=r['Name'].replace('(anonymous namespace)::','')[:80]
    print(f"{int(r['Calls'])/n:6.1f} {float(r['TotalDurationNs'])/n/1e3:9.1f}us {float(r['AverageNs'])/1e3:8.1f}  {nm}")
PY
