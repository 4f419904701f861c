#!/bin/bash
# per-kernel PMC evidence for the config-B step + the up-front pooled-count A/B (5 alternating same-box pairs)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ev}
O=gpurun_out
step() { echo "== $(date +%T) $*"; }
step pmc
timeout -k 10 600 python -u tools/kernel_pmc.py run $O/${T}_pmc > $O/${T}_pmc_run.log 2>&1 || { tail -30 $O/${T}_pmc_run.log; exit 1; }
python tools/kernel_pmc.py summarize $O/${T}_pmc > $O/${T}_pmc_summary.txt 2>&1
head -40 $O/${T}_pmc_summary.txt
step ab-pool-counts
for i in 1 2 3 4 5; do
  for v in 0 1; do
    SFX_POOL_COUNTS_UPFRONT=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-psnr --no-traffic --profile-only > $O/${T}_ab_${v}_${i}.json 2>/dev/null || { echo "ab run failed"; exit 1; }
    echo "upfront=$v pair=$i $(python -c "import json,sys; d=json.load(open('$O/${T}_ab_${v}_${i}.json')); print(d['value'], d['ms_per_step'])")"
  done
done | tee $O/${T}_ab_pool.txt
step done
