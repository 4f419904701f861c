#!/bin/bash
# Round-4 certification call 3: per-family PMC evidence, kernel stats, host gaps, config-E render kernels.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04_final}
mkdir -p $O
echo "== $(date +%T) kernel_pmc"
timeout -k 10 700 python -u tools/kernel_pmc.py run $O/${T}_pmc --steps 5 --warmup 2 > $O/${T}_pmc.log 2>&1 || { tail -20 $O/${T}_pmc.log; exit 1; }
python -u tools/kernel_pmc.py summarize $O/${T}_pmc > $O/${T}_kernel_pmc.txt 2>&1; head -40 $O/${T}_kernel_pmc.txt
echo "== $(date +%T) kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_stats.log 2>&1 || { tail -20 $O/${T}_stats.log; exit 1; }
echo "== $(date +%T) gaps"
bash tools/gpu_gaps.sh ${T}_gaps | tail -30 || exit 1
echo "== $(date +%T) config E render kernels"
bash tools/gpu_prof_e.sh || exit 1
echo "== $(date +%T) done"
