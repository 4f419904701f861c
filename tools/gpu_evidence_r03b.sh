#!/bin/bash
# steady-state per-kernel PMC evidence (config B), config E bench line, rocprof kernel stats of the config-B bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ev2}
O=gpurun_out
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
step pmc
timeout -k 10 600 python -u tools/kernel_pmc.py run $O/${T}_pmc > $O/${T}_pmc_run.log 2>&1 || { tail -30 $O/${T}_pmc_run.log; exit 1; }
python tools/kernel_pmc.py summarize $O/${T}_pmc > $O/${T}_pmc_summary.txt 2>&1
sed -n 1,50p $O/${T}_pmc_summary.txt
step stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_prof.log 2>&1 || { tail -30 $O/${T}_prof.log; exit 1; }
step benchE
timeout -k 10 400 python -u bench.py --config E --no-cpu-baseline --no-psnr --no-traffic > $O/${T}_benchE.json 2> $O/${T}_benchE.err || { tail -20 $O/${T}_benchE.err; exit 1; }
cat $O/${T}_benchE.json
step done
