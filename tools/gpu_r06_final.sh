#!/bin/bash
# round 6 final measurements: default bench line (as the driver runs it), configs A / C (fp32, amp) / E with whole-scene
# CPU baselines, rocprofv3 --kernel-trace --stats of the default command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06final
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_B.log 2>&1 || { tail -5 $O/bench_B.log; exit 1; }
tail -1 $O/bench_B.log | cut -c1-200
for c in A E; do
  timeout -k 10 600 python bench.py --config $c --no-traffic > $O/bench_$c.log 2>&1 || { tail -5 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log | cut -c1-160
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-traffic --no-psnr > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo done
