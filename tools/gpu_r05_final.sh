#!/bin/bash
# round 5 final measurements: the default bench line (roofline + traffic + cpu baseline + PSNR, as the driver runs
# it), the other configs' lines, a rocprofv3 --kernel-trace --stats summary of the default command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 900 python bench.py > gpurun_out/final/bench_B.log 2>&1 || { tail -5 gpurun_out/final/bench_B.log; exit 1; }
tail -1 gpurun_out/final/bench_B.log | cut -c1-200
for c in A C E; do
  timeout -k 10 600 python bench.py --config $c --no-traffic > gpurun_out/final/bench_$c.log 2>&1 || { tail -5 gpurun_out/final/bench_$c.log; exit 1; }
  tail -1 gpurun_out/final/bench_$c.log | cut -c1-160
done
timeout -k 10 600 python bench.py --config C --no-traffic --train-prec amp > gpurun_out/final/bench_C_amp.log 2>&1 || { tail -5 gpurun_out/final/bench_C_amp.log; exit 1; }
tail -1 gpurun_out/final/bench_C_amp.log | cut -c1-160
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/final/prof.log 2>&1 || { tail -5 gpurun_out/final/prof.log; exit 1; }
echo done
