#!/bin/bash
# round 5: final config C lines (fp32 and reference precision) after the training-MLP tail split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --config C --no-traffic > gpurun_out/final/bench_C.log 2>&1 || { tail -5 gpurun_out/final/bench_C.log; exit 1; }
tail -1 gpurun_out/final/bench_C.log | cut -c1-160
timeout -k 10 600 python bench.py --config C --no-traffic --train-prec amp > gpurun_out/final/bench_C_amp.log 2>&1 || { tail -5 gpurun_out/final/bench_C_amp.log; exit 1; }
tail -1 gpurun_out/final/bench_C_amp.log | cut -c1-160
