#!/bin/bash
# round 5: the default bench line with the whole-scene CPU baseline (config B)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final2
timeout -k 10 900 python bench.py > gpurun_out/final2/bench_B.log 2>&1 || { tail -5 gpurun_out/final2/bench_B.log; exit 1; }
tail -1 gpurun_out/final2/bench_B.log | cut -c1-200
timeout -k 10 600 python bench.py --config E --no-traffic --no-cpu-baseline --no-psnr > gpurun_out/final2/bench_E.log 2>&1 || { tail -5 gpurun_out/final2/bench_E.log; exit 1; }
tail -1 gpurun_out/final2/bench_E.log | cut -c1-160
