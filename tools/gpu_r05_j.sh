#!/bin/bash
# round 5: kernel trace of config C (training) to find its hot spots
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r05j_trace -o run --output-format csv -- python3 bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r05j_trace.log 2>&1 || { tail -5 gpurun_out/r05j_trace.log; exit 1; }
tail -1 gpurun_out/r05j_trace.log
