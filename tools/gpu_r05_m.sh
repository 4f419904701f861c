#!/bin/bash
# round 5: config-B kernel trace (default tree)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05m_trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/r05m_trace.log 2>&1 || { tail -5 gpurun_out/r05m_trace.log; exit 1; }
echo done
