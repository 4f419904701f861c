#!/bin/bash
# round 5: config C kernel trace with the fused training MLP
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t_C -o run --output-format csv -- python3 bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --profile-only > gpurun_out/r05t_C.log 2>&1 || { tail -5 gpurun_out/r05t_C.log; exit 1; }
echo done
