#!/bin/bash
# round 5: kernel traces of config C and config E after the training / fused-rule changes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05r_C -o run --output-format csv -- python3 bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --profile-only > gpurun_out/r05r_C.log 2>&1 || { tail -5 gpurun_out/r05r_C.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05r_E -o run --output-format csv -- python3 bench.py --config E --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/r05r_E.log 2>&1 || { tail -5 gpurun_out/r05r_E.log; exit 1; }
echo done
