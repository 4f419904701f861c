#!/bin/bash
# round 5: kernel trace of config E with the MLP tail split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/split/Etrace -o run --output-format csv -- python3 bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/split/Etrace.log 2>&1 || { tail -5 gpurun_out/split/Etrace.log; exit 1; }
echo done
