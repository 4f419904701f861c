#!/bin/bash
# round 5: per-launch GEMM-family list of one config-C training micro-step and of one config-B refine
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --gemm-calls gpurun_out/r05l_gemmC.jsonl > gpurun_out/r05l_C.log 2>&1 || { tail -5 gpurun_out/r05l_C.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr --gemm-calls gpurun_out/r05l_gemmB.jsonl > gpurun_out/r05l_B.log 2>&1 || { tail -5 gpurun_out/r05l_B.log; exit 1; }
echo done
