#!/bin/bash
# per-launch GEMM-family list of one config-B refine (roofline probe dump)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-psnr --gemm-calls $O/calls.jsonl > $O/bench.log 2>&1 || exit 1
