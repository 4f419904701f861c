#!/bin/bash
# fused attention + proj at C <= 96 only (default) vs off vs all: alternating A/B, 20-step lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06d
mkdir -p $O
for i in 1 2 3; do
  SFX_ATTN_PROJ=0 timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_off$i.log 2>&1 || exit 3
  timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_on$i.log 2>&1 || exit 4
done
