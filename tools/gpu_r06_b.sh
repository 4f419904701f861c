#!/bin/bash
# fused attention + proj: parity, full-size refine parity, A/B bench, kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_ptv3.py \
  -k "window_attention_proj or feature_predictor_matches" > $O/t1.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_full.py \
  -k "config_b_refine or config_b_end_to_end" > $O/t2.log 2>&1 || exit 2
for i in 1 2; do
  SFX_ATTN_PROJ=0 timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_off$i.log 2>&1 || exit 3
  timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_on$i.log 2>&1 || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --steps 10 --profile-only > $O/prof.log 2>&1 || exit 5
