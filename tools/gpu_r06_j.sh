#!/bin/bash
# fused pair-sum LN + qkv: parity, A/B bench, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_ptv3.py \
  -k "cpe_ln_qkv or feature_predictor_matches or backbone_feature_l2" > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_full.py \
  tests/test_gpu_real_clouds.py -k "config_b_refine or config_b_end_to_end or config_e_refine or config_a or real_cloud" > $O/t2.log 2>&1 || exit 2
for i in 1 2 3; do
  SFX_LN_QKV=0 timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_off$i.log 2>&1 || exit 3
  timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_on$i.log 2>&1 || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u bench.py --steps 10 --profile-only > $O/prof.log 2>&1 || exit 5
