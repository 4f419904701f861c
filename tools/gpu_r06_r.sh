#!/bin/bash
# pair lists by block counts (ABI v16) + gs_pack atomics + heads head-group split: parity, same-box A/B against the previous build, trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_ptv3.py tests/test_abi.py -k "pair_lists or subm or feature_predictor or abi or heads" > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_full.py -k "config_b_refine" > $O/t2.log 2>&1 || exit 2
bash tools/ab_env.sh $O "SFX_PAIR_LISTS=0 SFX_HEADS_SPLIT=0" "SFX_AB=1" 3 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --profile-only > $O/prof.log 2>&1 || exit 5
# fused C = 256 Block MLP vs LayerNorm + two GEMMs on the current GEMM tiles (SFX_MLP_CHANNELS)
for i in 1 2; do
  for v in fused unfused; do
    ch="64,96,128,256"; [ $v = unfused ] && ch="64,96,128"
    SFX_MLP_CHANNELS=$ch timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/mlp_${v}$i.log 2>&1 || exit 6
    echo "mlp $v $i $(tail -1 $O/mlp_${v}$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
