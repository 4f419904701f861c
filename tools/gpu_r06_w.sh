#!/bin/bash
# compacted pair positions for the pair-sum LayerNorm (sfx_cpe_residual_ln_cpairs, ABI v16): parity, same-box A/B, trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_ptv3.py tests/test_abi.py -k "pair_lists or subm or feature_predictor or abi or backbone" > $O/t1.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 480 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_real_clouds.py -k "config_b_refine or config_e_refine or real_cloud" > $O/t2.log 2>&1 || exit 2
bash tools/ab_env.sh $O "SFX_LN_COMPACT=0" "SFX_AB=1" 3 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --profile-only > $O/prof.log 2>&1 || exit 5
