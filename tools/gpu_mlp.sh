#!/bin/bash
# fused-MLP iteration: unit tests, micro-bench, block-level parity, bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-mlp}
O=gpurun_out
step() { echo "== $(date +%T) $*"; }
step mlp-tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_mlp_tests.log 2>&1 || { tail -40 $O/${T}_mlp_tests.log; exit 1; }
tail -2 $O/${T}_mlp_tests.log
step mlp-bench
timeout -k 10 120 python -u tools/mlp_bench.py > $O/${T}_mlp_bench.txt 2>&1 || { tail -20 $O/${T}_mlp_bench.txt; exit 1; }
cat $O/${T}_mlp_bench.txt
step block-tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "feature_predictor or backbone_feature or config_b_refine or config_b_end" > $O/${T}_block_tests.log 2>&1 || { tail -40 $O/${T}_block_tests.log; exit 1; }
tail -2 $O/${T}_block_tests.log
step bench
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
step done
