#!/bin/bash
# GEMM two-deep slab stream (PD = 2): GEMM parity, bench x3, tile sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_ptv3.py -k "linear or subm or gemm or feature_predictor" > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_full.py -k "config_b_refine" > $O/t2.log 2>&1 || exit 2
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench$i.log 2>&1 || exit 3
  tail -1 $O/bench$i.log | cut -c1-120
done
timeout -k 10 600 python -u tools/gemm_tune.py 100000 all 1 > $O/tune.jsonl 2>&1 || exit 4
