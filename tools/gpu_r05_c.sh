#!/bin/bash
# round 5: fused SubM CPE parity + per-stage microbench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptv3.py -k "subm" \
  > gpurun_out/r05c_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05c_tests.log; exit 1; }
tail -2 gpurun_out/r05c_tests.log
timeout -k 10 300 python -u tools/subm_bench.py > gpurun_out/r05c_subm_bench.log 2>&1 || { tail -20 gpurun_out/r05c_subm_bench.log; exit 1; }
cat gpurun_out/r05c_subm_bench.log
