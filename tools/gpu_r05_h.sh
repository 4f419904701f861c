#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SFX_SUBM_OS_VARIANT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptv3.py -k "subm_cpe" \
  > gpurun_out/r05h_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05h_tests.log; exit 1; }
tail -1 gpurun_out/r05h_tests.log
for v in 0 1; do SFX_SUBM_OS_VARIANT=$v timeout -k 10 300 python -u tools/subm_bench.py > gpurun_out/r05h_subm_bench_v$v.log 2>&1 || exit 1; grep "C=128\|C=256" gpurun_out/r05h_subm_bench_v$v.log; done
