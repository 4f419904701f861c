#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptv3.py -k "subm" \
  > gpurun_out/r05g_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05g_tests.log; exit 1; }
tail -1 gpurun_out/r05g_tests.log
timeout -k 10 300 python -u tools/subm_bench.py > gpurun_out/r05g_subm_bench.log 2>&1 || { tail -20 gpurun_out/r05g_subm_bench.log; exit 1; }
cat gpurun_out/r05g_subm_bench.log
for C in 64 256; do SFX_SUBM_OS_DEBUG=16 timeout -k 10 120 python -u tools/subm_bench.py --only $C > gpurun_out/r05g_stamps_$C.log 2>&1 || exit 1; done
grep -A20 "wave loader" gpurun_out/r05g_stamps_64.log > gpurun_out/r05g_stamps_64_head.txt || true
grep -A20 "wave loader" gpurun_out/r05g_stamps_256.log > gpurun_out/r05g_stamps_256_head.txt || true
