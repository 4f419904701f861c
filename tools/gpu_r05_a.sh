#!/bin/bash
# round 5: the register-summed SubM CPE kernel -- parity first, then a config-B line (A/B vs the pair path)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ptv3.py -k "subm" \
  > gpurun_out/r05a_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05a_tests.log; exit 1; }
tail -3 gpurun_out/r05a_tests.log
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/r05a_bench_on.log 2>&1 || exit 1
tail -1 gpurun_out/r05a_bench_on.log
SFX_SUBM_FUSED=0 timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05a_bench_off.log 2>&1 || exit 1
tail -1 gpurun_out/r05a_bench_off.log
