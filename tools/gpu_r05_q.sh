#!/bin/bash
# round 5: size-ruled fused SubM CPE default -- full-size parity (B, E, A, real clouds, ptv3 ops) + B / E bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_real_clouds.py tests/test_gpu_ptv3.py \
  > gpurun_out/r05q_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05q_tests.log; exit 1; }
tail -1 gpurun_out/r05q_tests.log
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05q_E.log 2>&1 || { tail -5 gpurun_out/r05q_E.log; exit 1; }
tail -1 gpurun_out/r05q_E.log | cut -c1-170
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05q_B.log 2>&1 || { tail -5 gpurun_out/r05q_B.log; exit 1; }
tail -1 gpurun_out/r05q_B.log | cut -c1-170
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_ops.py tests/test_gpu_train.py tests/test_gpu_config_c.py \
  > gpurun_out/r05q_train.log 2>&1 || { echo "train tests failed"; tail -30 gpurun_out/r05q_train.log; exit 1; }
tail -1 gpurun_out/r05q_train.log
timeout -k 10 300 python bench.py --config C --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/r05q_C.log 2>&1 || { tail -5 gpurun_out/r05q_C.log; exit 1; }
tail -1 gpurun_out/r05q_C.log | cut -c1-170
