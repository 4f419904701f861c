#!/bin/bash
# round 5: two-pass fp16x2 window-attention backward -- parity (train ops, training parity), config C bench + trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py -k "window_attention" \
  > gpurun_out/r05k_ops.log 2>&1 || { echo "ops tests failed"; tail -30 gpurun_out/r05k_ops.log; exit 1; }
tail -1 gpurun_out/r05k_ops.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_ops.py tests/test_gpu_train.py tests/test_gpu_config_c.py tests/test_gpu_config_d.py \
  > gpurun_out/r05k_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05k_tests.log; exit 1; }
tail -1 gpurun_out/r05k_tests.log
timeout -k 10 300 python bench.py --config C --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/r05k_benchC.log 2>&1 || { tail -5 gpurun_out/r05k_benchC.log; exit 1; }
tail -1 gpurun_out/r05k_benchC.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05k_trace -o run --output-format csv -- python3 bench.py --config C --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/r05k_trace.log 2>&1 || { tail -5 gpurun_out/r05k_trace.log; exit 1; }
echo done
