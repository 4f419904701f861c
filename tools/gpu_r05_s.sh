#!/bin/bash
# round 5: fused training MLP tail (forward + backward) -- op parity, training parity, config C bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py -k "block_mlp" \
  > gpurun_out/r05s_ops.log 2>&1 || { echo "op tests failed"; tail -30 gpurun_out/r05s_ops.log; exit 1; }
tail -1 gpurun_out/r05s_ops.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_ops.py tests/test_gpu_train.py tests/test_gpu_config_c.py tests/test_gpu_config_d.py \
  > gpurun_out/r05s_train.log 2>&1 || { echo "train tests failed"; tail -30 gpurun_out/r05s_train.log; exit 1; }
tail -1 gpurun_out/r05s_train.log
timeout -k 10 300 python bench.py --config C --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/r05s_C.log 2>&1 || { tail -5 gpurun_out/r05s_C.log; exit 1; }
tail -1 gpurun_out/r05s_C.log | cut -c1-170
SFX_MLP_TRAIN_FUSED=0 timeout -k 10 300 python bench.py --config C --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/r05s_C0.log 2>&1 || { tail -5 gpurun_out/r05s_C0.log; exit 1; }
tail -1 gpurun_out/r05s_C0.log | cut -c1-170
