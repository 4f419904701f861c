#!/bin/bash
# round 5: training render glue once per scene (no host reads of masks), loss summed on device -- render + training parity, config C bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_render.py tests/test_gpu_train.py tests/test_gpu_config_c.py tests/test_gpu_config_d.py \
  > gpurun_out/r05u_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05u_tests.log; exit 1; }
tail -1 gpurun_out/r05u_tests.log
timeout -k 10 300 python bench.py --config C --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/r05u_C.log 2>&1 || { tail -5 gpurun_out/r05u_C.log; exit 1; }
tail -1 gpurun_out/r05u_C.log | cut -c1-170
