#!/bin/bash
# round 5: config-C tests (both precision modes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_config_c.py \
  > gpurun_out/r05amp_configC_tests3.log 2>&1 || { grep -E "config C|passed|failed|Error" gpurun_out/r05amp_configC_tests3.log | tail -20; exit 1; }
grep -E "config C|passed|failed" gpurun_out/r05amp_configC_tests3.log | tail -12
