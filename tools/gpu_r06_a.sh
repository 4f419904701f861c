#!/bin/bash
# round 6, first GPU call: the changed / new GPU tests, then a default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_abi.py \
  tests/test_gpu_config_d_full.py tests/test_gpu_render.py > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --no-traffic > $O/bench.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_config_c.py \
  -k amp > $O/t2.log 2>&1 || exit 3
