#!/bin/bash
# round 5: render prep one thread per Gaussian over all views; element-wise gs_pack -- render + full parity, E / B bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_render.py tests/test_gpu_mlp.py tests/test_gpu_ptv3.py tests/test_gpu_full.py \
  > gpurun_out/r05y_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05y_tests.log; exit 1; }
tail -1 gpurun_out/r05y_tests.log
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05y_E.log 2>&1 || { tail -5 gpurun_out/r05y_E.log; exit 1; }
tail -1 gpurun_out/r05y_E.log | cut -c1-170
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05y_B.log 2>&1 || { tail -5 gpurun_out/r05y_B.log; exit 1; }
tail -1 gpurun_out/r05y_B.log | cut -c1-170
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05y_Etrace -o run --output-format csv -- python3 bench.py --config E --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/r05y_Etrace.log 2>&1 || { tail -5 gpurun_out/r05y_Etrace.log; exit 1; }
echo done
