#!/bin/bash
# heads split recalibration: heads parity tests, config B + E bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_full.py -x -q -m gpu -k "heads or config_b or config_e" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_B.log 2>&1 || exit 2
tail -1 $O/bench_B.log | cut -c1-150
timeout -k 10 300 python -u bench.py --config E --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_E.log 2>&1 || exit 3
tail -1 $O/bench_E.log | cut -c1-150
