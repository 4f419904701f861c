#!/bin/bash
# round 5: stage-0 serialized-order renumbering (SFX_REORDER) -- parity at full size, then A/B bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_real_clouds.py tests/test_gpu_ptv3.py \
  > gpurun_out/r05i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -1 gpurun_out/r05i_tests.log
for r in 1 0 1 0; do
  SFX_REORDER=$r timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05i_bench_$r.log 2>&1 || exit 1
  echo "reorder=$r $(tail -1 gpurun_out/r05i_bench_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
