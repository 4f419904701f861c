#!/bin/bash
# round 5: training-MLP tail split -- op tests, config-C tests, config C A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split3
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_train_ops.py tests/test_gpu_mlp.py > gpurun_out/split3/ops.log 2>&1 || { tail -30 gpurun_out/split3/ops.log; exit 1; }
tail -1 gpurun_out/split3/ops.log
for v in 0 1; do
  SFX_MLP_SPLIT=$v timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/split3/C_$v.log 2>&1 || { tail -5 gpurun_out/split3/C_$v.log; exit 1; }
  echo "C split=$v $(tail -1 gpurun_out/split3/C_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_config_c.py tests/test_gpu_train.py > gpurun_out/split3/c.log 2>&1 || { grep -E "config C|passed|failed|Error" gpurun_out/split3/c.log | tail -20; exit 1; }
grep -E "config C|passed|failed" gpurun_out/split3/c.log | tail -6
