#!/bin/bash
# round 5: C = 256 fused-MLP tail split -- tests + A/B on configs B and E
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_mlp.py > gpurun_out/split/tests.log 2>&1 || { tail -30 gpurun_out/split/tests.log; exit 1; }
tail -1 gpurun_out/split/tests.log
for i in 1 2; do
  for v in 0 1; do
    SFX_MLP_SPLIT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/split/B_${v}_$i.log 2>&1 || { tail -5 gpurun_out/split/B_${v}_$i.log; exit 1; }
    echo "B split=$v $(tail -1 gpurun_out/split/B_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for v in 0 1; do
  SFX_MLP_SPLIT=$v timeout -k 10 300 python bench.py --config E --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/split/E_$v.log 2>&1 || { tail -5 gpurun_out/split/E_$v.log; exit 1; }
  echo "E split=$v $(tail -1 gpurun_out/split/E_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_full.py -k "config_b or config_e_refine" > gpurun_out/split/full.log 2>&1 || { tail -20 gpurun_out/split/full.log; exit 1; }
tail -1 gpurun_out/split/full.log
