#!/bin/bash
# gemm2 in the Block: refine parity tests, then alternating same-box bench pairs (gemm2 off / on), GEMM breakdown
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-gi}
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_ptv3.py tests/test_gpu_gemm2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
for i in 1 2 3; do
  for v in off on; do
    if [ $v = off ]; then export SFX_GEMM2_CHANNELS=""; else unset SFX_GEMM2_CHANNELS; fi
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-psnr --no-traffic > $O/${T}_b_${v}_${i}.json 2>/dev/null || { echo "bench failed"; exit 1; }
    echo "gemm2=$v pair=$i $(python -c "import json; d=json.load(open('$O/${T}_b_${v}_${i}.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline'].get('gemm_ms_per_unit'))")"
  done
done
unset SFX_GEMM2_CHANNELS
timeout -k 10 300 python -u tools/gemm_calls.py > $O/${T}_gemm_calls.txt 2>&1; head -30 $O/${T}_gemm_calls.txt; tail -1 $O/${T}_gemm_calls.txt
