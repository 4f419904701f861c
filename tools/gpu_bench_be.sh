#!/bin/bash
# Config B and E bench lines (no traffic / CPU baseline), PTv3 GPU tests first.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-be}
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ptv3.py -x -q --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -20 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for c in B E; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-traffic > $O/${T}_bench_$c.json 2> $O/${T}_bench_$c.err || { tail -20 $O/${T}_bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
done
