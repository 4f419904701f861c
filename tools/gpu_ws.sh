#!/bin/bash
# WS GEMM check: GEMM / PTv3 GPU tests, then bench + per-launch breakdown with and without the WS kernel.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ws}
O=gpurun_out
mkdir -p $O
echo "== $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ptv3.py -v -x --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== $(date +%T) calls ws"
timeout -k 10 200 python -u tools/gemm_calls.py > $O/${T}_calls_ws.txt 2>&1 || { tail -20 $O/${T}_calls_ws.txt; exit 1; }
head -45 $O/${T}_calls_ws.txt
echo "== $(date +%T) bench ws"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench_ws.json 2> $O/${T}_bench_ws.err || { tail -20 $O/${T}_bench_ws.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_ws.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
echo "== $(date +%T) bench old"
SFX_GEMM_WS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench_old.json 2> $O/${T}_bench_old.err || { tail -20 $O/${T}_bench_old.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_old.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
echo "== $(date +%T) done"
