#!/bin/bash
# GEMM check: PTv3 GPU tests, per-launch breakdown, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-g}
O=gpurun_out
mkdir -p $O
echo "== $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ptv3.py -v -x --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== $(date +%T) calls"
timeout -k 10 200 python -u tools/gemm_calls.py > $O/${T}_calls.txt 2>&1 || { tail -20 $O/${T}_calls.txt; exit 1; }
grep -v amdgpu.ids $O/${T}_calls.txt | head -45
echo "== $(date +%T) bench"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
echo "== $(date +%T) done"
