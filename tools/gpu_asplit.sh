#!/bin/bash
# Pre-split A check: GEMM-family GPU tests, then per-call breakdown + bench with the A pre-split (default) and
# with the in-kernel split (SFX_GEMM_ASPLIT=0).  usage: bash tools/gpu_asplit.sh <tag> [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-as}
O=gpurun_out
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
if [ "$2" != "skip-tests" ]; then
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_full.py -v -x --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -30
[ $rc -eq 0 ] || exit $rc
fi
step calls presplit
timeout -k 10 200 python -u tools/gemm_calls.py > $O/${T}_calls_new.txt 2>&1 || { tail -20 $O/${T}_calls_new.txt; exit 1; }
head -24 $O/${T}_calls_new.txt; tail -1 $O/${T}_calls_new.txt
step calls inkernel
SFX_GEMM_ASPLIT=0 timeout -k 10 200 python -u tools/gemm_calls.py > $O/${T}_calls_old.txt 2>&1 || { tail -20 $O/${T}_calls_old.txt; exit 1; }
tail -1 $O/${T}_calls_old.txt
step bench presplit
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench_new.json 2> $O/${T}_bench_new.err || { tail -20 $O/${T}_bench_new.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_new.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
step bench inkernel
SFX_GEMM_ASPLIT=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench_old.json 2> $O/${T}_bench_old.err || { tail -20 $O/${T}_bench_old.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_old.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
step done
