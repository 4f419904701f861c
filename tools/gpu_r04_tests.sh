#!/bin/bash
# Round-4 certification call 1: the whole GPU test suite, then smoke().
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04_final}
mkdir -p $O
echo "== $(date +%T) pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { grep -E "FAILED|ERROR|Error|error" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -3 $O/${T}_gpu_tests.log
echo "== $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -2 $O/${T}_smoke.log
echo "== $(date +%T) done"
