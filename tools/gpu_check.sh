#!/bin/bash
# GPU check: all gpu tests + smoke + bench (config B, with roofline, traffic and CPU baseline).
# usage: bash tools/gpu_check.sh <tag> [bench args...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-chk}; shift
O=gpurun_out
echo "== $(date +%T) tests"
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/${T}_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -30 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
echo "== $(date +%T) bench"
timeout -k 10 900 python -u bench.py "$@" > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
