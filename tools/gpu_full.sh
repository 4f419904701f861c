#!/bin/bash
# One GPU call: all gpu tests, smoke, the default bench line (roofline + traffic + CPU baseline), then a
# rocprofv3 kernel-trace summary of the bench.  usage: bash tools/gpu_full.sh <tag> [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r02}
O=gpurun_out
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
if [ "$2" != "skip-tests" ]; then
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/${T}_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -30 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
fi
step bench
timeout -k 10 700 python -u bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_prof.log 2>&1 || { tail -30 $O/${T}_prof.log; exit 1; }
step done
