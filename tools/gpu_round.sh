#!/bin/bash
# One GPU call: gpu tests, smoke, bench (config B with CPU baseline), rocprofv3 stats + HBM PMC passes.
# usage: bash tools/gpu_round.sh <tag> [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r01}
O=gpurun_out
step() { echo "== $(date +%T) $*"; }
if [ "$2" != "skip-tests" ]; then
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -30 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
fi
step bench
timeout -k 10 400 python -u bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_prof.log 2>&1 || { tail -30 $O/${T}_prof.log; exit 1; }
step pmc-fetch
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/${T}_pmcF -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --profile-only > $O/${T}_pmcF.log 2>&1 || { tail -30 $O/${T}_pmcF.log; exit 1; }
step pmc-write
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/${T}_pmcW -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --profile-only > $O/${T}_pmcW.log 2>&1 || { tail -30 $O/${T}_pmcW.log; exit 1; }
step done
