#!/bin/bash
# One GPU call: the selected GPU tests (default: all), smoke, then the default bench line.
# usage: bash tools/gpu_tests_r03.sh <tag> [pytest selection...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r03}
shift
SEL=${@:-tests}
O=gpurun_out
step() { echo "== $(date +%T) $*"; }
step tests $SEL
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 900 --timeout-method thread -s --durations=25 > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -30 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
step bench
timeout -k 10 400 python -u bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
step done
