#!/bin/bash
# same-box A/B of an environment switch on the config-B bench (alternating pairs), after the PTv3 GPU tests.
# usage: bash tools/gpu_ab.sh <tag> <ENV_VAR> [pairs] [test files...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; VAR=$2; P=${3:-3}; shift 3
O=gpurun_out
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
  grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 $P); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --profile-only > $O/${T}_b${v}_$i.json 2> $O/${T}_b${v}_$i.err || { tail -20 $O/${T}_b${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${T}_b${v}_$i.json'));print('$VAR=$v pair $i', d['value'], d['ms_per_step'])" | tee -a $O/${T}_ab.txt
  done
done
