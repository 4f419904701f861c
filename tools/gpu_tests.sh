#!/bin/bash
# GPU tests only (optionally a subset): bash tools/gpu_tests.sh <tag> [pytest args...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-t}; shift
timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread --durations=10 "$@" > gpurun_out/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E  " gpurun_out/${T}_tests.log | head -40
exit $rc
