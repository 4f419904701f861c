#!/bin/bash
# round 5: the whole GPU suite (timing check against the driver's budget) + smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations=25 \
  > gpurun_out/r05final_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r05final_suite.log; exit 1; }
tail -30 gpurun_out/r05final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05final_smoke.log 2>&1 || { tail -20 gpurun_out/r05final_smoke.log; exit 1; }
tail -1 gpurun_out/r05final_smoke.log
