#!/bin/bash
# the full GPU suite as the driver runs it (timed), smoke, default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 900 --timeout-method thread --durations 25 > $O/suite.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit 3
