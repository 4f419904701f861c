#!/bin/bash
# culled training render: render + config-C parity tests, fwd+bwd timing, kernel trace of the training render
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-rt}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_config_c.py -x -v --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/render_bench.py train > $O/${T}_train.txt 2>&1 || { tail -20 $O/${T}_train.txt; exit 1; }
cat $O/${T}_train.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 tools/render_bench.py train > $O/${T}_prof.log 2>&1 || { tail -20 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | sort | sed -n 1p); [ -n "$f" ] && cut -d, -f1-4 "$f" | sed -n 1,16p
