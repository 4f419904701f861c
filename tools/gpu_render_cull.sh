#!/bin/bash
# culled eval render: parity tests, wall-clock A/B per config, kernel trace of the config-B render
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-rc}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py -x -v --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/render_bench.py B 10 > $O/${T}_rb_B.txt 2>&1 || { tail -20 $O/${T}_rb_B.txt; exit 1; }
cat $O/${T}_rb_B.txt
timeout -k 10 300 python -u tools/render_bench.py E 5 > $O/${T}_rb_E.txt 2>&1 || { tail -20 $O/${T}_rb_E.txt; exit 1; }
cat $O/${T}_rb_E.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 tools/render_bench.py B 3 > $O/${T}_prof.log 2>&1 || { tail -20 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | sort | sed -n 1p); [ -n "$f" ] && cut -d, -f1-4 "$f" | sed -n 1,30p
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -x -v --timeout 600 --timeout-method thread -k "render or cull" > $O/${T}_full.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_full.log | head -20
exit $rc
