#!/bin/bash
# kernel trace of 5 marked config-B steps -> host gaps inside each step (tools/trace_gaps.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-gp}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${T}_trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only --markers > $O/${T}_trace.log 2>&1 || { tail -20 $O/${T}_trace.log; exit 1; }
python3 tools/trace_gaps.py $O/${T}_trace > $O/${T}_gaps.txt 2>&1; cat $O/${T}_gaps.txt
