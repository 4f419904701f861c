#!/bin/bash
# gemm2 parity tests + shape bench + ablation (kernel times from HIP-graph replays).  usage: bash tools/gpu_gemm2.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-g2}
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm2.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
timeout -k 10 300 python -u tools/gemm2_bench.py > $O/${T}_bench.txt 2>&1 || { tail -30 $O/${T}_bench.txt; exit 1; }
cat $O/${T}_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${T}_prof -o run -- python -u tools/gemm2_bench.py > $O/${T}_prof.log 2>&1 || { tail -30 $O/${T}_prof.log; exit 1; }
python tools/kernel_runs.py $O/${T}_prof 9 > $O/${T}_runs.txt 2>&1; cat $O/${T}_runs.txt
