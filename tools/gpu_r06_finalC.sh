#!/bin/bash
# round 6 final: config C lines (fp32 and reference precision) with the whole-scene CPU train baseline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06final
mkdir -p $O
timeout -k 10 900 python bench.py --config C --no-traffic > $O/bench_C.log 2>&1 || { tail -5 $O/bench_C.log; exit 1; }
tail -1 $O/bench_C.log | cut -c1-160
timeout -k 10 600 python bench.py --config C --no-traffic --no-cpu-baseline --train-prec amp > $O/bench_C_amp.log 2>&1 || { tail -5 $O/bench_C_amp.log; exit 1; }
tail -1 $O/bench_C_amp.log | cut -c1-160
