#!/bin/bash
# round 5: per-stage fused vs pair SubM CPE at config-E and intermediate scene sizes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 500000 250000 100000; do
  SFX_SUBM_FUSED=1 timeout -k 10 300 python tools/subm_bench.py --n $n > gpurun_out/r05p_subm_$n.log 2>&1 || { tail -5 gpurun_out/r05p_subm_$n.log; exit 1; }
  echo "== n=$n"; cat gpurun_out/r05p_subm_$n.log
done
