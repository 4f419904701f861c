#!/bin/bash
# round 5: ablations of the fused SubM CPE kernel (SFX_SUBM_OS_DEBUG bits: 1 no MFMA, 2 no gathers, 4 no W DMA, 8 no epilogue)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for f in 0 1 2 4 8 15; do
  echo "== SFX_SUBM_OS_DEBUG=$f"
  SFX_SUBM_OS_DEBUG=$f timeout -k 10 120 python -u tools/subm_bench.py 2>&1 | grep "fused" || exit 1
done > gpurun_out/r05e_ablate.log 2>&1
cat gpurun_out/r05e_ablate.log
