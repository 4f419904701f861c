#!/bin/bash
# GEMM timing ablations (tools/gemm_ablate.py): which part of gemm_kernel bounds the config-B launches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
for m in 0 1 2 4 8 3 9 6 11 14 15; do
  SFX_GEMM_DEBUG=$m timeout -k 10 200 python -u tools/gemm_ablate.py > $O/abl_$m.jsonl 2>&1 || exit $m
  tail -1 $O/abl_$m.jsonl
done
