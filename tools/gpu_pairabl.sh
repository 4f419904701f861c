#!/bin/bash
# SubM pair-launch epilogue ablation: per-call breakdown with atomics (0), plain stores (1), no stores (2).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for v in 0 1 2; do
  echo "== $(date +%T) SFX_ABL_PAIR=$v"
  SFX_ABL_PAIR=$v timeout -k 10 200 python -u tools/gemm_calls.py > $O/pairabl_$v.txt 2>&1 || { tail -20 $O/pairabl_$v.txt; exit 1; }
  grep -E "subm_conv|total" $O/pairabl_$v.txt
done
