#!/bin/bash
# WS GEMM ablations on a few shapes: full, no MFMA (abl1), no global loads (abl2), and the general kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for S in "37759 256 1024 20" "37759 1024 256 20 gelu" "37759 1024 256 20" "37759 256 256 20" "14764 512 2048 20"; do
  echo "-- $S"
  timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1
  SFX_LIB=splatformer_amd/exp_abl1.so timeout -k 5 60 python3 tools/gemm_one.py $S | sed 's/^/noMFMA /' || exit 1
  SFX_LIB=splatformer_amd/exp_abl2.so timeout -k 5 60 python3 tools/gemm_one.py $S | sed 's/^/noLOAD /' || exit 1
  SFX_GEMM_WS=0 timeout -k 5 60 python3 tools/gemm_one.py $S | sed 's/^/old /' || exit 1
done
