#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for S in "37759 256 1024 20" "37759 1024 256 20 gelu" "37759 256 256 20"; do
  SFX_LIB=splatformer_amd/exp_trace.so SFX_WS_TRACE_READ=1 timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1
done
