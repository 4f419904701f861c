#!/bin/bash
# GEMM per-call timings of one refine for the default library and each experimental variant given
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = default ]; then L=splatformer_amd/libsfx.so; else L=splatformer_amd/exp_$v.so; fi
  SFX_LIB=$PWD/$L timeout -k 10 200 python3 tools/gemm_calls.py > gpurun_out/var_$v.txt 2>&1 || exit 1
  echo "== $v: $(tail -1 gpurun_out/var_$v.txt)"; head -8 gpurun_out/var_$v.txt | grep -v amdgpu.ids
done
