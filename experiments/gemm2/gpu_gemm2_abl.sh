#!/bin/bash
# gemm2 ablation variants (tools/build_variant.sh with -DG2_ABL=...): kernel time per variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base ${VARIANTS:-abl64 abl2 abl128 abl1}; do
  L=splatformer_amd/exp_$v.so; [ $v = base ] && L=splatformer_amd/libsfx.so
  SFX_LIB=$L timeout -k 10 120 python -u tools/gemm2_bench.py --quick 2>&1 | grep -v amdgpu.ids || exit 1
done
