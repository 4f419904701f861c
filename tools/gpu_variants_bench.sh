#!/bin/bash
# bench.py (config B, no CPU baseline) for the default library and each experimental variant given
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = default ]; then L=splatformer_amd/libsfx.so; else L=splatformer_amd/exp_$v.so; fi
  SFX_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.err || exit 1
  echo "== $v: $(python3 -c "import json;d=json.load(open('gpurun_out/vb_$v.json'));print(d['value'],d['ms_per_step'],d['roofline']['gemm_ms_per_scene'])")"
done
