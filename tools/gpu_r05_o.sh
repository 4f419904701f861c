#!/bin/bash
# round 5: register-summed SubM CPE (SFX_SUBM_FUSED=1) vs pair path on config E (500k), A/B alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for f in 1 0 1 0; do
  SFX_SUBM_FUSED=$f timeout -k 10 300 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/r05o_E_$f.log 2>&1 || { tail -5 gpurun_out/r05o_E_$f.log; exit 1; }
  echo "E fused=$f $(tail -1 gpurun_out/r05o_E_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
