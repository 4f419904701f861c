#!/bin/bash
# config E: register-summed SubM conv on the large maps (default from 120k points) vs the pair path with the centre
# offset in the lists (SFX_SUBM_FUSED=0), same box, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
for i in 1 2; do
  for v in A B; do
    e="SFX_AB=1"; [ $v = B ] && e="SFX_SUBM_FUSED=0"
    env $e timeout -k 10 300 python -u bench.py --config E --steps 10 --no-traffic --no-cpu-baseline --no-psnr > $O/e_${v}$i.log 2>&1 || exit 7
    echo "E $v $i $(tail -1 $O/e_${v}$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
