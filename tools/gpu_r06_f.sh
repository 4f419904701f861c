#!/bin/bash
# early stage-0 SubM map: A/B bench + kernel-trace gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
for i in 1 2 3; do
  SFX_NBR_EARLY=0 timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_off$i.log 2>&1 || exit 3
  timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr > $O/bench_on$i.log 2>&1 || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only --markers > $O/trace.log 2>&1 || exit 5
python3 tools/trace_gaps.py $O/trace > $O/gaps.txt 2>&1
timeout -k 10 300 python -u tools/host_profile.py 10 > $O/host_profile.txt 2>&1 || exit 6
