#!/bin/bash
# same-box A/B of two builds of libsfx (SFX_LIB): alternating default bench runs; usage:
#   bash tools/ab_lib.sh OUTDIR BASE_SO NEW_SO [ROUNDS] [extra bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$1; A=$2; B=$3; R=${4:-3}; shift 4
mkdir -p $O
for i in $(seq 1 $R); do
  for v in A B; do
    so=$A; [ $v = B ] && so=$B
    SFX_LIB=$so timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr "$@" > $O/bench_${v}$i.log 2>&1 || exit 3
    echo "$v $i $(tail -1 $O/bench_${v}$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
