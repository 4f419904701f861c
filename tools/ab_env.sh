#!/bin/bash
# same-box A/B of two environment settings of one build: alternating default bench runs; usage:
#   [BENCH_ARGS="--config E"] bash tools/ab_env.sh OUTDIR "ENV_A" "ENV_B" [ROUNDS]      (e.g. "SFX_PAIR_LISTS=0" "")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$1; A=$2; B=$3; R=${4:-3}
mkdir -p $O
for i in $(seq 1 $R); do
  for v in A B; do
    e=$A; [ $v = B ] && e=$B
    env $e timeout -k 10 200 python -u bench.py --steps 20 --no-traffic --no-cpu-baseline --no-psnr $BENCH_ARGS > $O/bench_${v}$i.log 2>&1 || exit 7
    echo "$v $i $(tail -1 $O/bench_${v}$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
