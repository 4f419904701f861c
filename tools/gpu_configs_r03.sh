#!/bin/bash
# bench lines of configs A and C on the round-3 build (no CPU baseline / PMC passes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-cfg3}
O=gpurun_out
mkdir -p $O
for c in A C; do
  timeout -k 10 500 python -u bench.py --config $c --no-cpu-baseline --no-traffic --no-psnr > $O/${T}_bench_$c.json 2> $O/${T}_bench_$c.err || { tail -20 $O/${T}_bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
