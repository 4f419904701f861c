#!/bin/bash
# Round-4 certification call 2: the default bench line (with CPU baseline, PMC traffic, PSNR) and configs E, A, C.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04_final}
mkdir -p $O
run() {  # tag, timeout, args...
  local tag=$1 to=$2; shift 2
  echo "== $(date +%T) bench $tag"
  timeout -k 10 $to python -u bench.py "$@" > $O/${T}_bench_$tag.json 2> $O/${T}_bench_$tag.err || { tail -30 $O/${T}_bench_$tag.err; return 1; }
  cut -c1-400 $O/${T}_bench_$tag.json
}
run B 700 && run E 400 --config E --steps 5 --no-cpu-baseline --no-traffic && \
  run A 300 --config A --steps 20 --no-cpu-baseline --no-traffic && \
  run C 400 --config C --steps 5 --no-cpu-baseline --no-traffic || exit 1
echo "== $(date +%T) done"
