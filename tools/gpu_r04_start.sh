#!/bin/bash
# Round-4 call: touched GPU tests, config-B bench line, kernel stats B and E.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04a}
SEL=${2:-"tests/test_gpu_ptv3.py tests/test_gpu_render.py"}
K=${3:-"fused or sort or scan or embed or seq or cull or backward"}
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
step tests
timeout -k 10 1000 python -u -m pytest $SEL -k "$K" -m gpu -x -v --timeout 600 --timeout-method thread -s > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
step bench
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-traffic > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
step bench_attn_old
SFX_ATTN_SEQ=0 timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --no-traffic --no-psnr > $O/${T}_bench_attn0.json 2> $O/${T}_bench_attn0.err || { tail -30 $O/${T}_bench_attn0.err; exit 1; }
python -c "import json; d=json.load(open('$O/${T}_bench_attn0.json')); print('attn-seq off', d['value'], d['ms_per_step'])"
step profB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_pb -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_pb.log 2>&1 || { tail -20 $O/${T}_pb.log; exit 1; }
step profC
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_pc -o run --output-format csv -- python3 bench.py --config C --steps 3 --warmup 1 --profile-only > $O/${T}_pc.log 2>&1 || { tail -20 $O/${T}_pc.log; exit 1; }
step done
