#!/bin/bash
# Round-4 A/B: config-B bench lines with the fused SubM conv / pipelined attention on and off, kernel stats of the
# old path, and the training render (fwd + bwd of 4 views 800x800) timing + kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r04f}
mkdir -p $O
line() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-traffic --no-psnr > $O/${T}_b_$tag.json 2> $O/${T}_b_$tag.err || { tail -30 $O/${T}_b_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/${T}_b_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
echo "== $(date +%T) bench A/B"
line old SFX_SUBM_FUSED=0 SFX_ATTN_SEQ=0 || exit 1
line fused SFX_SUBM_FUSED=1 SFX_ATTN_SEQ=0 || exit 1
line seq768 SFX_SUBM_FUSED=0 SFX_ATTN_SEQ=768 || exit 1
line seq1024 SFX_SUBM_FUSED=0 SFX_ATTN_SEQ=1024 || exit 1
line old2 SFX_SUBM_FUSED=0 SFX_ATTN_SEQ=0 || exit 1
echo "== $(date +%T) prof old"
SFX_SUBM_FUSED=0 SFX_ATTN_SEQ=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_pold -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > $O/${T}_pold.log 2>&1 || { tail -20 $O/${T}_pold.log; exit 1; }
echo "== $(date +%T) render train"
timeout -k 10 300 python -u tools/render_bench.py train > $O/${T}_rtrain.txt 2>&1 || { tail -20 $O/${T}_rtrain.txt; exit 1; }
cat $O/${T}_rtrain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prt -o run --output-format csv -- python3 tools/render_bench.py train > $O/${T}_prt.log 2>&1 || { tail -20 $O/${T}_prt.log; exit 1; }
echo "== $(date +%T) done"
