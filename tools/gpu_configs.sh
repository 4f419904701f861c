#!/bin/bash
# bench.py lines for configs B, C, E (1 GPU) and D (2 ranks on one GPU is not D: D runs 1 rank, accum 4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/cfgs.jsonl; : > $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 >> $O 2> gpurun_out/cfgs_B.err || exit 1
timeout -k 10 400 python -u bench.py --config C --no-cpu-baseline --steps 3 --warmup 1 >> $O 2> gpurun_out/cfgs_C.err || exit 1
timeout -k 10 400 python -u bench.py --config D --no-cpu-baseline --steps 3 --warmup 1 >> $O 2> gpurun_out/cfgs_D.err || exit 1
timeout -k 10 400 python -u bench.py --config E --no-cpu-baseline --steps 5 --warmup 2 >> $O 2> gpurun_out/cfgs_E.err || exit 1
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['config']['workload'][:40], d['value'], d['unit'], d['ms_per_step'])"
