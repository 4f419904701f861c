#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-rd}
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_full.py -v -x --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));print('B', d['value'],d['ms_per_step'])"
bash tools/gpu_prof_cfg.sh ${T}E E 2 | head -14
