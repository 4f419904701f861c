#!/bin/bash
# PTv3 + full-size B refine tests, host-gap trace, two 20-step bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-q3}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_full.py::test_config_b_refine -x -v --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_gaps.sh ${T}g || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --profile-only > $O/${T}_b$i.json 2> $O/${T}_b$i.err || { tail -20 $O/${T}_b$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_b$i.json'));print('bench', d['value'], d['ms_per_step'])"
done
