#!/bin/bash
# Atomic-free SubM conv check: PTv3 / full-size GPU tests, then the bench with the per-pair partials (default) and
# with the atomic accumulation (SFX_SUBM_ATOMIC=1).  usage: bash tools/gpu_subm.sh <tag> [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-sm}
O=gpurun_out
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
if [ "$2" != "skip-tests" ]; then
step tests
timeout -k 10 700 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_full.py tests/test_gpu_real_clouds.py -v -x --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|^E " $O/${T}_tests.log | head -30
[ $rc -eq 0 ] || exit $rc
fi
for mode in 0 1 0 1; do
step bench atomic=$mode
SFX_SUBM_ATOMIC=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/${T}_bench_$mode.json 2> $O/${T}_bench_$mode.err || { tail -20 $O/${T}_bench_$mode.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_$mode.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_ms_per_unit'])"
done
step done
