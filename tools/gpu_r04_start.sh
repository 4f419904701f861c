#!/bin/bash
# Round-4 opening call: the new / touched GPU tests, config-B bench line, config-E render kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
step() { echo "== $(date +%T) $*"; }
step tests
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_config_d.py tests/test_gpu_train.py -m gpu -x -v --timeout 600 --timeout-method thread -s > $O/r04a_tests.log 2>&1 || { tail -40 $O/r04a_tests.log; exit 1; }
tail -3 $O/r04a_tests.log
step bench
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline > $O/r04a_bench.json 2> $O/r04a_bench.err || { tail -30 $O/r04a_bench.err; exit 1; }
cat $O/r04a_bench.json
step profE
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r04a_pe -o run --output-format csv -- python3 bench.py --config E --steps 3 --warmup 1 --profile-only > $O/r04a_pe.log 2>&1 || { tail -20 $O/r04a_pe.log; exit 1; }
step done
