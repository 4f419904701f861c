cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pool_tests.log 2>&1; rc=$?; tail -15 gpurun_out/pool_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/pool_bench.json 2>gpurun_out/pool_bench.err; rc=$?; cat gpurun_out/pool_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pool_prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/pool_prof.log 2>&1
