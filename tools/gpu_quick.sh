cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pp_tests.log 2>&1; rc=$?; tail -15 gpurun_out/pp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/gemm_calls.py > gpurun_out/pp_calls.txt 2>&1 && tail -3 gpurun_out/pp_calls.txt && head -12 gpurun_out/pp_calls.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/pp_bench.json 2>gpurun_out/pp_bench.err; cat gpurun_out/pp_bench.json
