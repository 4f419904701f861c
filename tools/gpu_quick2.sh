cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_train.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/q2_tests.log 2>&1; rc=$?; tail -5 gpurun_out/q2_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/q2_bench$i.json 2>gpurun_out/q2_bench.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/q2_bench$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['gemm_ms_per_scene'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/q2_prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/q2_prof.log 2>&1
