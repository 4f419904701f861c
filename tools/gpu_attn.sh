cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ptv3.py tests/test_gpu_train_ops.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/at_tests.log 2>&1; rc=$?; tail -3 gpurun_out/at_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/at_bench$i.json 2>gpurun_out/at_bench.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/at_bench$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['gemm_ms_per_scene'])"; done
bash tools/pmc_two.sh at_pmc bench.py --steps 1 --warmup 1 --profile-only && python3 tools/traffic_summary.py gpurun_out/at_pmcF/run_counter_collection.csv gpurun_out/at_pmcW/run_counter_collection.csv 2 gpurun_out/at_traffic.json | head -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/at_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --profile-only > gpurun_out/at_prof.log 2>&1
grep window_attn gpurun_out/at_prof/run_kernel_stats.csv | cut -c1-200
