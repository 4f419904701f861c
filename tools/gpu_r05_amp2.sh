#!/bin/bash
# round 5: config C kernel traces in both precision modes + the config-C tests (autocast oracle with loss scaling)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_train_ops.py -k "block_mlp_train or reference_precision or test_window_attention_bwd" > gpurun_out/r05amp_units2.log 2>&1 || { tail -30 gpurun_out/r05amp_units2.log; exit 1; }
tail -2 gpurun_out/r05amp_units2.log
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 3 --no-traffic --no-cpu-baseline --train-prec amp > gpurun_out/r05amp_benchC_amp2.json 2> gpurun_out/r05amp_benchC_amp2.err || { tail -20 gpurun_out/r05amp_benchC_amp2.err; exit 1; }
cut -c1-200 gpurun_out/r05amp_benchC_amp2.json
for m in amp fp32; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05amp_trace_$m -o run --output-format csv -- python3 bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --profile-only --train-prec $m > gpurun_out/r05amp_trace_$m.log 2>&1 || { tail -5 gpurun_out/r05amp_trace_$m.log; exit 1; }
done
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_config_c.py \
  > gpurun_out/r05amp_configC_tests2.log 2>&1 || { tail -40 gpurun_out/r05amp_configC_tests2.log; exit 1; }
grep -E "config C|passed|failed" gpurun_out/r05amp_configC_tests2.log | tail -12
