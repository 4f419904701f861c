#!/bin/bash
# Round 5: reference-precision (autocast-class) training mode -- unit tests, the config-C tests of both modes, and
# config C benches in both modes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_ptv3.py -k "reference_precision or split_precision" tests/test_gpu_train_ops.py \
  > gpurun_out/r05amp_units.log 2>&1 || { tail -30 gpurun_out/r05amp_units.log; exit 1; }
tail -3 gpurun_out/r05amp_units.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_config_c.py \
  > gpurun_out/r05amp_configC_tests.log 2>&1 || { tail -40 gpurun_out/r05amp_configC_tests.log; exit 1; }
grep -E "config C|passed|failed" gpurun_out/r05amp_configC_tests.log | tail -12
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 3 --no-traffic --no-cpu-baseline --train-prec amp > gpurun_out/r05amp_benchC_amp.json 2> gpurun_out/r05amp_benchC_amp.err || { tail -20 gpurun_out/r05amp_benchC_amp.err; exit 1; }
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 3 --no-traffic --no-cpu-baseline > gpurun_out/r05amp_benchC_fp32.json 2> gpurun_out/r05amp_benchC_fp32.err || { tail -20 gpurun_out/r05amp_benchC_fp32.err; exit 1; }
python - <<'PY'
import json
for m in ("amp", "fp32"):
    d = json.loads(open(f"gpurun_out/r05amp_benchC_{m}.json").read().strip().splitlines()[-1])
    print(m, d["value"], d["ms_per_step"], d["dtype"][:40])
PY
