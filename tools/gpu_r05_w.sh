#!/bin/bash
# round 5: V^T chunk swizzle in the attention kernels -- attention parity (fwd, bwd, flash), full B parity, B bench,
# then the per-kernel PMC passes of config B (tools/kernel_pmc.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ptv3.py tests/test_gpu_train_ops.py -k "attention or attn" \
  > gpurun_out/r05w_attn.log 2>&1 || { echo "attn tests failed"; tail -30 gpurun_out/r05w_attn.log; exit 1; }
tail -1 gpurun_out/r05w_attn.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "config_b or config_a" \
  > gpurun_out/r05w_full.log 2>&1 || { echo "full tests failed"; tail -30 gpurun_out/r05w_full.log; exit 1; }
tail -1 gpurun_out/r05w_full.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05w_B.log 2>&1 || { tail -5 gpurun_out/r05w_B.log; exit 1; }
tail -1 gpurun_out/r05w_B.log | cut -c1-170
timeout -k 10 900 python tools/kernel_pmc.py run gpurun_out/r05w_pmc > gpurun_out/r05w_pmc.log 2>&1 || { tail -20 gpurun_out/r05w_pmc.log; exit 1; }
python tools/kernel_pmc.py summarize gpurun_out/r05w_pmc > gpurun_out/r05w_pmc_summary.txt 2>&1
echo done
