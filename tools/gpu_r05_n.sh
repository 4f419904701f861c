#!/bin/bash
# round 5: exact-fp32 GEMM config-B bench line (verdict r04 item 7) + current config E line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SFX_GEMM_PREC=fp32 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/r05n_B_gemmfp32.log 2>&1 || { tail -5 gpurun_out/r05n_B_gemmfp32.log; exit 1; }
tail -1 gpurun_out/r05n_B_gemmfp32.log | cut -c1-160
SFX_GEMM_PREC=fp32 SFX_ATTN_PREC=fp32 timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/r05n_B_allfp32.log 2>&1 || { tail -5 gpurun_out/r05n_B_allfp32.log; exit 1; }
tail -1 gpurun_out/r05n_B_allfp32.log | cut -c1-160
timeout -k 10 400 python bench.py --config E --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-psnr > gpurun_out/r05n_E.log 2>&1 || { tail -5 gpurun_out/r05n_E.log; exit 1; }
tail -1 gpurun_out/r05n_E.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n_Etrace -o run --output-format csv -- python3 bench.py --config E --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-psnr --profile-only > gpurun_out/r05n_Etrace.log 2>&1 || { tail -5 gpurun_out/r05n_Etrace.log; exit 1; }
echo done
