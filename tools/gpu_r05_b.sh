#!/bin/bash
# round 5: per-stage timing of the fused SubM CPE vs the pair path, kernel trace and SQ counters of the microbench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/subm_bench.py > gpurun_out/r05b_subm_bench.log 2>&1 || { tail -20 gpurun_out/r05b_subm_bench.log; exit 1; }
cat gpurun_out/r05b_subm_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b_trace -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05b_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r05b_sq -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05b_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r05b_sq2 -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05b_sq2.log 2>&1 || exit 1
echo done
