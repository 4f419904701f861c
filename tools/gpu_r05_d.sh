#!/bin/bash
# round 5: counters of the fused SubM CPE microbench (C = 256 stage)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r05d_sq -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05d_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES -d gpurun_out/r05d_sq2 -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05d_sq2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/r05d_tcc -o run --output-format csv -- python3 tools/subm_bench.py --only 256 > gpurun_out/r05d_tcc.log 2>&1 || exit 1
echo done
