#!/bin/bash
# SQ counter passes over any python command: bash tools/pmc_cmd.sh <prefix> <python args...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=$1; shift
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}0 -o run -- python3 "$@" > gpurun_out/${P}0.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/${P}1 -o run --output-format csv -- python3 "$@" > gpurun_out/${P}1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS -d gpurun_out/${P}2 -o run --output-format csv -- python3 "$@" > gpurun_out/${P}2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/${P}3 -o run --output-format csv -- python3 "$@" > gpurun_out/${P}3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/${P}4 -o run --output-format csv -- python3 "$@" > gpurun_out/${P}4.log 2>&1
