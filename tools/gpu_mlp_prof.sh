#!/bin/bash
# fused MLP: debug check, micro-bench (chunk rotation on / off), SQ counters of the mlp kernels
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-mlpp}
O=gpurun_out
timeout -k 10 120 python -u tools/mlp_debug.py > $O/${T}_dbg.txt 2>&1 || { tail -20 $O/${T}_dbg.txt; exit 1; }
cat $O/${T}_dbg.txt
SFX_MLP_ROT=0 timeout -k 10 120 python -u tools/mlp_bench.py > $O/${T}_bench_rot0.txt 2>&1 || { tail -20 $O/${T}_bench_rot0.txt; exit 1; }
cat $O/${T}_bench_rot0.txt
timeout -k 10 120 python -u tools/mlp_bench.py > $O/${T}_bench.txt 2>&1 || { tail -20 $O/${T}_bench.txt; exit 1; }
cat $O/${T}_bench.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/${T}_sq1 -o run --output-format csv -- python3 tools/mlp_bench.py > $O/${T}_sq1.log 2>&1 || { tail -5 $O/${T}_sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/${T}_sq2 -o run --output-format csv -- python3 tools/mlp_bench.py > $O/${T}_sq2.log 2>&1 || { tail -5 $O/${T}_sq2.log; exit 1; }
echo done
