cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/sq1 -o run --output-format csv -- python3 tools/gemm_one.py > gpurun_out/sq1.log 2>&1
rc=$?; tail -3 gpurun_out/sq1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/sq2 -o run --output-format csv -- python3 tools/gemm_one.py > gpurun_out/sq2.log 2>&1
rc=$?; tail -3 gpurun_out/sq2.log; exit $rc
