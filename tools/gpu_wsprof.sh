#!/bin/bash
# WS GEMM diagnosis on one shape: timing (WS on/off, per tile config) + SQ / cache counter passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=${1:-"37759 256 1024 20"}
P=${2:-wsp}
O=gpurun_out
for c in 0 1 2 3 4; do SFX_GEMM_WS_CFG=$c timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1; done
SFX_GEMM_WS=0 timeout -k 5 60 python3 tools/gemm_one.py $S || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $O/${P}1 -o run --output-format csv -- python3 tools/gemm_one.py $S > $O/${P}1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS -d $O/${P}2 -o run --output-format csv -- python3 tools/gemm_one.py $S > $O/${P}2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/${P}3 -o run --output-format csv -- python3 tools/gemm_one.py $S > $O/${P}3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY -d $O/${P}4 -o run --output-format csv -- python3 tools/gemm_one.py $S > $O/${P}4.log 2>&1
rc=$?
python3 - <<PY
import csv, glob, collections
for i in range(1, 5):
    fs = glob.glob("$O/${P}%d/**/*counter_collection.csv" % i, recursive=True)
    if not fs: print("pass", i, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        if "gemm" in k: print(i, k, {c: f"{x:.3g}" for c, x in v.items()})
PY
exit $rc
