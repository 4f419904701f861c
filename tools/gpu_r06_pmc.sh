#!/bin/bash
# round 6 final: per-kernel PMC passes of config B (tools/kernel_pmc.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python tools/kernel_pmc.py run gpurun_out/r06_pmc > gpurun_out/r06_pmc.log 2>&1 || { tail -20 gpurun_out/r06_pmc.log; exit 1; }
python tools/kernel_pmc.py summarize gpurun_out/r06_pmc > gpurun_out/r06_pmc_summary.txt 2>&1
head -20 gpurun_out/r06_pmc_summary.txt
