#!/bin/bash
# re-sweep the GEMM tile table on the current kernels (config B refine launches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 600 python -u tools/gemm_tune.py 100000 all 1 > $O/tune.jsonl 2>&1 || exit 1
