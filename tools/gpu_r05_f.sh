#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for C in 64 256; do SFX_SUBM_OS_DEBUG=16 timeout -k 10 120 python -u tools/subm_bench.py --only $C > gpurun_out/r05f_stamps_$C.log 2>&1 || exit 1; done
grep -A62 "wave loader" gpurun_out/r05f_stamps_64.log | head -64
grep -A40 "wave loader" gpurun_out/r05f_stamps_256.log | head -42
