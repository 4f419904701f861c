#!/bin/bash
# round 5: host-side (Python) cost of the config-B step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_profile.py 20 > gpurun_out/r05x_host.txt 2>&1 || { tail -20 gpurun_out/r05x_host.txt; exit 1; }
head -4 gpurun_out/r05x_host.txt
