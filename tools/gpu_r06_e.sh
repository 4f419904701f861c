#!/bin/bash
# FETCH_SIZE calibration on random record gathers (tools/fetch_gather_probe.hip); each counter group in its own pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06e2
mkdir -p $O
timeout -k 10 60 ./tools/fetch_gather_probe > $O/plain.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- ./tools/fetch_gather_probe > $O/fetch.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o run --output-format csv -- ./tools/fetch_gather_probe > $O/rdreq.log 2>&1 || true
