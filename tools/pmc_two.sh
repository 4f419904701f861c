#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over one python command: bash tools/pmc_two.sh <prefix> <python args...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=$1; shift
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}F -o run --output-format csv -- python3 "$@" > gpurun_out/${P}F.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}W -o run --output-format csv -- python3 "$@" > gpurun_out/${P}W.log 2>&1
