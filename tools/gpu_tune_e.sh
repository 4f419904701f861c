#!/bin/bash
# Config E tile sweep: every distinct GEMM launch of a 500k SH3 refine over all tile configurations.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/gemm_tune.py 500000 all 3 > gpurun_out/tune_e.jsonl 2>&1; rc=$?
tail -3 gpurun_out/tune_e.jsonl
exit $rc
