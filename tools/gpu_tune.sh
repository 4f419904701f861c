#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/gemm_tune.py > gpurun_out/${1:-tune}.jsonl 2> gpurun_out/${1:-tune}.err; rc=$?
tail -3 gpurun_out/${1:-tune}.jsonl; exit $rc
