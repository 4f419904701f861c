#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v -s -x --timeout 300 --timeout-method thread > gpurun_out/${1:-tr}_train.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E |qkv grads|worst" gpurun_out/${1:-tr}_train.log | head -30
exit $rc
