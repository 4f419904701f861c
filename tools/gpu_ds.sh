cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_downsample.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ds_tests.log 2>&1; rc=$?; tail -25 gpurun_out/ds_tests.log; exit $rc
