cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_ptv3.py tests/test_gpu_downsample.py -v -x --timeout 240 --timeout-method thread -k "project or ring or wide or fps or empty or fused or bin_and" > $O/r02c_tests.log 2>&1; echo rc=$?; tail -25 $O/r02c_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -v --timeout 300 --timeout-method thread --durations=0 > $O/r02c_full.log 2>&1; echo rc=$?; tail -40 $O/r02c_full.log
