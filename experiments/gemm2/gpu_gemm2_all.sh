#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_gemm2.sh ${1:-g2} && SFX_LIB=splatformer_amd/exp_stamp.so timeout -k 10 120 python -u tools/gemm2_stamps.py
