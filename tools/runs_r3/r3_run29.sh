#!/bin/bash
# Round-3 run 29: the LDS-patch stem with 16-row tiles (default) vs 8-row tiles vs the gather kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py > gpurun_out/tests29.log 2>&1
tail -2 gpurun_out/tests29.log
MMT_CONV_STEM_TH=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py -k stem >> gpurun_out/tests29.log 2>&1
tail -1 gpurun_out/tests29.log
ARGS="--workload mfdimp_rgbt --batch 32" ENV_B="MMT_CONV_STEM_TH=8" bash tools/ab_env.sh
ARGS="--workload mfdimp_rgbt --batch 32" ENV_B="MMT_CONV_STEM_OLD=1" bash tools/ab_env.sh
