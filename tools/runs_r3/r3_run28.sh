#!/bin/bash
# Round-3 run 28: DiMP stem as 2-D tiles from an LDS input patch (one round trip per workgroup): DiMP GPU tests
# (the padded-input stem test compares it bit for bit with the gather kernel), env A/B of mfDiMP, kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py > gpurun_out/tests28.log 2>&1
tail -2 gpurun_out/tests28.log
ARGS="--workload mfdimp_rgbt --batch 32" ENV_B="MMT_CONV_STEM_OLD=1" bash tools/ab_env.sh
TAG=prof28 STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh
grep -i "stem\|maxpool\|true>" gpurun_out/prof28/summary.txt | head
