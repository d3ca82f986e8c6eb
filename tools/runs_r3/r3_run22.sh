#!/bin/bash
# Round-3 run 22: split-K for the under-filled fc2 launches (MMT_SK128): bench-path parity with it on, the
# fc2 sweep shapes, then a one-box env A/B at 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
MMT_SK128=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchpath.py > gpurun_out/tests22.log 2>&1
tail -2 gpurun_out/tests22.log
ARGS="" ENV_B="MMT_SK128=1" bash tools/ab_env.sh
ENV_B="MMT_SK128=2" bash tools/ab_env.sh
