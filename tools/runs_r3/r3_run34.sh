#!/bin/bash
# Round-3 run 34: N = 768, K <= 1024 f16x3 GEMMs (proj, patch) on the register-pipelined 64-deep tile: bench-path
# parity, then an env A/B against the 32-deep tile (MMT_SPLIT_K32) at 32 sequences and on OSTrack-384
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchpath.py tests/test_gpu_f16x3.py > gpurun_out/tests34.log 2>&1
tail -1 gpurun_out/tests34.log
ENV_B="MMT_SPLIT_K32=1" bash tools/ab_env.sh
ARGS="--workload ostrack384" ENV_B="MMT_SPLIT_K32=1" bash tools/ab_env.sh
