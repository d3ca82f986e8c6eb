#!/bin/bash
# Round-3 run 36: qkv / fc1 with fewer than 160 256-wide tiles on the register-pipelined 128 x 128 tile (from 400
# 128-tiles): sweep, bench-path parity, env A/B against the previous rule
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
SHAPES=qkv_half,fc1_half,qkv_243,fc1_243,qkv_152,fc1_152 timeout -k 10 120 python tools/bench_f16x3.py > gpurun_out/sweep36.jsonl
cat gpurun_out/sweep36.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchpath.py > gpurun_out/tests36.log 2>&1
tail -1 gpurun_out/tests36.log
ENV_B="MMT_256S_MIN=128 MMT_SPLIT_K64_MIN=100000" bash tools/ab_env.sh
