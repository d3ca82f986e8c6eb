#!/bin/bash
# Round-3 run 20: register pipelining for every f16x3 gemm_kernel tile that fits (libC) vs only the LDS-bound ones
# (libB = HEAD), one box; then a rocprofv3 kernel trace of the 32-sequence line on HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
TAG=prof20 STEPS=40 bash tools/prof_bench.sh
head -12 gpurun_out/prof20/summary.txt
