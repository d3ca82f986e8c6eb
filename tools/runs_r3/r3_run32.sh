#!/bin/bash
# Round-3 run 32: the conv epilogue operands batched per row fragment (libB_epi) vs HEAD (libA_head), per shape
# and end to end
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/conv32.jsonl
for lib in abx/libA_head.so abx/libB_epi.so abx/libA_head.so abx/libB_epi.so; do
  MMTRACK_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_conv_f16x3.py | sed "s|^{|{\"lib\": \"$lib\", |" >> gpurun_out/conv32.jsonl
done
: > gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=30 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/ab_bench.sh
