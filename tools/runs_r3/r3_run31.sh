#!/bin/bash
# Round-3 run 31: conv split-K over 512 slots for the long-K layers (libI) vs HEAD (libF): conv shapes, DiMP tests,
# one-box A/B of mfDiMP
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/conv31.jsonl
for lib in abx/libF_attn.so abx/libI_slots.so; do
  MMTRACK_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_conv_f16x3.py | sed "s|^{|{\"lib\": \"$lib\", |" >> gpurun_out/conv31.jsonl
done
MMTRACK_LIB=$PWD/abx/libI_slots.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py > gpurun_out/tests31.log 2>&1
tail -1 gpurun_out/tests31.log
: > gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=30 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/ab_bench.sh
