#!/bin/bash
# Round-3 run 25: gemm256s ring of 10 half-tile slots (160 KB, 8 half-tiles in flight) vs 8 (HEAD's schedule,
# refactored): f16x3 GEMM tests on the 10-slot library, qkv / fc1 sweep, one-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
MMTRACK_LIB=$PWD/abx/libG10_256s.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py > gpurun_out/tests25.log 2>&1
tail -2 gpurun_out/tests25.log
: > gpurun_out/sweep25.jsonl
for lib in abx/libF_attn.so abx/libG8_256s.so abx/libG10_256s.so; do
  MMTRACK_LIB=$PWD/$lib SHAPES=fc1,qkv,fc1_152,qkv_152 timeout -k 10 120 python tools/bench_f16x3.py | sed "s|^{|{\"lib\": \"$lib\", |" >> gpurun_out/sweep25.jsonl
done
cat gpurun_out/sweep25.jsonl
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh
