#!/bin/bash
# Round-3 run 19: register-pipelined gemm_kernel only where the LDS ring already holds the CU (fc2's 2-stage 64-deep
# tile): f16x3 sweep of the default configs, GEMM GPU tests, one-box A/B (ViT 32 / 1 sequences)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep19.jsonl
for lib in abx/libA_head.so abx/libB_pipe.so; do
  for cfg in -1 0 9 1; do
    if [ "$cfg" = "-1" ]; then unset MMT_SPLIT_CFG; else export MMT_SPLIT_CFG=$cfg; fi
    MMTRACK_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_f16x3.py | sed "s|^{|{\"lib\": \"$lib\", |" >> gpurun_out/sweep19.jsonl
  done
done
unset MMT_SPLIT_CFG
echo sweep done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_kernels.py tests/test_gpu_benchpath.py > gpurun_out/tests19.log 2>&1
tail -3 gpurun_out/tests19.log
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
