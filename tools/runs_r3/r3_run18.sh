#!/bin/bash
# Round-3 run 18: register-double-buffered gemm_kernel K loop -- f16x3 GEMM sweep (new vs HEAD library), GEMM
# GPU tests on the new library, then a one-box A/B of the whole step (ViT 32 / 1 sequences)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep18.jsonl
for lib in abx/libA_head.so abx/libB_pipe.so; do
  for cfg in -1 0 3 7 9 12 1 4; do
    if [ "$cfg" = "-1" ]; then unset MMT_SPLIT_CFG; else export MMT_SPLIT_CFG=$cfg; fi
    MMTRACK_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_f16x3.py | sed "s|^{|{\"lib\": \"$lib\", |" >> gpurun_out/sweep18.jsonl
  done
done
unset MMT_SPLIT_CFG
echo sweep done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_kernels.py tests/test_gpu_benchpath.py > gpurun_out/tests18.log 2>&1
tail -3 gpurun_out/tests18.log
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
