#!/bin/bash
# Round-3 run 24: attention K / V tiles by LDS-DMA into a two-stage ring (one barrier per tile): attention and
# bench-path GPU tests on the new library, then one-box A/B against HEAD (libD_tok)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py tests/test_gpu_parity.py > gpurun_out/tests24.log 2>&1
tail -2 gpurun_out/tests24.log
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
echo "# OSTrack-384 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=30 ARGS="--workload ostrack384" bash tools/ab_bench.sh
