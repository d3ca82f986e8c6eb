#!/bin/bash
# Round-3 run 27: DiMP conv epilogue operands (bias, residual, merge) by raw buffer loads issued together per row
# fragment instead of a dependent round trip each: DiMP GPU tests on the new library, one-box A/B of mfDiMP
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py > gpurun_out/tests27.log 2>&1
tail -2 gpurun_out/tests27.log
: > gpurun_out/ab.log
echo "# mfDiMP 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=30 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/ab_bench.sh
