#!/bin/bash
# Round-3 run 23: token kernels -- the fovea a8 stage in dynamic LDS sized by the sequence, variants without the
# deferred-reduce registers (libD), and libD with ln_prompt held to 80 VGPRs (libE); parity on libE, one-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
MMTRACK_LIB=$PWD/abx/libE_tok.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchpath.py tests/test_gpu_parity.py > gpurun_out/tests23.log 2>&1
tail -2 gpurun_out/tests23.log
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
