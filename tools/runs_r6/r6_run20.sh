#!/bin/bash
# Round 6, run 20: the LayerNorm affine requested at row-kernel entry (ln_kernel, ce_ln_kernel, final_norm_kernel,
# layer-0 prompt_reduce_kernel) instead of after the residual store -- one dependent memory round trip fewer per
# launch.  Parity (goldens, bitwise batch tests), then one sequence and 32 sequences against the previous build
# (abx/libprev.so via MMTRACK_LIB)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run20
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_benchpath.py tests/test_gpu_kernels.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
