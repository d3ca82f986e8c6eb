#!/bin/bash
# Round 5, run 6: the staged split epilogue in gemm_kernel (one-sequence qkv / fc1, head convs): tests, per-block
# stamps of the gemm_kernel shapes, A/B at one and 32 sequences; the DiMP per-frame patch diagnostic
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run6
mkdir -p $O
rm -f abx/libr5b_stampfix.so
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py tests/test_gpu_parity.py tests/test_gpu_kernels.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python tools/diag/dimp_patch_diag.py > $O/dimp_patch_diag.txt 2>&1; cat $O/dimp_patch_diag.txt | tail -8
timeout -k 10 200 python tools/gemm_stamps_f16x3.py > $O/gemm_stamps.jsonl 2> $O/gemm_stamps.err || { tail -3 $O/gemm_stamps.err; exit 1; }
cat $O/gemm_stamps.jsonl
rm -f gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b1.log; rm -f gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b32.log
cat $O/ab_b1.log $O/ab_b32.log
