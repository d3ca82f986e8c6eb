#!/bin/bash
# Round 5, run 5: the LDS-staged split epilogue of gemm256s (qkv / fc1 at 32 sequences): op-level and path parity
# tests, phase stamps, one-box A/B at 32 sequences against the previous build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run5
mkdir -p $O
rm -f abx/libr5a_base.so
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py tests/test_gpu_parity.py tests/test_gpu_kernels.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
MMTRACK_LIB=$PWD/abv/libphase.so timeout -k 10 200 python tools/gemm256s_phases.py > $O/gemm256s_phases.jsonl 2> $O/gemm256s_phases.err || { tail -3 $O/gemm256s_phases.err; exit 1; }
cat $O/gemm256s_phases.jsonl
rm -f gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b32.log
cat $O/ab_b32.log
