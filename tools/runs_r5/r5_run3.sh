#!/bin/bash
# Round 5, run 3: the GPU suite on the build with the GEMM stamp-pointer fix (a vector reload + vmcnt(0) that drained
# the prologue's loads in every tile) and the early bias loads; one-box A/B against the round-start library at one
# and 32 sequences; the one-sequence GEMM study's Infinity-Cache (prefetched weights) mode
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head -20; tail -3 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt

rm -f gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b1.log; rm -f gpurun_out/ab.log
LIBDIR=abx ROUNDS=3 STEPS=60 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b32.log
cat $O/ab_b1.log $O/ab_b32.log
SHAPES=qkv,fc1,fc2,proj timeout -k 10 200 python tools/b1_gemm_study.py > $O/b1_gemm_mall.jsonl 2> $O/b1_gemm_mall.err || { tail -3 $O/b1_gemm_mall.err; exit 1; }
grep -E '"mall"|_single' $O/b1_gemm_mall.jsonl
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_dimp_stages.py > $O/dimp_stages.txt 2>&1
grep -E "^\[f16x3\] (filter after (7|8|10)|frame [1-6] (confidence|sample|state|patch))" $O/dimp_stages.txt
MMTRACK_LIB=$PWD/abv/libphase.so timeout -k 10 200 python tools/gemm256s_phases.py > $O/gemm256s_phases.jsonl 2> $O/gemm256s_phases.err || { tail -3 $O/gemm256s_phases.err; exit 1; }
cat $O/gemm256s_phases.jsonl
