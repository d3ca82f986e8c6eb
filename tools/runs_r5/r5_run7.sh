#!/bin/bash
# Round 5, run 7: the GPU suite (-s, DiMP confidence drifts printed) with frames that no longer depend on the box's
# scalar type (synth.make_frames), packed-fp32 GELU in the staged epilogues; A/B of the packed GELU at 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run7
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head -20; tail -3 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
grep -E "max confidence rel|relative confidence differences|teacher-forced per-step|per-frame IoU" $O/gpu_suite.txt | cut -c1-300
grep -E "^\[(f16x3|fp32)\] (filter after (7|8|10)|frame [1-6] confidence)" $O/gpu_suite.txt
rm -f gpurun_out/ab.log
LIBDIR=abx3 ROUNDS=3 STEPS=60 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b32.log; rm -f gpurun_out/ab.log
LIBDIR=abx3 ROUNDS=3 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cp gpurun_out/ab.log $O/ab_b1.log
cat $O/ab_b1.log

cat $O/ab_b32.log
