#!/bin/bash
# Round 5, run 18: the deep prompt reduce and LN1 as one launch (prompt_ln_kernel, per-sequence barrier): its bitwise
# test first (alone, short limit: a broken barrier shows as a time-out here), the full GPU suite, A/B at one sequence
# (MMT_PROMPT_FUSED=0 switches it off) and at 32 (MMT_PROMPT_FUSED=64 switches it on), steady trace at one sequence
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run18
mkdir -p $O
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fused_prompt_ln > $O/fused_test.txt 2>&1 || { tail -30 $O/fused_test.txt; exit 1; }
grep -E "PASS|FAIL" $O/fused_test.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head; tail -3 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_PROMPT_FUSED=0" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=3 STEPS=60 timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_PROMPT_FUSED=64" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof1 -o run -- \
  python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extras --probe none --host-frames 0 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
python tools/trace_steps.py $(find $O/prof1 -name '*kernel_trace.csv' | head -1) crop_kernel 30 60 > $O/b1_steady.txt
head -12 $O/b1_steady.txt
rm -rf $O/prof1
