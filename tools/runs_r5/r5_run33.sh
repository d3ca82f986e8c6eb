#!/bin/bash
# Round 5, run 33: GEMM launch knobs re-checked at 32 sequences after the 128 x 192 rule (short-K super-tile height,
# the 128 x 128 threshold, split-K for under-filled long-K residual GEMMs), one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run33
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 1000 bash tools/ab_envs.sh "" "MMT_GM=4" "MMT_GM=16" "MMT_SPLIT_T128=128" "MMT_SK128=2" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
