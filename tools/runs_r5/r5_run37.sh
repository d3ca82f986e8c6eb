#!/bin/bash
# Round 5, run 37: split-K minimum K-tiles per slice at one sequence (MMT_SPLITK_MINKT 4 default, 3, 2: proj's K = 768
# then splits 4 / 6 ways instead of 3), one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run37
mkdir -p $O
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_SPLITK_MINKT=3" "MMT_SPLITK_MINKT=2" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
