#!/bin/bash
# Round 5, run 38: the 32-deep two-workgroups-per-CU tile for the short-K N = 768 GEMMs (proj, patch; MMT_SPLIT_K32)
# re-checked at 32 sequences after the 128 x 192 rule, one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run38
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_SPLIT_K32=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
