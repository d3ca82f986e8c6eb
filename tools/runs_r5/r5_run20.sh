#!/bin/bash
# Round 5, run 20: attention workgroup size per layer length at 32 sequences (MMT_ATTN_W=-1: 8 waves only where the
# 128-query tiles pad no more than the 64-query ones; 4: the 4-wave kernel everywhere), A/B against the default
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run20
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_ATTN_W=-1" "MMT_ATTN_W=4" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
