#!/bin/bash
# Round 5, run 27: slots per wave of the deep prompt / LN1 kernels at 32 sequences (MMT_TOK_R: 2 default, 4, 1)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run27
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 700 bash tools/ab_envs.sh "" "MMT_TOK_R=4" "MMT_TOK_R=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
