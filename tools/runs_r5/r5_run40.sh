#!/bin/bash
# Round 5, run 40: super-tile height of the 256 x 256 kernel's tile order (MMT_GM256: 4 default, 2, 8), 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run40
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 700 bash tools/ab_envs.sh "" "MMT_GM256=2" "MMT_GM256=8" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
