#!/bin/bash
# Round 5, run 21: launch-shape knobs re-checked on the round-5 kernels at 32 sequences (stream parts 3 / 4, the 256 x 256
# kernel's tile threshold, the long-K super-tile height), one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run21
mkdir -p $O
ROUNDS=3 STEPS=60 timeout -k 10 900 bash tools/ab_envs.sh "" "MMT_NPARTS=3" "MMT_NPARTS=4" "MMT_GM_LONGK=2" "MMT_GM_LONGK=8" "MMT_256S_MIN=256" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
