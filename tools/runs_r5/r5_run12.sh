#!/bin/bash
# Round 5, run 12: one sequence -- in-launch split-K combine now that only the head convs split without deferral
# (MMT_SK_INLAUNCH=1 write-through slabs, =2 release/acquire), env A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run12
mkdir -p $O
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_SK_INLAUNCH=1" "MMT_SK_INLAUNCH=2" > $O/ab_inlaunch_b1.txt 2>&1 || { tail -5 $O/ab_inlaunch_b1.txt; exit 1; }
cat $O/ab_inlaunch_b1.txt
