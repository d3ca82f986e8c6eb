#!/bin/bash
# Round 5, run 35: the DiMP conv launch plan re-checked on the round-5 kernels (layer3's 1 x 1 convs make 324 workgroups
# for 512 slots): 64-wide tiles below 512 tiles (MMT_CONV_PREFER64), split-K counted against 512 slots (MMT_CONV_SLOTS)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run35
mkdir -p $O
ROUNDS=3 STEPS=30 ARGS="--workload mfdimp_rgbt" timeout -k 10 900 bash tools/ab_envs.sh "" "MMT_CONV_PREFER64=1" "MMT_CONV_SLOTS=512" > $O/ab_dimp.txt 2>&1 || { tail -5 $O/ab_dimp.txt; exit 1; }
cat $O/ab_dimp.txt
