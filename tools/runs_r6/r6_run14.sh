#!/bin/bash
# Round 6, run 14: fc2 on the eight-phase kernel where its tiles fill a round (the default rule, MMT_FC2_256S=1) against
# never (0), everywhere (2) and proj too where it fills a round (3) -- OSTrack-384 and the 32-sequence ViT line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run14
mkdir -p $O
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_FC2_256S=0" "" "MMT_FC2_256S=2" "MMT_FC2_256S=3" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
ROUNDS=2 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_FC2_256S=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
