#!/bin/bash
# Round 6 (second session), run 5: the 128 x 256 tile by a one-round rule (>= 90 % of the slots, counting the other
# stream half, where 128 x 128 takes two rounds: proj / fc2 of the 320-token layers) -- A/B of the line, OSTrack-384
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run5
mkdir -p $O
ROUNDS=3 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "MMT_W256=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_W256=0" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
