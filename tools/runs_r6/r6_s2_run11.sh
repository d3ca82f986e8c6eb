#!/bin/bash
# Round 6 (second session), run 11: the 128 x 256 tile's one-round rule at a lower fill threshold (MMT_W256_FILL=70: also
# the 244-token layers' 2 x 93 tiles) against the 90 % default -- A/B of the line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run11
mkdir -p $O
ROUNDS=3 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "" "MMT_W256_FILL=70" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
