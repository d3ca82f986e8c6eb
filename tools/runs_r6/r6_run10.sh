#!/bin/bash
# Round 6, run 10: 320 x 256 tiles for every qkv / fc1 launch (MMT_T320=2) against the round rule, 32 sequences and
# OSTrack-384 (in the overlapped step the round count matters less than each tile's fixed prologue / epilogue)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run10
mkdir -p $O
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_T320=2" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_T320=2" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
