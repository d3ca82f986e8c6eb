#!/bin/bash
# Round 6, run 19: the step-boundary gap vs the scope of the per-step completion event's release (MMT_EVENT_DEVICE:
# (MMT_FRAME_QUERY and MMT_EVENT_DEVICE were experiment switches, removed after these runs)
# 0 system scope (default), 1 device scope, 2 no system fence); one sequence and 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run19
mkdir -p $O
for arm in 0 1 2; do
  MMT_EVENT_DEVICE=$arm TAG=r6_run19/b1_$arm STEPS=200 ARGS="--batch 1 --host-frames 0" bash tools/prof_bench.sh || exit 1
  python tools/trace_idle.py $(find $O/b1_$arm -name '*kernel_trace.csv' | head -1) 20 4 > $O/idle_b1_$arm.txt 2>&1 || true
  echo "== b1 event $arm"; cat $O/idle_b1_$arm.txt
done
find $O -name '*kernel_trace.csv' -delete
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "MMT_EVENT_DEVICE=0" "MMT_EVENT_DEVICE=1" "MMT_EVENT_DEVICE=2" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=2 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_EVENT_DEVICE=0" "MMT_EVENT_DEVICE=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
