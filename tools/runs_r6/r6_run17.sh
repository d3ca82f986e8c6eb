#!/bin/bash
# Round 6, run 17: GPU idle inside the timed loop of the 32-sequence line (no host-frames phase after it, so the last
# 40 ms of the kernel trace are timed-loop steps), and of OSTrack-384
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run17
mkdir -p $O
TAG=r6_run17/prof32 STEPS=25 ARGS="--batch 32 --host-frames 0" bash tools/prof_bench.sh || exit 1
python tools/trace_idle.py $(find $O/prof32 -name '*kernel_trace.csv' | head -1) 40 15 > $O/b32_idle.txt 2>&1 || true
cat $O/b32_idle.txt
TAG=r6_run17/profost STEPS=12 ARGS="--workload ostrack384 --host-frames 0" bash tools/prof_bench.sh || exit 1
python tools/trace_idle.py $(find $O/profost -name '*kernel_trace.csv' | head -1) 40 15 > $O/ost_idle.txt 2>&1 || true
cat $O/ost_idle.txt
head -20 $O/profost/summary.txt
find $O -name '*kernel_trace.csv' -delete
