#!/bin/bash
# Round 6, run 18: the ~26 us gap between steps (decode -> next geometry) at 32 sequences -- frame-stream event skipped
# (MMT_FRAME_QUERY and MMT_EVENT_DEVICE were experiment switches, removed after these runs)
# when the caller's stream is idle (MMT_FRAME_QUERY=1, default) vs always recorded (=0), and halves off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run18
mkdir -p $O
for arm in "MMT_FRAME_QUERY=1" "MMT_FRAME_QUERY=0" "MMT_OVERLAP_MIN=0"; do
  t=$(echo $arm | tr '=' '_')
  env $arm TAG=r6_run18/$t STEPS=25 ARGS="--batch 32 --host-frames 0" bash tools/prof_bench.sh || exit 1
  python tools/trace_idle.py $(find $O/$t -name '*kernel_trace.csv' | head -1) 40 6 > $O/idle_$t.txt 2>&1 || true
  echo "== $arm"; cat $O/idle_$t.txt
done
env MMT_FRAME_QUERY=1 TAG=r6_run18/b1q STEPS=200 ARGS="--batch 1 --host-frames 0" bash tools/prof_bench.sh || exit 1
python tools/trace_idle.py $(find $O/b1q -name '*kernel_trace.csv' | head -1) 20 6 > $O/idle_b1q.txt 2>&1 || true
echo "== b1 query"; cat $O/idle_b1q.txt
env MMT_FRAME_QUERY=0 TAG=r6_run18/b1n STEPS=200 ARGS="--batch 1 --host-frames 0" bash tools/prof_bench.sh || exit 1
python tools/trace_idle.py $(find $O/b1n -name '*kernel_trace.csv' | head -1) 20 6 > $O/idle_b1n.txt 2>&1 || true
echo "== b1 no query"; cat $O/idle_b1n.txt
find $O -name '*kernel_trace.csv' -delete
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_FRAME_QUERY=0" "MMT_FRAME_QUERY=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "MMT_FRAME_QUERY=0" "MMT_FRAME_QUERY=1" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
