#!/bin/bash
# Round 5, run 10: launch floor of back-to-back graph kernels (tools/launch_floor.hip), one-sequence steady trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run10
mkdir -p $O
timeout -k 10 120 ./tools/launch_floor > $O/launch_floor.jsonl 2>&1 || { cat $O/launch_floor.jsonl; exit 1; }
cat $O/launch_floor.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof1 -o run -- \
  python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extras --probe none --host-frames 0 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
python tools/trace_steps.py $(find $O/prof1 -name '*kernel_trace.csv' | head -1) geometry_kernel 30 60 > $O/b1_steady.txt
cat $O/b1_steady.txt
rm -rf $O/prof1
