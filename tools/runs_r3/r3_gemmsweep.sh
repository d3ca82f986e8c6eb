#!/bin/bash
# f16x3 tile-config sweep on the N = 768 / 2304 / 3072 shapes (kernel alone, halves off)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_gemmsweep
mkdir -p $O
for c in -1 0 9 2 10 1 4 5 6 13 14; do
  MMT_SPLIT_CFG=$c timeout -k 10 120 python tools/bench_f16x3.py >> $O/sweep.jsonl 2>> $O/err.log || exit $?
done
