#!/bin/bash
# Round 6, run 3: is the 8-phase 256 x 256 kernel faster per FLOP than the 128 x 128 kernel on fc2's N = 768?
# (MMT_SPLIT_CFG=14 pins the 256 x 256 kernel; fc2_sk2_emul = the FLOPs of fc2 at 32 sequences in one round of
# 240 K = 1536 tiles)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run3
mkdir -p $O
for cfg in -1 14; do
  MMT_SPLIT_CFG=$cfg SHAPES=fc2,fc2_sk2_emul,fc2_k1536,fc2_half timeout -k 10 120 python tools/bench_f16x3.py >> $O/bench.jsonl 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
done
cat $O/bench.jsonl
