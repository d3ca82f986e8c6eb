#!/bin/bash
# Round-3 run 21: f16x3 tile configs at the rows one half keeps after candidate elimination (HEAD library)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep21.jsonl
for cfg in -1 0 2 8 10 11 9 12; do
  if [ "$cfg" = "-1" ]; then unset MMT_SPLIT_CFG; else export MMT_SPLIT_CFG=$cfg; fi
  SHAPES=fc2_half,fc2_243,fc2_189,fc2_152,proj_152,fc1_152,qkv_152 timeout -k 10 120 python tools/bench_f16x3.py >> gpurun_out/sweep21.jsonl
done
