#!/bin/bash
# Round-3 run 35: qkv / fc1 at one half's rows under the f16x3 tile configs (256 x 128 / 128 x 256 register-pipelined
# tiles vs the 256 x 256 kernel and the 128 x 128 ones)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep35.jsonl
for cfg in -1 14 1 5 4 13 0 9; do
  if [ "$cfg" = "-1" ]; then unset MMT_SPLIT_CFG; else export MMT_SPLIT_CFG=$cfg; fi
  SHAPES=qkv_half,fc1_half,qkv_243,fc1_243,qkv_152,fc1_152 timeout -k 10 120 python tools/bench_f16x3.py >> gpurun_out/sweep35.jsonl
done
