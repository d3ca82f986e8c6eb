#!/bin/bash
# Round-3 run 33: proj (K = 768, N = 768) at one half's rows per CE stage under the f16x3 tile configs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep33.jsonl
for cfg in -1 8 0 11 2; do
  if [ "$cfg" = "-1" ]; then unset MMT_SPLIT_CFG; else export MMT_SPLIT_CFG=$cfg; fi
  SHAPES=proj_half,proj_243,proj_189,proj_152 timeout -k 10 120 python tools/bench_f16x3.py >> gpurun_out/sweep33.jsonl
done
