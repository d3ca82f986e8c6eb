#!/bin/bash
# Round-3 run 30: f16x3 conv timing on the DiMP shapes under the split / tile knobs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/conv30.jsonl
timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
MMT_CONV_SLOTS=512 timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
MMT_CONV_SLOTS=1024 timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
MMT_CONV_PREFER64=1 timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
MMT_CONV_PREFER64=1 MMT_CONV_SLOTS=512 timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
MMT_CONV_NOSPLIT=1 timeout -k 10 120 python tools/bench_conv_f16x3.py >> gpurun_out/conv30.jsonl
