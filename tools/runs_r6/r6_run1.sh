#!/bin/bash
# Round 6, run 1: baseline on this round's first box -- the default bench line, and a halves-off kernel trace of the
# 32-sequence step with per-layer durations of the 256 x 256 GEMMs (qkv / fc1 round counts)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run1
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench32.json 2> $O/bench32.err || { tail -5 $O/bench32.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench32.json')); print('vit32', d['value'], d['roofline']['frac'], {k: v['value'] for k, v in d['extra_workloads'].items()})"
MMT_OVERLAP_MIN=1000 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python3 bench.py --steps 20 --warmup 0 --no-cpu-baseline --no-extras --probe none > $O/trace_bench.log 2>&1 || { tail -5 $O/trace_bench.log; exit 1; }
TR=$(find $O/tr -name '*kernel_trace.csv' | head -n 1)
python tools/trace_layers.py $TR 'crop_kernel<true>' 5 gemm attn > $O/layers.txt
gzip -c $TR > $O/kernel_trace.csv.gz && rm -rf $O/tr
cat $O/layers.txt | tail -60
