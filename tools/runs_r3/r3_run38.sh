#!/bin/bash
# Round-3 run 38 (evidence on the final build): bench lines (ViT 32, OSTrack-384, mfDiMP 32), rocprofv3 kernel
# summaries of the 32-sequence line with the two-stream halves on (as timed) and off (the probe's launch shapes,
# to set against the line's per-launch fc2 time), and the SURVEY §8 row tool (SiamFC on the HIP backbone)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run38
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_b32.json 2> $O/bench_b32.err || exit 1
cat $O/bench_b32.json
TAG=r3_run38/prof32 STEPS=40 bash tools/prof_bench.sh || exit 1
MMT_OVERLAP_MIN=0 TAG=r3_run38/prof32_halves_off STEPS=40 bash tools/prof_bench.sh || exit 1
timeout -k 10 300 python bench.py --workload ostrack384 --no-cpu-baseline > $O/bench_ost.json 2> $O/bench_ost.err || exit 1
timeout -k 10 300 python bench.py --workload mfdimp_rgbt --batch 32 --no-cpu-baseline > $O/bench_dimp.json 2> $O/bench_dimp.err || exit 1
timeout -k 10 300 python tools/bench_rows.py --cpu-seconds 3 > $O/rows.jsonl 2> $O/rows.err || exit 1
for f in $O/bench_*.json; do echo "$f: $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline'].get('kernel'), d['roofline'].get('frac'), d['roofline'].get('avg_launch_us'))")"; done
head -4 gpurun_out/r3_run38/prof32_halves_off/summary.txt
