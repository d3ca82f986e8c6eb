#!/bin/bash
# Round 6, run 7: the default bench line (with its extra workloads), OSTrack-384 with / without the 320 x 256 rule,
# and a steady kernel trace of the one-sequence frame
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run7
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench32.json 2> $O/bench32.err || { tail -5 $O/bench32.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench32.json')); print('vit32', d['value'], d['roofline']['kernel'], d['roofline']['frac'], {k: v['value'] for k, v in d['extra_workloads'].items()})"
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_T320=0" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr1 -o run -- \
  python3 bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extras --probe none > $O/trace_b1.log 2>&1 || { tail -5 $O/trace_b1.log; exit 1; }
TR=$(find $O/tr1 -name '*kernel_trace.csv' | head -n 1)
python tools/trace_steps.py $TR 'crop_kernel<true>' 30 40 > $O/b1_steady_kernels.txt
gzip -c $TR > $O/b1_kernel_trace.csv.gz && rm -rf $O/tr1
head -30 $O/b1_steady_kernels.txt
