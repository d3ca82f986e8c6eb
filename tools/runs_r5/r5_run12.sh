#!/bin/bash
# Round 5, run 12: mfDiMP steady-state kernel trace after the downsample / sampler fusions; one-sequence in-launch
# split-K combine env A/B (only the head convs split without deferral now)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run12
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profd -o run -- \
  python bench.py --workload mfdimp_rgbt --steps 40 --warmup 5 --no-cpu-baseline --no-extras --probe none > $O/profd.log 2>&1 || { tail -5 $O/profd.log; exit 1; }
python tools/trace_steps.py $(find $O/profd -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 8 60 > $O/dimp_steady.txt
cat $O/dimp_steady.txt
rm -rf $O/profd
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_SK_INLAUNCH=1" "MMT_SK_INLAUNCH=2" > $O/ab_inlaunch_b1.txt 2>&1 || { tail -5 $O/ab_inlaunch_b1.txt; exit 1; }
cat $O/ab_inlaunch_b1.txt
