#!/bin/bash
# Round 5, run 13: one-sequence launch cuts -- candidate elimination fused into the LN2 that gathers its survivors
# (ce_ln_kernel) and the crop geometry formed by the crop kernel (no geometry launch): full GPU suite, env A/B at one
# sequence (MMT_CE_FUSED=0 / MMT_GEOM_KERNEL=1 switch each back), steady trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run13
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_CE_FUSED=0" "MMT_GEOM_KERNEL=1" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof1 -o run -- \
  python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extras --probe none --host-frames 0 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
python tools/trace_steps.py $(find $O/prof1 -name '*kernel_trace.csv' | head -1) crop_kernel 30 60 > $O/b1_steady.txt
head -3 $O/b1_steady.txt
rm -rf $O/prof1
