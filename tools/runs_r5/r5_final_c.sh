#!/bin/bash
# Round-5 final measurements, part C (after part B showed the default bench's extra-workload children inside the
# profiled process): the 32-sequence kernel traces and the ViT PMC traffic without them, then part A again on the
# final library (the staged DiMP conv epilogue)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${FINAL_TAG:-r5_final}
mkdir -p $O
rm -rf $O/prof32 $O/prof32_halves_off $O/pmc
TAG=${FINAL_TAG:-r5_final}/prof32 STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh || exit 1
MMT_OVERLAP_MIN=0 TAG=${FINAL_TAG:-r5_final}/prof32_halves_off STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh || exit 1
python tools/prof_split_resid.py $(find $O/prof32_halves_off -name '*kernel_trace.csv' | head -1) >> $O/prof32_halves_off/summary.txt 2>&1 || true
OUT=$O/pmc bash tools/pmc_bench.sh || exit 1
python tools/pmc_traffic.py $O/pmc $O/r05_pmc_traffic_fp32_b32.json > $O/pmc_traffic.txt 2>&1 || exit 1
head -12 $O/pmc_traffic.txt
rm -rf $O/pmc/fetch $O/pmc/write $O/pmc/l2
for d in prof32 prof32_halves_off; do head -14 $O/$d/summary.txt; done
FINAL_TAG=${FINAL_TAG:-r5_final} bash tools/runs_r5/r5_final_a.sh
