#!/bin/bash
# Round-6 final measurements, part B: rocprofv3 kernel traces (32 sequences halves on / off, one sequence, mfDiMP)
# and the PMC traffic passes (ViT fc2 classes, mfDiMP feature net), summaries for profiles/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${FINAL_TAG:-r6_final}
mkdir -p $O
TAG=${FINAL_TAG:-r6_final}/prof32 STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh || exit 1
MMT_OVERLAP_MIN=0 TAG=${FINAL_TAG:-r6_final}/prof32_halves_off STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh || exit 1
python tools/prof_split_resid.py $(find $O/prof32_halves_off -name '*kernel_trace.csv' | head -1) >> $O/prof32_halves_off/summary.txt 2>&1 || true
TAG=${FINAL_TAG:-r6_final}/prof1 STEPS=200 ARGS="--batch 1" bash tools/prof_bench.sh || exit 1
TAG=${FINAL_TAG:-r6_final}/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
OUT=$O/pmc bash tools/pmc_bench.sh || exit 1
python tools/pmc_traffic.py $O/pmc $O/r06_pmc_traffic_fp32_b32.json > $O/pmc_traffic.txt 2>&1 || exit 1
head -12 $O/pmc_traffic.txt
OUT=$O/pmc_dimp DEST=$O/r06_pmc_traffic_dimp.json bash tools/pmc_dimp_traffic.sh || exit 1
rm -rf $O/pmc/fetch $O/pmc/write $O/pmc/l2
for d in prof32 prof32_halves_off prof1 profdimp; do head -14 $O/$d/summary.txt; done
# steady-state per-kernel tables (one sequence; mfDiMP)
python tools/trace_steps.py $(find $O/prof1 -name '*kernel_trace.csv' | head -1) crop_kernel 30 60 > $O/b1_steady.txt || true
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 4 60 > $O/dimp32_steady.txt || true
head -3 $O/b1_steady.txt $O/dimp32_steady.txt
python tools/trace_idle.py $(find $O/prof32 -name '*kernel_trace.csv' | head -1) 20 15 > $O/b32_idle.txt 2>&1 || true
head -20 $O/b32_idle.txt
