#!/bin/bash
# Round-3 A/B 17: HEAD vs batched epilogue loads, one box: ViT 32 / 1 sequences and mfDiMP
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out
: > gpurun_out/ab.log
echo "# ViT 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=60 bash tools/ab_bench.sh
echo "# ViT 1" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=300 ARGS="--batch 1" bash tools/ab_bench.sh
echo "# mfDiMP 32" >> gpurun_out/ab.log
LIBDIR=abx ROUNDS=2 STEPS=30 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/ab_bench.sh
