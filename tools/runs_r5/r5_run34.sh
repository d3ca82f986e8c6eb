#!/bin/bash
# Round 5, run 34: MFMA-busy / LDS / wait counters of the mfDiMP step and of the one-sequence frame (two PMC passes each)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run34
mkdir -p $O
ARGS="--workload mfdimp_rgbt --steps 5 --warmup 2 --no-cpu-baseline --no-extras --probe none --host-frames 0" OUT=$O/dimp bash tools/pmc_mfma.sh || exit 1
python tools/pmc_mfma_summary.py $O/dimp > $O/pmc_mfma_dimp.txt 2>&1 || exit 1
rm -rf $O/dimp/p1 $O/dimp/p2
ARGS="--batch 1 --steps 30 --warmup 5 --no-cpu-baseline --no-extras --probe none --host-frames 0" OUT=$O/b1 bash tools/pmc_mfma.sh || exit 1
python tools/pmc_mfma_summary.py $O/b1 > $O/pmc_mfma_b1.txt 2>&1 || exit 1
rm -rf $O/b1/p1 $O/b1/p2
grep -E "conv_f16x3|patch" $O/pmc_mfma_dimp.txt | cut -c1-60,200- | head -5
grep -E "gemm|attn" $O/pmc_mfma_b1.txt | cut -c1-60,200- | head -6
