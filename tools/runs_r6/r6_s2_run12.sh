#!/bin/bash
# Round 6 (second session), run 12: MFMA-busy / LDS counters of the final build (128 x 256 tile) at 32 sequences, halves off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run12
mkdir -p $O
OUT=$O/pmc timeout -k 10 400 bash tools/pmc_mfma.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_mfma_summary.py $O/pmc > $O/pmc_summary.txt 2>&1; rm -rf $O/pmc/p1 $O/pmc/p2
grep -E "gemm|attn" $O/pmc_summary.txt | cut -c1-60,200-260
