#!/bin/bash
# Round 6, run 12: MFMA-busy / LDS counters of the 32-sequence step's kernels on the final build (halves off, the probe's
# launch shapes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run12
mkdir -p $O
OUT=$O/pmc timeout -k 10 400 bash tools/pmc_mfma.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_mfma_summary.py $O/pmc > $O/pmc_summary.txt 2>&1; rm -rf $O/pmc/p1 $O/pmc/p2
cut -c1-60,200-260 $O/pmc_summary.txt | head -30
