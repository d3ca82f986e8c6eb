#!/bin/bash
# Round 5, run 26: MFMA-busy / LDS / wait counters of the final build at 32 sequences (halves off, two PMC passes), then
# the final measurements again on the final library (suite, smoke, the four bench lines)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_final2
mkdir -p $O
OUT=$O/pmc_mfma bash tools/pmc_mfma.sh || exit 1
python tools/pmc_mfma_summary.py $O/pmc_mfma > $O/pmc_mfma.txt 2>&1 || exit 1
rm -rf $O/pmc_mfma/p1 $O/pmc_mfma/p2
grep -E "gemm|attn" $O/pmc_mfma.txt | cut -c1-60,200- | head
FINAL_TAG=r5_final2 bash tools/runs_r5/r5_final_a.sh
