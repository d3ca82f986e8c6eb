#!/bin/bash
# Round-3 GPU run 11: MFMA / wait / LDS counters of the conv v3 mainloop (mfDiMP bench, 32 sequences)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
OUT=gpurun_out/r3_pmc_dimp3 bash tools/pmc_dimp.sh
O=gpurun_out/r3_pmc_dimp3
ARGS="--workload mfdimp_rgbt --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --sync --probe none"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p3 -- python bench.py $ARGS > $O/p3.log 2>&1
python tools/pmc_mfma_summary.py $O/p3 > $O/summary_p3.txt
rm -rf $O/p3
