#!/bin/bash
# Round-3 GPU run 8: evidence on the current build -- PMC HBM traffic of the ViT bench at 32 sequences, MFMA / wait /
# LDS counters of the mfDiMP kernels, rocprofv3 kernel summaries at 32 and 1 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
OUT=gpurun_out/r3_pmc_vit bash tools/pmc_bench.sh
python tools/pmc_traffic.py gpurun_out/r3_pmc_vit gpurun_out/r3_pmc_vit/r03_pmc_traffic_fp32_b32.json > gpurun_out/r3_pmc_vit/traffic.txt
rm -rf gpurun_out/r3_pmc_vit/fetch gpurun_out/r3_pmc_vit/write gpurun_out/r3_pmc_vit/l2
OUT=gpurun_out/r3_pmc_dimp bash tools/pmc_dimp.sh
O=gpurun_out/r3_pmc_dimp
ARGS="--workload mfdimp_rgbt --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --sync --probe none"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p3 -- python bench.py $ARGS > $O/p3.log 2>&1
python tools/pmc_mfma_summary.py $O/p3 > $O/summary_p3.txt
rm -rf $O/p3
TAG=r3_prof_b32 STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh
TAG=r3_prof_b1 STEPS=100 ARGS="--batch 1" bash tools/prof_bench.sh
for t in r3_prof_b32 r3_prof_b1; do find gpurun_out/$t -mindepth 1 -type d -exec rm -rf {} +; done
