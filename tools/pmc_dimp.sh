# MFMA / LDS / wait counters of the mfDiMP bench's kernels (tuning tool): two PMC passes, each its own run
set -e
OUT=${OUT:-gpurun_out/pmc_dimp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--workload mfdimp_rgbt --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --sync"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -- python bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -- python bench.py $ARGS > $OUT/p2.log 2>&1
python tools/pmc_mfma_summary.py $OUT > $OUT/summary.txt
rm -rf $OUT/p1 $OUT/p2
