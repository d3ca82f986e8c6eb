# MFMA / LDS / clock counters of the bench's kernels (tuning tool): two PMC passes, each its own run
set -e
OUT=${OUT:-gpurun_out/pmc_mfma}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS=${ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-extras --probe none --host-frames 0}
export MMT_OVERLAP_MIN=0
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -- python bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU_MFMA_MOPS_F16 --output-format csv -d $OUT/p2 -- python bench.py $ARGS > $OUT/p2.log 2>&1 || echo "pass 2 failed"
