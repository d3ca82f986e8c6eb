# HBM traffic of the bench's kernels: rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs,
# counters only with --kernel-trace semantics, no sys/runtime trace) over a short bench.py run.
set -e
OUT=${OUT:-gpurun_out/pmc_bench}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS=${ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-extras --probe none --host-frames 0}
# the timing probe's launch shapes: two-stream halves off (pmc_traffic.py assigns classes by layer order)
export MMT_OVERLAP_MIN=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2 -- python bench.py $ARGS > $OUT/l2.log 2>&1
