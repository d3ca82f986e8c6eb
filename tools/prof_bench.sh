# rocprofv3 kernel-trace --stats of a bench.py run + per-step breakdown (tuning tool).
# usage: TAG=name STEPS=25 ARGS="--batch 32" bash tools/prof_bench.sh
set -e
TAG=${TAG:-prof}
STEPS=${STEPS:-25}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python bench.py --steps $STEPS --warmup 0 --no-cpu-baseline --no-extras --probe none ${ARGS:-} > $OUT/bench.log 2>&1
STATS=$(find $OUT -name '*kernel_stats.csv' | head -n 1)
cp $STATS $OUT/kernel_stats.csv
python tools/prof_summary.py $OUT/kernel_stats.csv auto 30 > $OUT/summary.txt
