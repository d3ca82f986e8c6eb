# A/B of library variants on ONE box (box-to-box spread is larger than most single changes):
# runs bench.py alternately with each ab/lib*.so, ROUNDS times.  usage: ROUNDS=2 ARGS=... bash tools/ab_bench.sh  (LIBDIR: another directory of libraries; ab/ itself is gpurun-ignored)
set -e
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for lib in ${LIBDIR:-ab}/lib*.so; do
    v=$(MMTRACK_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-extras --probe none ${ARGS:-} 2>gpurun_out/ab_err.log | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
    echo "$lib round $r: $v" | tee -a gpurun_out/ab.log
  done
done
