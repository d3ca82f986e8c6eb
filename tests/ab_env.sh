# A/B of environment knobs on ONE box (box-to-box spread exceeds most single changes): runs bench.py
# alternately under each "VAR=value ..." setting of AB_SETS (separated by ';'), ROUNDS times.
# usage: ROUNDS=3 AB_SETS="MMT_X=0;MMT_X=1" ARGS="--batch 32" bash tests/ab_env.sh
set -e
ROUNDS=${ROUNDS:-3}
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "$AB_SETS"
for r in $(seq 1 $ROUNDS); do
  for set in "${SETS[@]}"; do
    v=$(env $set timeout -k 10 200 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --probe none ${ARGS:-} 2>>gpurun_out/ab_err.log | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
    echo "[$set] round $r: $v" | tee -a gpurun_out/ab.log
  done
done
