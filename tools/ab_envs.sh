# A/B/C.. of environment settings on one box (tuning tool): each argument is one arm's environment ("" = none);
# ROUNDS rounds, arms alternating; ARGS are passed to bench.py.  usage: ROUNDS=3 ARGS="--batch 1" bash tools/ab_envs.sh "" "X=1"
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    env $envs timeout -k 10 200 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-extras --host-frames 0 --probe none ${ARGS:-} > gpurun_out/abenv.json 2>gpurun_out/abenv.err
    python -c "import json; d=json.load(open('gpurun_out/abenv.json')); print('arm $i [$envs] round $r fps', d['value'])"
  done
done
