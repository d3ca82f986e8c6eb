# A/B of an environment switch on one box (tuning tool): ENV_B="VAR=1" runs arm B with it, arm A without; 3 rounds
set -e
for r in 1 2 3; do
  for arm in A B; do
    if [ $arm = B ]; then envs="$ENV_B"; else envs=""; fi
    env $envs timeout -k 10 150 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none ${ARGS:-} > gpurun_out/abenv.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/abenv.json')); print('$arm round $r fps', d['value'])"
  done
done
