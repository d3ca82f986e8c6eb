# split-K slice count rounded down (workgroups <= CUs: one round) vs up, at one sequence (tuning tool)
set -o pipefail
for r in 1 2 3; do
  for v in "MMT_SPLITK_CEIL=1" "MMT_NONE=1" "MMT_SPLITK_MINKT=3" "MMT_SPLITK_MAX=16 MMT_SPLITK_MINKT=3"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/skr_b1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/skr_b1.json'))
print('$v round $r B=1 fps', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['classes'].items()})"
  done
done > gpurun_out/skr_ab.log 2>&1
