# 64 x 64 few-tile GEMMs (one sequence) with 8 waves instead of 4 (tuning tool)
set -o pipefail
for r in 1 2 3; do
  for v in "MMT_NONE=1" "MMT_FEW_W8=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/w8_b1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/w8_b1.json'))
print('$v round $r B=1 fps', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['classes'].items()})"
  done
done > gpurun_out/w8_ab.log 2>&1
