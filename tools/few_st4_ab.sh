# 4-deep LDS rings for the one-sequence 8-wave 64 x 64 GEMMs (MMT_FEW_ST4) and split-K slices (MMT_SK_ST4) (tuning tool)
set -o pipefail
for r in 1 2 3; do
  for v in "MMT_NONE=1" "MMT_FEW_ST4=1" "MMT_SK_ST4=1" "MMT_FEW_ST4=1 MMT_SK_ST4=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 300 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/st4_b1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/st4_b1.json'))
print('$v round $r B=1 fps', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['classes'].items()})"
  done
done > gpurun_out/st4_ab.log 2>&1
