# deep LDS rings for the 64 x 64 f16x3 tiles at B = 1 (tuning tool; forced config applies to every split GEMM)
set -e
for c in -1 17 16 18 19; do
  MMT_SPLIT_CFG=$c timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/rb1.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/rb1.json'))
print('cfg $c fps', d['value'], {k:v['avg_launch_us'] for k,v in d['roofline']['classes'].items()})"
done
