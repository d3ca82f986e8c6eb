# 256 x 128 / 128 x 256 f16x3 tiles for the N % 256 == 0 GEMMs that take the 128 x 128 rule (tuning tool)
set -e
for r in 1 2; do
  for v in 0 1 2 3; do
    MMT_SPLIT_N768=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/n768.json 2>/dev/null
    python -c "
import json; d=json.load(open('gpurun_out/n768.json'))
print('n768 $v round $r fps', d['value'], {k:v['avg_launch_us'] for k,v in d['roofline']['classes'].items()})"
  done
done
