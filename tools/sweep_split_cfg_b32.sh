# forced f16x3 tile configs at B = 32 (tuning tool): whole-step fps + per-class launch time
set -e
for c in ${CFGS:--1 0 7 9 12 1 4 13 14}; do
  MMT_SPLIT_CFG=$c timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --host-frames 0 \
    > gpurun_out/sw32.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/sw32.json'))
print('cfg $c fps', d['value'], {k:(v['avg_launch_us'], round(v['frac_of_peak'],3)) for k,v in d['roofline']['classes'].items()})"
done
