# super-tile height sweep for long-K GEMMs at B = 32 (tuning tool)
set -e
for g in 8 1 2 4; do
  MMT_GM_LONGK=$g timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --host-frames 0 > gpurun_out/gm.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/gm.json'))
print('gm_longk $g fps', d['value'], {k:(v['avg_launch_us'], round(v['frac_of_peak'],3)) for k,v in d['roofline']['classes'].items()})"
done
CFGS="0 7 9 12 13" bash tools/sweep_split_cfg_b32.sh
