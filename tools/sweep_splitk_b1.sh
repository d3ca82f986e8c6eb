# split-K tuning at B = 1 (parity mode): MMT_SPLITK_{TILES,TARGET,MINKT,MAX} per run (tuning tool)
set -e
for spec in "128 256 4 8" "512 512 3 8" "512 768 2 12" "512 1024 2 16" "512 512 2 8"; do
  set -- $spec
  MMT_SPLITK_TILES=$1 MMT_SPLITK_TARGET=$2 MMT_SPLITK_MINKT=$3 MMT_SPLITK_MAX=$4 timeout -k 10 120 \
    python bench.py --batch 1 --steps 200 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/sk.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/sk.json'))
print('splitk $spec fps', d['value'], {k:v['avg_launch_us'] for k,v in d['roofline']['classes'].items()})"
done
