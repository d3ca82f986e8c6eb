# B = 1 and B = 32 lines after a dispatch change (tuning tool)
set -e
timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/b1c.json 2>/dev/null
python -c "
import json; d=json.load(open('gpurun_out/b1c.json'))
print('B=1 fps', d['value'], {k:v['avg_launch_us'] for k,v in d['roofline']['classes'].items()})"
timeout -k 10 150 python bench.py --steps 50 --no-cpu-baseline --host-frames 0 > gpurun_out/b32c.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/b32c.json')); print('B=32 fps', d['value'])"
for b in 4 8 16; do
  timeout -k 10 150 python bench.py --batch $b --steps 100 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/bxc.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/bxc.json')); print('B=$b fps', d['value'])"
done
