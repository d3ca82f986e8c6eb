# HIP stream priorities for the stream parts (tuning tool)
set -o pipefail
for r in 1 2 3; do
  for v in "MMT_PART_PRIO=0" "MMT_PART_PRIO=1" "MMT_PART_PRIO=2"; do
    env $v timeout -k 10 150 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/prio.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/prio.json'))
print('$v round $r B=32 fps', d['value'])"
  done
done > gpurun_out/prio_ab.log 2>&1
