# OSTrack-384 (720 tokens) under the round-2 dispatch choices (tuning tool)
set -o pipefail
for r in 1 2; do
  for v in "MMT_NONE=1" "MMT_PART_PRIO=0" "MMT_GM_LONGK=8" "MMT_SPLIT_T128=1000000" "MMT_SPLIT_CONV_OLD=1" "MMT_256S_MIN=1000000" "MMT_RING_COPY=1"; do
    env $v timeout -k 10 200 python bench.py --workload ostrack384 --steps 30 --warmup 5 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/ost.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ost.json'))
print('$v round $r ost fps', d['value'])"
  done
done > gpurun_out/ost_ab.log 2>&1
