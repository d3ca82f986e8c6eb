set -e
for c in -1 0 2 8 10 11; do
  echo "== cfg $c"
  MMT_SPLIT_CFG=$c timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/sw_b1_$c.json 2>/dev/null
  python - <<PY
import json; d=json.load(open("gpurun_out/sw_b1_$c.json"))
print("cfg $c fps", d["value"], {k:(v["avg_launch_us"], v["ms_per_step"]) for k,v in d["roofline"]["classes"].items()})
PY
done
