# threshold (128 x 128 f16x3 tiles from this many tiles) sweep at 32 sequences, alternating, 2 rounds (tuning tool)
set -e
for r in 1 2; do
  for t in 200 96 128 64; do
    MMT_SPLIT_T128=$t timeout -k 10 150 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/t128.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/t128.json')); print('t128 $t round $r fps', d['value'])"
  done
done
