# threshold (256 x 256 8-phase f16x3 kernel from this many tiles) sweep at 32 sequences, 2 rounds (tuning tool)
set -e
for r in 1 2; do
  for t in 128 96 64 48; do
    MMT_256S_MIN=$t timeout -k 10 150 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/t256.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/t256.json')); print('t256 $t round $r fps', d['value'])"
  done
done
