# A/B of the f16x3 dispatch rule on one box (tuning tool): new default vs MMT_SPLIT_OLD=1 MMT_GM_LONGK=8, 3 rounds
set -e
for r in 1 2 3; do
  for arm in new old; do
    if [ $arm = old ]; then export MMT_SPLIT_OLD=1 MMT_GM_LONGK=8; else unset MMT_SPLIT_OLD; unset MMT_GM_LONGK; fi
    timeout -k 10 150 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/ab.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$arm round $r fps', d['value'])"
  done
done
unset MMT_SPLIT_OLD MMT_GM_LONGK
timeout -k 10 150 python bench.py --batch 1 --steps 200 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/ab1.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/ab1.json')); print('new B=1 fps', d['value'])"
