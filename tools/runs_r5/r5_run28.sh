#!/bin/bash
# Round 5, run 28: the head's conv1 on 128 x 192 tiles (MMT_CONV192: 256 tiles for the two 16-sequence halves together,
# one round, instead of 384): network goldens and the benchmarked launch with it, then A/B at 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run28
mkdir -p $O
MMT_CONV192=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_CONV192=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
for v in "" "MMT_CONV192=1"; do
  env $v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras > $O/p.json 2>$O/p.err || { tail -3 $O/p.err; exit 1; }
  python -c "import json; c=json.load(open('$O/p.json'))['roofline']['classes']['conv1']; print('[$v] conv1 probe us', c['avg_launch_us'], 'frac', c['frac_of_peak'])"
done
