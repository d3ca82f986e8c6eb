#!/bin/bash
# Round 5, run 30: 128 x 192 tiles for the wide GEMMs (qkv, fc1) where 256 x 256 tiles take two rounds (MMT_T192W =
# the assumed efficiency penalty in percent): forced-on correctness (parity / benchpath with MMT_T192W=1000), A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run30
mkdir -p $O
MMT_T192W=1000 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 timeout -k 10 800 bash tools/ab_envs.sh "" "MMT_T192W=150" "MMT_T192W=250" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
for v in "X=0" "MMT_T192W=150" "MMT_T192W=250"; do
  env $v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras > $O/p.json 2>$O/p.err || { tail -3 $O/p.err; exit 1; }
  python -c "import json; c=json.load(open('$O/p.json'))['roofline']['classes']; print('[$v]', {k: (c[k]['avg_launch_us'], c[k]['frac_of_peak']) for k in ('qkv','fc1')})"
done
