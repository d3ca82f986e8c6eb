#!/bin/bash
# Round 5, run 29: 128 x 192 f16x3 tiles where they take fewer rounds counting the concurrent stream part (conv1,
# fc2 / proj after candidate elimination; MMT_T192=0 switches the rule off): the GPU suite's ViT / f16x3 tests,
# A/B at 32 sequences and OSTrack-384, probe class times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run29
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_benchpath.py tests/test_gpu_f16x3.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_T192=0" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_T192=0" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
for v in "X=0" "MMT_T192=0"; do
  env $v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras > $O/p.json 2>$O/p.err || { tail -3 $O/p.err; exit 1; }
  python -c "import json; c=json.load(open('$O/p.json'))['roofline']['classes']; print('[$v]', {k: (c[k]['avg_launch_us'], c[k]['frac_of_peak']) for k in c})"
done
