#!/bin/bash
# Round 6, run 6: attention waves past N skip their compute -- attention op tests vs fp64, the benchmarked-launch
# goldens, an A/B of the 32-sequence line against the previous commit, and the probe's attention class (bench line)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run6
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py tests/test_gpu_kernels.py -k "attention or attn or benchpath" > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
for arm in prev new; do
  if [ $arm = prev ]; then export MMTRACK_LIB=$PWD/abx/libprev.so; else unset MMTRACK_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$arm.json 2> $O/bench_$arm.err || { tail -5 $O/bench_$arm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$arm.json')); c=d['roofline']['classes']; print('$arm', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
done
