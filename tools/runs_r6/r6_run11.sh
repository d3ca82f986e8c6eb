#!/bin/bash
# Round 6, run 11: the eight-phase kernel with fragment pre-reads (every phase's fragments read during the previous
# phase's MFMA section; loads by waves 0-3 only) -- op tests, benchmarked-launch goldens, and the 32-sequence line
# against the previous commit with 256-row tiles only in both arms (MMT_T320=0: the 320-row variant spills in this build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run11
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_T320=0 MMTRACK_LIB=$PWD/abx/libprev.so" "MMT_T320=0" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
for arm in prev new; do
  if [ $arm = prev ]; then export MMTRACK_LIB=$PWD/abx/libprev.so; else unset MMTRACK_LIB; fi
  MMT_T320=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$arm.json 2> $O/bench_$arm.err || { tail -5 $O/bench_$arm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$arm.json')); c=d['roofline']['classes']; print('$arm', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
done
