#!/bin/bash
# Round 6, run 9: 192-row tiles of the eight-phase kernel (the tile-height rule over 192 / 256 / 320) -- op tests,
# benchmarked-launch goldens, A/Bs of the 32-sequence line and OSTrack-384 against the previous commit, the probe
# classes, and the halves-off per-layer trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run9
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
for arm in prev new; do
  if [ $arm = prev ]; then export MMTRACK_LIB=$PWD/abx/libprev.so; else unset MMTRACK_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$arm.json 2> $O/bench_$arm.err || { tail -5 $O/bench_$arm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$arm.json')); c=d['roofline']['classes']; print('$arm', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
done
unset MMTRACK_LIB
MMT_OVERLAP_MIN=1000 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python3 bench.py --steps 20 --warmup 0 --no-cpu-baseline --no-extras --probe none > $O/trace_bench.log 2>&1 || { tail -5 $O/trace_bench.log; exit 1; }
TR=$(find $O/tr -name '*kernel_trace.csv' | head -n 1)
python tools/trace_layers.py $TR 'crop_kernel<true>' 5 gemm256s > $O/layers.txt
rm -rf $O/tr
cat $O/layers.txt | tail -6
