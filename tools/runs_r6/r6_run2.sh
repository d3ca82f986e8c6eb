#!/bin/bash
# Round 6, run 2: the 320 x 256 f16x3 tile -- op tests vs fp64 + bitwise vs 256 x 256, the benchmarked-launch goldens,
# then an A/B of the round rule (MMT_T320=0 = round 5's tiles) on the 32-sequence line and the per-layer trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|error" $O/tests.txt | head -20; tail -5 $O/tests.txt; exit 1; }
grep -E "320x256|passed|failed" $O/tests.txt | tail -12
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_T320=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
MMT_OVERLAP_MIN=1000 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- \
  python3 bench.py --steps 20 --warmup 0 --no-cpu-baseline --no-extras --probe none > $O/trace_bench.log 2>&1 || { tail -5 $O/trace_bench.log; exit 1; }
TR=$(find $O/tr -name '*kernel_trace.csv' | head -n 1)
python tools/trace_layers.py $TR 'crop_kernel<true>' 5 gemm256s > $O/layers.txt
rm -rf $O/tr
cat $O/layers.txt
