#!/bin/bash
# Round 5, run 22: attention with the key mask only in the tail tile (compile-time flag): attention tests and the
# parity goldens on the in-tree library, then base vs peeled library on one box (32 sequences; attention class time
# from the probe)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run22
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for lib in abx/liba_base.so abx/libb_peel.so; do
    MMTRACK_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); c=d['roofline']['classes']; print('$lib round $r fps', d['value'], 'attn us', c['attn']['avg_launch_us'], 'frac', c['attn']['frac_of_peak'])"
  done
done
ROUNDS=2 STEPS=300 ARGS="--batch 1" LIBDIR=abx timeout -k 10 400 bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
