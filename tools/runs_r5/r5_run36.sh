#!/bin/bash
# Round 5, run 36: five-wave key-split attention for 257..320 keys (one key tile per wave; the CE logits kept in
# registers and stored into the free V slots after the loop): attention / parity tests, base vs variant at one
# sequence with the attention kernels' times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run36
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" LIBDIR=abx timeout -k 10 500 bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
for lib in a_base b_ks5; do
  MMTRACK_LIB=$PWD/abx/lib$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extras --probe none --host-frames 0 > $O/prof_$lib.log 2>&1 || { tail -5 $O/prof_$lib.log; exit 1; }
  echo "$lib:"; grep -h attn_kernel $(find $O/prof_$lib -name '*kernel_stats.csv') | cut -d, -f1-6
  rm -rf $O/prof_$lib
done
