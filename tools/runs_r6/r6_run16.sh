#!/bin/bash
# Round 6, run 16: the f16x3 eight-wave attention with a three-stage K / V ring (MMT_ATTN_NS=3: two tiles in flight,
# one workgroup per CU) against the two-stage ring (two workgroups per CU) -- parity under the new ring, 32 sequences,
# and the attention class time of the probe
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run16
mkdir -p $O
MMT_ATTN_NS=3 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -k attention tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for ns in 2 3; do
  MMT_ATTN_NS=$ns timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_ns$ns.json 2> $O/bench_ns$ns.err || { tail -5 $O/bench_ns$ns.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_ns$ns.json')); c=d['roofline']['classes']; print('ns$ns', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
done
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_ATTN_NS=3" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
