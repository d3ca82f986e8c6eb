#!/bin/bash
# Round 6 (second session), run 1: the 128 x 256 two-group tile (gemm128w_kernel) for the N = 768 residual GEMMs --
# op tests vs fp64 and bit for bit against the 256 x 256 tile, the benchmarked-launch goldens, the probe classes of
# both arms (MMT_W256=0: the previous 128 x 128 / 128 x 192 choice) and one-box A/Bs of the 32-sequence line and
# OSTrack-384
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -s > $O/f16x3.txt 2>&1 || { grep -E "FAIL|Error|assert|f16x3 gemm 128x256" $O/f16x3.txt | head -30; tail -3 $O/f16x3.txt; exit 1; }
grep "128x256" $O/f16x3.txt; tail -1 $O/f16x3.txt
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_benchpath.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for arm in 0 1; do
  MMT_W256=$arm timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --no-extras > $O/probe_$arm.json 2> $O/probe_$arm.err || { tail -5 $O/probe_$arm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/probe_$arm.json')); c=d['roofline']['classes']; print('W256=$arm', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
done
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_W256=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_W256=0" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
