#!/bin/bash
# Round 6, run 13: fc2 on the eight-phase 256 x 256 kernel, unsplit (MMT_FC2_256S=1: 120 tiles at 32 sequences, the
# other stream half fills the rest of the chip) against the 128 x 128 / 128 x 192 kernel -- 32 sequences, OSTrack-384,
# and the probe classes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run13
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -k "residual or t320" > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_FC2_256S=1" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_FC2_256S=1" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
MMT_FC2_256S=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_new.json 2> $O/bench_new.err || { tail -5 $O/bench_new.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_new.json')); c=d['roofline']['classes']; print('new', d['value'], {k: (v['avg_launch_us'], v['frac_of_peak']) for k, v in c.items()})"
