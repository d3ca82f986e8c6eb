#!/bin/bash
# Round 6, run 8: the deep prompt kernel's split-K slabs requested with the row (one sequence) -- parity tests, an A/B
# of the one-sequence line against the previous commit; OSTrack-384 with the 320 x 256 rule taking ties (MMT_T320=3)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=4 STEPS=400 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_T320=3" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
