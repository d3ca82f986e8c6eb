#!/bin/bash
# Round 6, run 15: the residual GEMMs (fc2, proj) on the eight-phase kernel where its tiles fill 3/4 of a round (the
# default rule) -- op tests, the OSTrack-384 goldens, and OSTrack-384 / the 32-sequence line against never (MMT_RESID_256S=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run15
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_parity.py -k "residual or ostrack or t320 or vs_fp64" > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_RESID_256S=0" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
ROUNDS=2 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMT_RESID_256S=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
