#!/bin/bash
# Round 5, run 24: the second stream half started after the first half's k-th GEMM (MMT_HALF_LAG=k: the halves out of
# phase, so one half's GEMMs meet the other's row kernels / attention) -- the split-launch tests with a lag, then A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run24
mkdir -p $O
MMT_HALF_LAG=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split_launch" tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 timeout -k 10 900 bash tools/ab_envs.sh "" "MMT_HALF_LAG=1" "MMT_HALF_LAG=2" "MMT_HALF_LAG=3" "MMT_HALF_LAG=5" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
