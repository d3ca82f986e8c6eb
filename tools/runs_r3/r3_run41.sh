#!/bin/bash
# Round-3 run 41: four rows per wave in the deep prompt / LN1 kernels (MMT_TOK_R=4): bench-path parity with it, then
# a one-box A/B against the default two (arm B = MMT_TOK_R=4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run41
mkdir -p $O
MMT_TOK_R=4 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_benchpath.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ENV_B="MMT_TOK_R=4" bash tools/ab_env.sh 2>&1 | tee $O/ab.txt
