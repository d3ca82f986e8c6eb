#!/bin/bash
# Round-3 run 40: two rows per wave in the deep prompt / LN1 kernels from 8 sequences up (the block's weight fill
# and fovea statistics shared by 16 rows): golden / bench-path parity, then a one-box A/B (arm B = MMT_TOK_R=1,
# the previous one row per wave)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run40
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_benchpath.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ENV_B="MMT_TOK_R=1" bash tools/ab_env.sh 2>&1 | tee $O/ab.txt
