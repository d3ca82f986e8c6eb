#!/bin/bash
# Round 6 (second session), run 4: the 128 x 256 tile (no read drain before the barriers) with and without the two
# stream halves at 32 sequences -- A/B/C/D of the line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -k "w256 or vs_fp64" > $O/f16x3.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/f16x3.txt | head -30; tail -3 $O/f16x3.txt; exit 1; }
tail -1 $O/f16x3.txt
ROUNDS=2 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "MMT_W256=0" "" "MMT_OVERLAP_MIN=64 MMT_W256=0" "MMT_OVERLAP_MIN=64" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
