#!/bin/bash
# Round 6 (second session), run 7: the 128 x 256 tile's residual chunks requested at kernel entry (W256_RPRE=1, the
# build) against after the K loop (abx/librpre0.so) -- op tests, stamps of the proj / fc2 halves, A/B of the line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run7
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -k "w256 or vs_fp64" > $O/f16x3.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/f16x3.txt | head -30; tail -3 $O/f16x3.txt; exit 1; }
tail -1 $O/f16x3.txt
export SHAPES=proj_half,fc2_half
echo "## rpre 0"; MMTRACK_LIB=$PWD/abx/librpre0.so MMT_FORCE=128 timeout -k 10 120 python tools/gemm_stamps_f16x3.py 2>&1 | grep shape || exit 1
echo "## rpre 1"; MMT_FORCE=128 timeout -k 10 120 python tools/gemm_stamps_f16x3.py 2>&1 | grep shape || exit 1
ROUNDS=3 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/librpre0.so" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
