#!/bin/bash
# Round 6 (second session), run 9: the 128 x 256 two-group tile for the 16-bit-output qkv / fc1 launches the eight-phase
# kernel leaves (153-token layers) -- op tests, bitwise against the build before the 128 x 256 tile, A/B (arm 1
# MMT_W256_BF16=0) of the 32-sequence line and OSTrack-384
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py -s > $O/f16x3.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/f16x3.txt | head -30; tail -3 $O/f16x3.txt; exit 1; }
grep "128x256" $O/f16x3.txt | tail -2; tail -1 $O/f16x3.txt
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 32 12 > $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
grep bitwise $O/bitwise.txt
ROUNDS=3 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "MMT_W256_BF16=0" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 STEPS=20 ARGS="--workload ostrack384" timeout -k 10 600 bash tools/ab_envs.sh "MMT_W256_BF16=0" "" > $O/ab_ost.txt 2>&1 || { tail -5 $O/ab_ost.txt; exit 1; }
cat $O/ab_ost.txt
