#!/bin/bash
# Round 6 (second session), run 8: the 3 x 3 patch conv's weight ring 4 stages deep for the 64-wide tiles (three taps
# ahead instead of one) -- bitwise against the previous build on the mfDiMP tracker, the DiMP tests, A/B of the
# mfDiMP line (arm 1 previous build, arm 2 this build, arm 3 + the 128-wide tiles at 3 stages, abx/libnst128.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run8
mkdir -p $O
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 32 6 mfdimp_rgbt > $O/bitwise.txt 2>&1; tail -2 $O/bitwise.txt
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so abx/libnst128.so 32 6 mfdimp_rgbt >> $O/bitwise.txt 2>&1; tail -1 $O/bitwise.txt
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py tests/test_gpu_dimp_stages.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=30 ARGS="--workload mfdimp_rgbt" timeout -k 10 900 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" "MMTRACK_LIB=$PWD/abx/libnst128.so" > $O/ab_dimp.txt 2>&1 || { tail -5 $O/ab_dimp.txt; exit 1; }
cat $O/ab_dimp.txt
