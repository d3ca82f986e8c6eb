#!/bin/bash
# Round 6 (second session), run 6: the 128 x 256 tile by the one-round rule -- bitwise against the previous commit's
# build at 32 and 1 sequences (tools/lib_bitwise.py), op tests, benchmarked-launch goldens and parity tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run6
mkdir -p $O
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 32 12 > $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 1 30 >> $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
grep bitwise $O/bitwise.txt
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_f16x3.py > $O/f16x3.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/f16x3.txt | head -30; tail -3 $O/f16x3.txt; exit 1; }
tail -1 $O/f16x3.txt
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_benchpath.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
