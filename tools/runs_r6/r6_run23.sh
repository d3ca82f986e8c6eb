#!/bin/bash
# Round 6, run 23: few-row launches of the one-sequence row kernels -- LN (and the final norm) one row per workgroup, the deep
# prompt with its fc2 slabs two slots per workgroup (128 threads) -- so each CU takes in fewer rows and slabs:
# bitwise against the previous build (tools/lib_bitwise.py, 32 and 1 sequences), parity tests, the row-kernel stamps
# of the new build, one sequence and 32 sequences A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run23
mkdir -p $O
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 32 12 > $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 1 30 >> $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
grep bitwise $O/bitwise.txt
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
MMTRACK_LIB=$PWD/abx/librowst.so timeout -k 10 300 python tools/b1_row_stamps.py 40 > $O/row_stamps.jsonl 2> $O/row_stamps.err || { tail -5 $O/row_stamps.err; exit 1; }
cat $O/row_stamps.jsonl
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=2 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
