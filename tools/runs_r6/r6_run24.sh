#!/bin/bash
# Round 6, run 24: (a) LN / final norm with one row per workgroup at one sequence alone (the build), (b) the deep prompt
# and LN1 weight fills walked from a per-block offset (abx/librot.so, -DWFILL_ROT: blocks of a launch no longer
# request the same lines in the same order) -- bitwise vs the previous build, stamps, one-sequence A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run24
mkdir -p $O
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so abx/librot.so 1 30 > $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
timeout -k 10 300 python tools/lib_bitwise.py abx/libprev.so multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so 1 30 >> $O/bitwise.txt 2>&1 || { tail -5 $O/bitwise.txt; exit 1; }
grep bitwise $O/bitwise.txt
MMTRACK_LIB=$PWD/abx/librowst.so timeout -k 10 300 python tools/b1_row_stamps.py 40 > $O/row_stamps.jsonl 2> $O/row_stamps.err || { tail -5 $O/row_stamps.err; exit 1; }
MMTRACK_LIB=$PWD/abx/librowstrot.so timeout -k 10 300 python tools/b1_row_stamps.py 40 > $O/row_stamps_rot.jsonl 2> $O/row_stamps.err || { tail -5 $O/row_stamps.err; exit 1; }
cat $O/row_stamps.jsonl $O/row_stamps_rot.jsonl
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 900 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" "MMTRACK_LIB=$PWD/abx/librot.so" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
