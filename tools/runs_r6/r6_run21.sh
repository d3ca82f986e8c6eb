#!/bin/bash
# Round 6, run 21: phase stamps of the one-sequence row kernels (ROW_STAMPS build, tools/b1_row_stamps.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run21
mkdir -p $O
MMTRACK_LIB=$PWD/abx/librowst.so timeout -k 10 300 python tools/b1_row_stamps.py 40 > $O/row_stamps.jsonl 2> $O/row_stamps.err || { tail -5 $O/row_stamps.err; exit 1; }
cat $O/row_stamps.jsonl
