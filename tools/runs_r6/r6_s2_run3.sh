#!/bin/bash
# Round 6 (second session), run 3: per-block stamps (prologue / K loop / epilogue cycles) of fc2 / proj shapes on the
# 128 x 128 / 128 x 192 tiles, the 128 x 256 two-group tile (with and without the read drain before each barrier,
# abx/libw256nolgkm.so) and the 256 x 256 eight-phase tile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run3
mkdir -p $O
export SHAPES=fc2_full,proj_full,fc2_half,proj_half,fc2_244
echo "## default tiles (MMT_W256=0)"; MMT_W256=0 timeout -k 10 120 python tools/gemm_stamps_f16x3.py || exit 1
echo "## 128 x 256"; MMT_FORCE=128 timeout -k 10 120 python tools/gemm_stamps_f16x3.py || exit 1
echo "## 128 x 256 without the read drain"; MMTRACK_LIB=$PWD/abx/libw256nolgkm.so MMT_FORCE=128 timeout -k 10 120 python tools/gemm_stamps_f16x3.py || exit 1
echo "## 256 x 256"; MMT_FORCE=256 timeout -k 10 120 python tools/gemm_stamps_f16x3.py || exit 1
