#!/bin/bash
# Round 6 (second session), run 10: 128 x 256 tile micro-variants -- load issue after the fragment reads
# (abx/libw256late.so), no MFMA priority (abx/libw256noprio.so) -- stamps of the proj / fc2 halves and the line A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run10
mkdir -p $O
export SHAPES=proj_half,fc2_half,fc2_full,proj_full
for v in base w256late w256noprio; do
  echo "## $v"
  if [ $v = base ]; then L=""; else L="MMTRACK_LIB=$PWD/abx/lib$v.so"; fi
  env $L MMT_FORCE=128 timeout -k 10 120 python tools/gemm_stamps_f16x3.py 2>&1 | grep shape || exit 1
done
ROUNDS=3 STEPS=100 timeout -k 10 900 bash tools/ab_envs.sh "" "MMTRACK_LIB=$PWD/abx/libw256late.so" "MMTRACK_LIB=$PWD/abx/libw256noprio.so" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
