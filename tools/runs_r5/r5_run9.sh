#!/bin/bash
# Round 5, run 9: previous-LN1 fovea statistics handed to the deep prompt kernel + split-K tile threshold 100:
# parity (ViPT / OSTrack trackers, prompt ops), the DiMP classifier-input dump for tools/diag/dimp_feed_ref.py,
# library A/B at one and 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run9
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_benchpath.py > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -3 $O/parity.txt
timeout -k 10 300 python -u tools/diag/dimp_init_dump.py > $O/dump.txt 2>&1 || { tail -20 $O/dump.txt; exit 1; }
cat $O/dump.txt
ROUNDS=3 ARGS="--batch 1" LIBDIR=abx5 timeout -k 10 400 bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=2 LIBDIR=abx5 timeout -k 10 400 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
