#!/bin/bash
# Round 5, run 39: qkv / fc1 whose 256 x 256 tiles spill a small tail into a second round of the chip (qkv of the
# 244-token layers, fc1 of the 190-token layers: 1.125 rounds with both halves) on the 128 x 128 kernel instead
# (MMT_256S_TAIL=percent), A/B at 32 sequences after the parity / benchpath tests with it on
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run39
mkdir -p $O
MMT_256S_TAIL=25 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split_launch" tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 timeout -k 10 700 bash tools/ab_envs.sh "" "MMT_256S_TAIL=25" "MMT_256S_TAIL=50" > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
