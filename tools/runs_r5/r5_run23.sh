#!/bin/bash
# Round 5, run 23: the DiMP branch sequences asserted past near-ties the device decides as the reference did
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run23
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dimp_branches.py -k "branches_match or coverage" > $O/branches.txt 2>&1; rc=$?
grep -E "asserted|PASS|FAIL|Error" $O/branches.txt | head -60
exit $rc
