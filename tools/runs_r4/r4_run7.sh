#!/bin/bash
# Round-4 run 7: diagnose the DiMP golden failure of run 6 (fused stem pool vs separate; old conv kernel vs deep)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run7
mkdir -p $O
echo "== default"; timeout -k 10 200 python tools/diag/stempool_net.py 2>&1 | tail -4 || exit 1
echo "== MMT_CONV_OLD"; MMT_CONV_OLD=1 timeout -k 10 200 python tools/diag/stempool_net.py 2>&1 | tail -4 || exit 1
echo "== MMT_CONV_NOPATCH"; MMT_CONV_NOPATCH=1 timeout -k 10 200 python tools/diag/stempool_net.py 2>&1 | tail -4 || exit 1
