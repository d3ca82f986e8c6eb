#!/bin/bash
# Round 5, run 17: the DiMP deep conv's LDS-staged epilogue (full-line residual loads / output stores) and the conv
# epilogue arithmetic spelled out: DiMP tests on the variant library, then the mfDiMP line A/B (MMT_CONV_STAGED=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run17
mkdir -p $O
export MMTRACK_LIB=$PWD/abx/libstaged.so MMT_CONV_STAGED=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py tests/test_gpu_dimp.py -s > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 ARGS="--workload mfdimp_rgbt" timeout -k 10 500 bash tools/ab_envs.sh "MMT_CONV_STAGED=1" "MMT_CONV_STAGED=0" > $O/ab_staged.txt 2>&1 || { tail -5 $O/ab_staged.txt; exit 1; }
cat $O/ab_staged.txt
