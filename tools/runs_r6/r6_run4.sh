#!/bin/bash
# Round 6, run 4: the GPU suite on this build (320 x 256 tiles, pruned paths, crop params race fix, near-tie rule,
# fp32 conv with four accumulator sets), then the fp32 DiMP tests on a build with one accumulator set (round 5's)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head -20; tail -3 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
MMTRACK_LIB=$PWD/abx/libnacc1.so timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dimpnet.py::test_conv2d_fp32_per_layer_vs_fp64 tests/test_gpu_dimp_stages.py "tests/test_gpu_dimp_branches.py" -k "fp32 or per_layer or stages" > $O/nacc1.txt 2>&1
tail -2 $O/nacc1.txt
# the 256 x 256 / 320 x 256 kernel's wave priorities: per-phase flips (default) / static priority 1 for waves 4-7 / none
ROUNDS=3 STEPS=100 timeout -k 10 600 bash tools/ab_envs.sh "" "MMTRACK_LIB=$PWD/abx/libprio1.so" "MMTRACK_LIB=$PWD/abx/libprio2.so" > $O/ab_prio.txt 2>&1 || { tail -5 $O/ab_prio.txt; exit 1; }
cat $O/ab_prio.txt
