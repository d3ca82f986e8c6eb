#!/bin/bash
# Round 6, run 5: the stem-pool patch stored by column parity (bank conflicts) -- the DiMP net tests, an mfDiMP A/B
# against the previous commit's build, and the LDS / MFMA counters of the mfDiMP step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_run5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ROUNDS=3 STEPS=60 ARGS="--workload mfdimp_rgbt" timeout -k 10 600 bash tools/ab_envs.sh "MMTRACK_LIB=$PWD/abx/libprev.so" "" > $O/ab_dimp.txt 2>&1 || { tail -5 $O/ab_dimp.txt; exit 1; }
cat $O/ab_dimp.txt
OUT=$O/pmc ARGS="--workload mfdimp_rgbt --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --no-extras" timeout -k 10 400 bash tools/pmc_mfma.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_mfma_summary.py $O/pmc > $O/pmc_summary.txt 2>&1; rm -rf $O/pmc/p1 $O/pmc/p2
grep -E "stem_pool|l2norm_scale|deep_kernel|patch_f16x3" $O/pmc_summary.txt | cut -c1-250
