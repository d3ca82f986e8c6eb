#!/bin/bash
# Round 5, run 11: GELU epilogue with the two Horner chains interleaved (gelu_erf4) and the DiMP conv3 + downsample
# fused into one GEMM: GEMM / DiMP tests, fc1 phase stamps, library A/B (GELU) at 32 and one sequence, env A/B of the
# downsample fusion on the mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run11
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f16x3.py tests/test_gpu_kernels.py tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py tests/test_gpu_dimp_stages.py -s > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
grep -E "max confidence rel|relative confidence differences" $O/tests.txt | cut -c1-260
SHAPES=fc1_half,qkv_half MMTRACK_LIB=$PWD/abx/libphase.so timeout -k 10 120 python tools/gemm256s_phases.py > $O/phases.jsonl 2>&1 || { tail -5 $O/phases.jsonl; exit 1; }
cut -c1-400 $O/phases.jsonl
ROUNDS=3 LIBDIR=abx7 timeout -k 10 400 bash tools/ab_bench.sh > $O/ab_b32.txt 2>&1 || { tail -5 $O/ab_b32.txt; exit 1; }
cat $O/ab_b32.txt
ROUNDS=2 ARGS="--batch 1" LIBDIR=abx7 timeout -k 10 300 bash tools/ab_bench.sh > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
ROUNDS=3 ARGS="--workload mfdimp_rgbt" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_DIMP_DSFUSE=0" "MMT_DIMP_FUSED_SAMPLE=0" > $O/ab_dsfuse.txt 2>&1 || { tail -5 $O/ab_dsfuse.txt; exit 1; }
cat $O/ab_dsfuse.txt
