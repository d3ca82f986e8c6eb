#!/bin/bash
# Round 5, run 4: weight prefetch A/B at one sequence (off / on with 16, 32, 64 prefetch blocks), the DiMP stage
# comparison with per-frame state, gemm256s phase stamps, the one-sequence GEMM study's Infinity-Cache mode
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_dimp_stages.py > $O/dimp_stages.txt 2>&1
grep -E "^\[f16x3\] (filter after (7|8|10)|frame [1-6] (confidence|sample|state|patch))" $O/dimp_stages.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 600 bash tools/ab_envs.sh "" "MMT_PREFETCH=1" "MMT_PREFETCH=1 MMT_PREFETCH_BLOCKS=64" "MMT_PREFETCH=1 MMT_PREFETCH_BLOCKS=16" > $O/ab_prefetch_b1.txt 2>&1 || { tail -5 $O/ab_prefetch_b1.txt; cat gpurun_out/abenv.err | tail -5; exit 1; }
cat $O/ab_prefetch_b1.txt
MMTRACK_LIB=$PWD/abv/libphase.so timeout -k 10 200 python tools/gemm256s_phases.py > $O/gemm256s_phases.jsonl 2> $O/gemm256s_phases.err || { tail -3 $O/gemm256s_phases.err; exit 1; }
cat $O/gemm256s_phases.jsonl
SHAPES=qkv,fc1,fc2,proj timeout -k 10 200 python tools/b1_gemm_study.py > $O/b1_gemm_mall.jsonl 2> $O/b1_gemm_mall.err || { tail -3 $O/b1_gemm_mall.err; exit 1; }
grep -E '"mall"|_single' $O/b1_gemm_mall.jsonl
