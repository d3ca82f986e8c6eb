#!/bin/bash
# Round 5, run 8: the one-sequence frame on the current build -- rocprofv3 steady-state kernel trace (launch count
# and per-kernel time), env A/B of qkv without split-K in the CE-pruned layers (MMT_SPLITK_TILES=100)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run8
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof1 -o run -- \
  python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extras --probe none --host-frames 0 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
python tools/trace_steps.py $(find $O/prof1 -name '*kernel_trace.csv' | head -1) geometry_kernel 30 60 > $O/b1_steady.txt
head -45 $O/b1_steady.txt
rm -rf $O/prof1
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 400 bash tools/ab_envs.sh "" "MMT_SPLITK_TILES=100" > $O/ab_splitk_tiles_b1.txt 2>&1 || { tail -5 $O/ab_splitk_tiles_b1.txt; exit 1; }
cat $O/ab_splitk_tiles_b1.txt
# gemm256s with the next half-tile's DMA issued inside the MFMA cluster (GEMM256S_DMA_IN_MFMA=1) vs default, B=32
ROUNDS=3 LIBDIR=abx4 timeout -k 10 500 bash tools/ab_bench.sh > $O/ab_dmamfma_b32.txt 2>&1 || { tail -5 $O/ab_dmamfma_b32.txt; exit 1; }
cat $O/ab_dmamfma_b32.txt
