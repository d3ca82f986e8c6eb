#!/bin/bash
# Round-3 GPU run 16: epilogue operands requested together (f16x3 GEMMs, gemm256s, DiMP convs): GPU suite, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run16
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_b32.json 2> $O/bench_b32.err &&
timeout -k 10 300 python bench.py --batch 1 --steps 200 --warmup 20 > $O/bench_b1.json 2> $O/bench_b1.err &&
timeout -k 10 300 python bench.py --workload mfdimp_rgbt --batch 32 --no-cpu-baseline > $O/bench_dimp.json 2> $O/bench_dimp.err
