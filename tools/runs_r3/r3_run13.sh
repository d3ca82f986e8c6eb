#!/bin/bash
# Round-3 GPU run 13: one max-word atomic per conv workgroup
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run13
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dimpnet.py -k "conv2d or stem" \
  > $O/pytest_conv.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py \
  > $O/pytest_dimpnet.log 2>&1 &&
timeout -k 10 300 python bench.py --workload mfdimp_rgbt --batch 32 --no-cpu-baseline \
  > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --workload mfdimp_rgbt --batch 32 --steps 30 --warmup 3 --no-cpu-baseline --probe none \
  > $O/bench_prof.log 2>&1
cp $(find $O/prof -name '*kernel_trace.csv' | head -n 1) $O/kernel_trace.csv
gzip -f $O/kernel_trace.csv
rm -rf $O/prof
