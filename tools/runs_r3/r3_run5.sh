#!/bin/bash
# Round-3 GPU run 5: grouped / split-K f16x3 convs, two-pass InstanceL2Norm, unrolled 4x4 filter
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py \
  > $O/pytest_dimpnet.log 2>&1 &&
timeout -k 10 200 python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --warmup 3 --no-cpu-baseline --sync \
  > $O/bench_sync.json 2> $O/bench_sync.err &&
timeout -k 10 200 python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --warmup 3 --no-cpu-baseline \
  > $O/bench_pipe.json 2> $O/bench_pipe.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --workload mfdimp_rgbt --batch 32 --steps 10 --warmup 2 --no-cpu-baseline --sync --probe none \
  > $O/bench_prof.log 2>&1
cp $(find $O/prof -name '*kernel_trace.csv' | head -n 1) $O/kernel_trace.csv
gzip -f $O/kernel_trace.csv
rm -rf $O/prof
