#!/bin/bash
# Round-4 run 14: the strip DiMP filter kernel on 16-channel chunks (MMT_DIMP_STRIP_CC=16: 108 VGPRs, four
# workgroups per CU) against 32-channel chunks (166 VGPRs, three): bitwise dump comparison, mfDiMP line, traces
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run14
mkdir -p $O
MMT_DIMP_STRIP_CC=32 timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/cc32.npz > $O/d32.txt 2>&1 || { tail -3 $O/d32.txt; exit 1; }
MMT_DIMP_STRIP_CC=16 timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/cc16.npz > $O/d16.txt 2>&1 || { tail -3 $O/d16.txt; exit 1; }
python -c "
import numpy as np
a, b = np.load('$O/cc32.npz'), np.load('$O/cc16.npz')
print('dumps', {k: float(np.abs(a[k] - b[k]).max()) for k in a.files if not np.array_equal(a[k], b[k])} or 'bitwise equal')
"
for r in 1 2; do
  for v in 32 16; do
    MMT_DIMP_STRIP_CC=$v timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp cc=$v r$r: $(python -c "import json; d=json.load(open('$O/dimp_$v$r.json')); print(d['value'])")"
  done
done
for v in 32 16; do
  MMT_DIMP_STRIP_CC=$v TAG=r4_run14/prof$v STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
  python tools/trace_steps.py $(find $O/prof$v -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/prof$v/steady.txt
  echo "cc=$v"; grep -E "steps:|dimp_filter" $O/prof$v/steady.txt
done
