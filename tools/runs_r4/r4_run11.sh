#!/bin/bash
# Round-4 run 11c: the strip DiMP filter kernel with two chunks in flight against the strip kernel with one (abx/libprev.so)
# correlation dump comparison (bitwise expected), DiMP tests, mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run11
mkdir -p $O
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprev.so
MMTRACK_LIB=$P timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/prev.npz > $O/dump_prev.txt 2>&1 || { tail -5 $O/dump_prev.txt; exit 1; }
MMTRACK_LIB=$L timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/new.npz > $O/dump_new.txt 2>&1 || { tail -5 $O/dump_new.txt; exit 1; }
python -c "
import numpy as np
a, b = np.load('$O/prev.npz'), np.load('$O/new.npz')
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print('correlation dumps:', len(a.files), 'arrays,', 'bitwise equal' if not bad else 'differ (max rel %.2e)' % max(float(np.abs(a[k] - b[k]).max() / (np.abs(a[k]).max() + 1e-30)) for k in bad))
"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimp.py tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in prev new; do
    lib=$L; [ $v = prev ] && lib=$P
    MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp $v$r: $(python -c "import json; d=json.load(open('$O/dimp_$v$r.json')); print(d['value'], d['roofline']['frac'])")"
  done
done
TAG=r4_run11/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/profdimp/steady.txt
grep -E "steps:|dimp_filter|dimp_transpose" $O/profdimp/steady.txt
