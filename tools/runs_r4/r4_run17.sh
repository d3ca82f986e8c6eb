#!/bin/bash
# Round-4 run 17: the strip-blocked DiMP transpose kernel (filter gradient) against the previous build
# (abx/libprev.so): DiMP tests, dump comparison (another summation order), the mfDiMP line, the steady-state trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run17
mkdir -p $O
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprev.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimp.py tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
MMTRACK_LIB=$P timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/prev.npz > $O/dp.txt 2>&1 || exit 1
MMTRACK_LIB=$L timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/new.npz > $O/dn.txt 2>&1 || exit 1
python -c "
import numpy as np
a, b = np.load('$O/prev.npz'), np.load('$O/new.npz')
print('dumps', {k: '%.2e' % float(np.abs(a[k] - b[k]).max() / (np.abs(a[k]).max() + 1e-30)) for k in a.files if not np.array_equal(a[k], b[k])} or 'bitwise equal')
"
for r in 1 2; do
  for v in prev new; do
    lib=$L; [ $v = prev ] && lib=$P
    MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp $v r$r: $(python -c "import json; print(json.load(open('$O/dimp_$v$r.json'))['value'])")"
  done
done
TAG=r4_run17/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/profdimp/steady.txt
grep -E "steps:|dimp_transpose|dimp_filter" $O/profdimp/steady.txt
