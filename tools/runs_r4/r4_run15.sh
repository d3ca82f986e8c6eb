#!/bin/bash
# Round-4 run 15: the conv epilogue operands (bias, residual) requested together before use (deep and patch kernels,
# previous build (abx/libprev.so): DiMP net / bitwise tests, the mfDiMP line, the steady-state trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run15
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprev.so
for r in 1 2; do
  for v in prev new; do
    lib=$L; [ $v = prev ] && lib=$P
    MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp $v$r: $(python -c "import json; d=json.load(open('$O/dimp_$v$r.json')); print(d['value'])")"
  done
done
TAG=r4_run15/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/profdimp/steady.txt
head -12 $O/profdimp/steady.txt
