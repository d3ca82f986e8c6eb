#!/bin/bash
# Round-4 run 20: no DiMP split-K at 32 images (256-slot rule): DiMP tests, the mfDiMP line (two rounds), the steady
# trace (launches per step)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run20
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py tests/test_gpu_dimp.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp$r.json 2>$O/err.log || exit 1
  echo "mfdimp r$r: $(python -c "import json; print(json.load(open('$O/dimp$r.json'))['value'])")"
done
TAG=r4_run20/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/profdimp/steady.txt
head -8 $O/profdimp/steady.txt
