#!/bin/bash
# Round-4 run 18: the 3 x 3 patch conv tiled over the flattened batch (no partial tile at each image's end: 18 x 18
# maps 96 -> 81 tiles per 32 images) against per-image tiles (MMT_CONV_PATCH_PERIMG=1): DiMP tests, conv shapes,
# the mfDiMP line, the steady-state trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run18
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in perimg batch; do
    if [ $v = perimg ]; then export MMT_CONV_PATCH_PERIMG=1; else unset MMT_CONV_PATCH_PERIMG; fi
    timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v$r.jsonl 2>$O/err.log || { tail -3 $O/err.log; exit 1; }
    timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "$v r$r: mfdimp $(python -c "import json; print(json.load(open('$O/dimp_$v$r.json'))['value'])") conv $(python -c "
import json
print(' '.join('%s %s' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$v$r.jsonl'))))")"
  done
done
unset MMT_CONV_PATCH_PERIMG
TAG=r4_run18/profdimp STEPS=20 ARGS="--workload mfdimp_rgbt --batch 32" bash tools/prof_bench.sh || exit 1
python tools/trace_steps.py $(find $O/profdimp -name '*kernel_trace.csv' | head -1) dimp_sample_kernel 5 40 > $O/profdimp/steady.txt
grep -E "steps:|patch" $O/profdimp/steady.txt
