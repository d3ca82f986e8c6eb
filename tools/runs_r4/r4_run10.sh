#!/bin/bash
# Round-4 run 10: the deep conv's XCD-aware tile order only for wide outputs / short launches (hybrid rule) against
# the previous build (abx/libprev.so: M tiles fastest everywhere); DiMP tests, per-shape conv times, mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprev.so
for r in 1 2; do
  for v in prev hybrid; do
    lib=$L; [ $v = prev ] && lib=$P
    MMTRACK_LIB=$lib MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v$r.jsonl 2>$O/err.log || exit 1
    echo "== generic conv $v$r: $(python -c "
import json
print(' '.join('%s %s' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$v$r.jsonl'))))")"
    MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp $v$r: $(python -c "import json; d=json.load(open('$O/dimp_$v$r.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'])")"
  done
done
