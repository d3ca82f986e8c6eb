#!/bin/bash
# Round-4 run 3: the deep-pipelined generic conv (asm activation loads, weights two K-tiles ahead): bitwise vs the
# two-deep kernel, the DiMP tests, conv timings per variant, and the mfDiMP line A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in old deep2 deep3 patch; do
  unset MMT_CONV_OLD MMT_CONV_NR MMT_CONV_NOPATCH
  case $v in old) export MMT_CONV_OLD=1 MMT_CONV_NOPATCH=1;; deep2) export MMT_CONV_NR=2 MMT_CONV_NOPATCH=1;; deep3) export MMT_CONV_NOPATCH=1;; esac
  timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v.jsonl 2>$O/conv_$v.err || { tail -5 $O/conv_$v.err; exit 1; }
  echo "== $v: $(python -c "
import json
print(' '.join('%s %.1f' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$v.jsonl'))))")"
done
unset MMT_CONV_OLD MMT_CONV_NR MMT_CONV_NOPATCH
for v in new old new old; do
  if [ $v = old ]; then export MMT_CONV_OLD=1 MMT_CONV_NOPATCH=1; else unset MMT_CONV_OLD MMT_CONV_NOPATCH; fi
  timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v.json 2> $O/dimp_$v.err || exit 1
  python -c "import json; d=json.load(open('$O/dimp_$v.json')); print('mfdimp $v', d['value'], d['roofline']['frac'], d['roofline']['frac_of_layer_roofline'])"
done
