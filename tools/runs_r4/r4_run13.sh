#!/bin/bash
# Round-4 run 13: the generic conv with the activations DMA'd into an NS-stage ring (MMT_CONV_DMA=3/4/5) against
# the default deep kernel: bitwise test, per-shape conv times, the mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run13
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py -k "bitwise or golden" > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert|Mismatch" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in 0 3 4 5; do
    MMT_CONV_DMA=$v MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v$r.jsonl 2>$O/err.log || { tail -3 $O/err.log; exit 1; }
    echo "== generic conv dma=$v r$r: $(python -c "
import json
print(' '.join('%s %s' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$v$r.jsonl'))))")"
  done
done
for r in 1 2; do
  for v in 0 4 5; do
    MMT_CONV_DMA=$v timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "mfdimp dma=$v r$r: $(python -c "import json; d=json.load(open('$O/dimp_$v$r.json')); print(d['value'], d['roofline']['frac'])")"
  done
done
