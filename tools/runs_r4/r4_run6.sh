#!/bin/bash
# Round-4 run 6: generic conv with the next K-tile's split woven between the MFMAs (MMT_CONV_OVL) against the default:
# bitwise test, per-shape kernel times, phase stamps, the mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run6
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in base ovl base ovl; do
  if [ $v = ovl ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v.jsonl 2>$O/err.log || exit 1
  echo "== generic conv $v"; python -c "
import json
for l in open('$O/conv_$v.jsonl'): d=json.loads(l); print(d['shape'], d['us'], d['frac_f16x3'])"
done
unset MMT_CONV_OVL
for v in base ovl; do
  if [ $v = ovl ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v.json 2>$O/err.log || exit 1
  echo "mfdimp $v: $(python -c "import json; d=json.load(open('$O/dimp_$v.json')); print(d['value'], d['roofline']['frac'])")"
done
MMT_CONV_OVL=1 MMTRACK_LIB=$PWD/abx/libstamps.so MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/stamps.jsonl 2> $O/stamps.err || { tail -3 $O/stamps.err; exit 0; }
grep "conv stamps" $O/stamps.err | sort | uniq -c | sort -rn | head -12
