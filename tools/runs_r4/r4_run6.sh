#!/bin/bash
# Round-4 run 6: generic conv -- wave-uniform (tap, chunk) counters instead of divisions (new vs abx/libhead.so), and
# the next K-tile's split woven between the MFMAs (MMT_CONV_OVL): bitwise test, per-shape kernel times, phase stamps,
# the mfDiMP line; the stem with its max-pool fused (MMT_DIMP_STEMPOOL=0: separate)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run6
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run_conv() {   # name, lib, ovl
  if [ "$3" = 1 ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  MMTRACK_LIB=$2 MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$1.jsonl 2>$O/err.log || exit 1
  echo "== generic conv $1: $(python -c "
import json
print(' '.join('%s %s' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$1.jsonl'))))")"
  unset MMT_CONV_OVL
}
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
for r in 1 2; do
  run_conv head$r $PWD/abx/libhead.so 0
  run_conv new$r $L 0
  run_conv ovl$r $L 1
done
for v in head nopool new ovl; do
  if [ $v = ovl ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  if [ $v = head ] || [ $v = nopool ]; then export MMT_DIMP_STEMPOOL=0; else unset MMT_DIMP_STEMPOOL; fi
  lib=$L; [ $v = head ] && lib=$PWD/abx/libhead.so
  MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v.json 2>$O/err.log || exit 1
  echo "mfdimp $v: $(python -c "import json; d=json.load(open('$O/dimp_$v.json')); print(d['value'], d['roofline']['frac'])")"
done
unset MMT_DIMP_STEMPOOL
unset MMT_CONV_OVL
for v in 0 1; do
  if [ $v = 1 ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  MMTRACK_LIB=$PWD/abx/libstamps.so MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/stamps$v.jsonl 2> $O/stamps$v.err || { tail -3 $O/stamps$v.err; exit 0; }
  echo "stamps ovl=$v"; grep "conv stamps" $O/stamps$v.err | sort | uniq -c | sort -rn | head -8
done
