#!/bin/bash
# Round-4 run 8: generic conv A/B -- default, MMT_CONV_OVL (split woven into the MFMAs), and abx/libprio.so (the
# MFMA phase at raised wave priority, with and without OVL); per-shape times and the mfDiMP line, two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run8
mkdir -p $O
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprio.so
run_conv() {   # name, lib, ovl
  if [ "$3" = 1 ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  MMTRACK_LIB=$2 MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$1.jsonl 2>$O/err.log || exit 1
  echo "== generic conv $1: $(python -c "
import json
print(' '.join('%s %s' % (d['shape'], d['us']) for d in map(json.loads, open('$O/conv_$1.jsonl'))))")"
  unset MMT_CONV_OVL
}
run_dimp() {   # name, lib, ovl
  if [ "$3" = 1 ]; then export MMT_CONV_OVL=1; else unset MMT_CONV_OVL; fi
  MMTRACK_LIB=$2 timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$1.json 2>$O/err.log || exit 1
  echo "mfdimp $1: $(python -c "import json; d=json.load(open('$O/dimp_$1.json')); print(d['value'], d['roofline']['frac'])")"
  unset MMT_CONV_OVL
}
for r in 1 2; do
  run_conv base$r $L 0; run_conv ovl$r $L 1; run_conv prio$r $P 0; run_conv prioovl$r $P 1
done
for r in 1 2; do
  run_dimp base$r $L 0; run_dimp ovl$r $L 1; run_dimp prio$r $P 0; run_dimp prioovl$r $P 1
done
