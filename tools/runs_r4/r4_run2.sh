#!/bin/bash
# Round-4 run 2: the 3x3 patch conv (DiMP) and the geometry kernel resetting the token indices: conv / DiMP / ViT
# parity tests, then conv timings patch vs generic, the conv bottleneck experiment, and the two bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py \
   tests/test_gpu_parity.py tests/test_gpu_benchpath.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in patch nopatch; do
  if [ $v = nopatch ]; then export MMT_CONV_NOPATCH=1; else unset MMT_CONV_NOPATCH; fi
  timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_$v.jsonl 2>$O/conv_$v.err || { tail -5 $O/conv_$v.err; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/conv_$v.jsonl'): d=json.loads(l); print(d['shape'], d['us'], d['frac_f16x3'])"
done
unset MMT_CONV_NOPATCH
for v in base hionly nostash onemfma floor; do
  MMTRACK_LIB=$PWD/abx/lib$v.so MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/exp_$v.jsonl 2>$O/exp_$v.err || { tail -5 $O/exp_$v.err; exit 1; }
  echo "== exp $v"; python -c "
import json
print(' '.join('%s %.1f' % (d['shape'], d['us']) for d in map(json.loads, open('$O/exp_$v.jsonl'))))"
done
for v in patch nopatch patch nopatch; do
  if [ $v = nopatch ]; then export MMT_CONV_NOPATCH=1; else unset MMT_CONV_NOPATCH; fi
  timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v.json 2> $O/dimp_$v.err || exit 1
  python -c "import json; d=json.load(open('$O/dimp_$v.json')); print('mfdimp $v', d['value'], d['roofline']['frac'])"
done
unset MMT_CONV_NOPATCH
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/vit32.json 2> $O/vit32.err || exit 1
python -c "import json; d=json.load(open('$O/vit32.json')); print('vit32', d['value'], d['roofline']['frac'])"
# FETCH_SIZE calibration on known byte counts (512 MB per kernel launch, 2 launches each)
mkdir -p $O/calib
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib/fetch -- ./tools/micro/fetch_calib > $O/calib/fetch.log 2>&1 || { echo "calib failed"; exit 0; }
python - <<PY
import csv, glob
for f in glob.glob('$O/calib/fetch/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Kernel_Name'][:30], r['Counter_Name'], float(r['Counter_Value']) * 1024 / (512 << 20), 'x of the bytes read')
PY
timeout -s KILL 60 rocprofv3 --list-avail > $O/calib/avail.txt 2>&1 || true
grep -i "TCC_EA0_RDREQ\|TCC_BUBBLE\|TCC_EA0_RD" $O/calib/avail.txt | head -20
