#!/bin/bash
# Round-4 run 5: attention softmax trimmed (qk scale folded into the exponent, CE export without per-key bounds,
# tail mask inside its branch): attention / parity / benchpath tests, then one-box A/B old vs new library
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f16x3.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py tests/test_gpu_benchpath.py tests/test_gpu_dimpnet.py::test_conv_kernels_bitwise > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in old new; do
    MMTRACK_LIB=$PWD/abx/lib$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/vit_$v.json 2>$O/err.log || exit 1
    echo "vit32 $v round $r: $(python -c "import json; d=json.load(open('$O/vit_$v.json')); print(d['value'], d['roofline']['frac'], {c: v['avg_launch_us'] for c, v in d['roofline']['classes'].items()})")"
  done
done
for v in old new; do
  MMTRACK_LIB=$PWD/abx/lib$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --steps 200 --warmup 20 --probe none > $O/b1_$v.json 2>$O/err.log || exit 1
  echo "b1 $v: $(python -c "import json; print(json.load(open('$O/b1_$v.json'))['value'])")"
done
# 256-pixel generic conv tiles (MMT_CONV_BM=256) against 128: per-shape kernel times and the mfDiMP line
for bm in 128 256; do
  MMT_CONV_BM=$bm MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/conv_bm$bm.jsonl 2>$O/err.log || exit 1
  echo "== generic conv BM $bm"; python -c "
import json
for l in open('$O/conv_bm$bm.jsonl'): d=json.loads(l); print(d['shape'], d['us'], d['frac_f16x3'])"
done
for bm in 128 256; do
  MMT_CONV_BM=$bm timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_bm$bm.json 2>$O/err.log || exit 1
  echo "mfdimp BM $bm: $(python -c "import json; d=json.load(open('$O/dimp_bm$bm.json')); print(d['value'], d['roofline']['frac'])")"
done
# phase stamps of the deep generic conv (tuning build abx/libstamps.so; all shapes through the generic kernel)
MMTRACK_LIB=$PWD/abx/libstamps.so MMT_CONV_NOPATCH=1 timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/stamps.jsonl 2> $O/stamps.err || { tail -3 $O/stamps.err; exit 0; }
grep "conv stamps" $O/stamps.err | sort | uniq -c | head -20
