#!/bin/bash
# Round-4 run 4: -fno-slp-vectorize A/B (packed fp32 VALU beside MFMAs), then MFMA / LDS / wait counters per kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run4
mkdir -p $O
for r in 1 2; do
  for v in base noslp; do
    MMTRACK_LIB=$PWD/abx/lib$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --probe none > $O/vit_$v.json 2>$O/err.log || exit 1
    echo "vit32 $v round $r: $(python -c "import json; print(json.load(open('$O/vit_$v.json'))['value'])")"
  done
done
for v in base noslp; do
  MMTRACK_LIB=$PWD/abx/lib$v.so timeout -k 10 200 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v.json 2>$O/err.log || exit 1
  echo "mfdimp $v: $(python -c "import json; print(json.load(open('$O/dimp_$v.json'))['value'])")"
done
OUT=$O/pmc bash tools/pmc_mfma.sh && python tools/pmc_mfma_summary.py $O/pmc > $O/pmc_summary.txt 2>&1; head -30 $O/pmc_summary.txt
