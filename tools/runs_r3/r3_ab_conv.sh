#!/bin/bash
# A/B of mfDiMP conv tuning knobs on one box (alternating, 2 rounds): usage bash tools/runs_r3/r3_ab_conv.sh "ENV=1" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_ab_conv
mkdir -p $O
: > $O/ab.txt
for round in 1 2; do
  for v in "MMT_NONE=1" "$@"; do
    env $v timeout -k 10 200 python bench.py --workload mfdimp_rgbt --batch 32 --steps 30 --warmup 5 --no-cpu-baseline \
      --probe none > $O/line.json 2> $O/err.txt || { echo "$v failed"; tail -5 $O/err.txt; exit 1; }
    python -c "import json; d=json.load(open('$O/line.json')); print('$v round $round fps', d['value'], 'feat_ms', d['roofline']['avg_batch_ms'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
