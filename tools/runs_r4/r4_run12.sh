#!/bin/bash
# Round-4 run 12: one-sequence split-K rule sweep (env knobs, no rebuild): MMT_SPLITK_TILES (split below this many
# 64 x 64 tiles; 128) and MMT_SPLITK_TARGET (slices x tiles aimed at; 256), two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run12
mkdir -p $O
for r in 1 2; do
  for cfg in "128 256" "100 256" "64 256" "128 384" "128 192" "100 384"; do
    set -- $cfg
    MMT_SPLITK_TILES=$1 MMT_SPLITK_TARGET=$2 timeout -k 10 200 python bench.py --batch 1 --steps 300 --warmup 30 --no-cpu-baseline --probe none > $O/b1_$1_$2.json 2>$O/err.log || { tail -3 $O/err.log; exit 1; }
    echo "round $r tiles $1 target $2: $(python -c "import json; print(json.load(open('$O/b1_$1_$2.json'))['value'])")"
  done
done
