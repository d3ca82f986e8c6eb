#!/bin/bash
# Round 5, run 25: a static s_setprio 1 for the second half of the 8-wave attention workgroup (ATTN_PRIO), base vs
# variant library on one box at 32 sequences (line and the probe's attention class time)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run25
mkdir -p $O
for r in 1 2 3; do
  for lib in abx/liba_base.so abx/libb_prio.so; do
    MMTRACK_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); c=d['roofline']['classes']; print('$lib round $r fps', d['value'], 'attn us', c['attn']['avg_launch_us'], 'frac', c['attn']['frac_of_peak'])"
  done
done
