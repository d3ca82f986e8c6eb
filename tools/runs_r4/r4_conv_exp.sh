#!/bin/bash
# conv_f16x3_kernel bottleneck experiment: the same conv shapes with the A split removed (hi only), the A stash
# removed, two of the three MFMAs removed, and both (wrong-result builds, timing only)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_conv_exp
mkdir -p $O
for v in base hionly nostash onemfma floor base; do
  MMTRACK_LIB=$PWD/abx/lib$v.so timeout -k 10 120 python tools/bench_conv_f16x3.py > $O/$v.jsonl 2>$O/$v.err || { cat $O/$v.err | tail -5; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('$O/$v.jsonl'): d=json.loads(l); print(d['shape'], d['us'], d['frac_f16x3'])"
done
