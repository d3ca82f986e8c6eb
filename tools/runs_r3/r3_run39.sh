#!/bin/bash
# Round-3 run 39: LDS-private depth histogram + parallel median search (f1) and the parallel NCHW correlation (A18):
# SURVEY §8 row tool
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run39${SUFFIX:-}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_frames.py tests/test_gpu_siamfc.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_rows.py --cpu-seconds 3 > $O/rows.jsonl 2> $O/rows.err || exit 1
python -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); print(d['row'], {k:v for k,v in d.items() if k not in ('cpu_baseline',)})"
