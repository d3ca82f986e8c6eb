#!/bin/bash
# Round-3 run 42 (final build of the round): GPU suite, smoke, bench lines, one-sequence kernel summary
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run42
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_b32.json 2> $O/bench_b32.err || exit 1
timeout -k 10 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_b1.json 2> $O/bench_b1.err || exit 1
TAG=r3_run42/prof1 STEPS=200 ARGS="--batch 1" bash tools/prof_bench.sh || exit 1
for f in $O/bench_*.json; do echo "$f: $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline'].get('kernel'), d['roofline'].get('frac'))")"; done
