#!/bin/bash
# Round-3 GPU run 26 (evidence on the current build): GPU suite, smoke, PMC traffic of the probe's launch shapes,
# the bench lines (ViT 32 / 1 sequences, OSTrack-384, mfDiMP 32) and rocprofv3 kernel summaries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run26
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
OUT=$O/pmc bash tools/pmc_bench.sh || exit 1
python tools/pmc_traffic.py $O/pmc $O/r03_pmc_traffic_fp32_b32_final.json > $O/pmc_traffic.txt 2>&1 || exit 1
cp $O/r03_pmc_traffic_fp32_b32_final.json profiles/r03_pmc_traffic_fp32_b32.json
timeout -k 10 300 python bench.py > $O/bench_b32.json 2> $O/bench_b32.err || exit 1
timeout -k 10 300 python bench.py --batch 1 --steps 200 --warmup 20 > $O/bench_b1.json 2> $O/bench_b1.err || exit 1
timeout -k 10 300 python bench.py --workload ostrack384 > $O/bench_ost.json 2> $O/bench_ost.err || exit 1
timeout -k 10 300 python bench.py --workload mfdimp_rgbt --batch 32 --no-cpu-baseline > $O/bench_dimp.json 2> $O/bench_dimp.err || exit 1
TAG=r3_run26/prof32 STEPS=40 bash tools/prof_bench.sh || exit 1
TAG=r3_run26/prof1 STEPS=200 ARGS="--batch 1" bash tools/prof_bench.sh || exit 1
for f in $O/bench_*.json; do echo "$f: $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline'].get('kernel'), d['roofline'].get('frac'))")"; done
