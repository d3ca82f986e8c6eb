#!/bin/bash
# Round-3 run 43: PMC HBM traffic of the probe's launch shapes on the final build (FETCH_SIZE / WRITE_SIZE in
# separate rocprofv3 passes), then the bench line that reads it
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run43
mkdir -p $O
OUT=$O/pmc bash tools/pmc_bench.sh || exit 1
python tools/pmc_traffic.py $O/pmc $O/r03_pmc_traffic_fp32_b32_final.json > $O/pmc_traffic.txt 2>&1 || exit 1
cat $O/pmc_traffic.txt
cp $O/r03_pmc_traffic_fp32_b32_final.json profiles/r03_pmc_traffic_fp32_b32.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b32.json 2> $O/bench_b32.err || exit 1
python -c "import json; d=json.load(open('$O/bench_b32.json')); r=d['roofline']; print(d['value'], r['frac'], r['traffic'], r['traffic_source'])"
