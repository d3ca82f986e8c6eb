#!/bin/bash
# Round 5, run 1: the GPU suite after the ABI / test changes, smoke, and the default bench line with its extra
# workloads (one sequence, OSTrack-384, mfDiMP as child processes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head -20; tail -3 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
s=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench32.json 2> $O/bench32.err || { tail -5 $O/bench32.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
python -c "import json; d=json.load(open('$O/bench32.json')); print('vit32', d['value'], d['roofline']['frac'], d['cpu_baseline']['value']); print({k: (v.get('value'), v.get('frac'), v['seconds']) for k, v in d['extra_workloads'].items()})"
