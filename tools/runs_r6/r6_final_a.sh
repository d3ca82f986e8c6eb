#!/bin/bash
# Round-6 final measurements, part A: the GPU suite, smoke, and the bench lines (default ViT 32 sequences with its CPU
# baseline, one sequence, OSTrack-384, mfDiMP with its CPU baseline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${FINAL_TAG:-r6_final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head -20; tail -3 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
T0=$SECONDS
timeout -k 10 400 python bench.py > $O/bench32.json 2> $O/bench32.err || { tail -5 $O/bench32.err; exit 1; }
echo "default bench.py invocation: $((SECONDS - T0)) s wall" | tee $O/bench32_wall.txt
python -c "import json; d=json.load(open('$O/bench32.json')); print('vit32', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --batch 1 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || exit 1
python -c "import json; d=json.load(open('$O/bench1.json')); print('vit1', d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload ostrack384 --no-cpu-baseline > $O/bench_ostrack384.json 2> $O/bench_ost.err || exit 1
python -c "import json; d=json.load(open('$O/bench_ostrack384.json')); print('ostrack384', d['value'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py --workload mfdimp_rgbt > $O/bench_mfdimp32.json 2> $O/bench_dimp.err || exit 1
python -c "import json; d=json.load(open('$O/bench_mfdimp32.json')); print('mfdimp', d['value'], d['roofline']['frac'], d['roofline']['frac_of_layer_roofline'], d['cpu_baseline'])"
