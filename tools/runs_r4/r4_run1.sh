#!/bin/bash
# Round-4 run 1: the new parity tests (DiMP branch goldens, 32-slot pool launch, non-blocking launch,
# teacher-forced ViT tracker steps), then the whole GPU suite and the default bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_dimp_branches.py \
  "tests/test_gpu_parity.py::test_tracker_steps_match_reference" "tests/test_gpu_parity.py::test_tracker_sequence_matches_reference" \
  tests/test_gpu_parity.py::test_ostrack384_tracker_sequence_matches_reference > $O/new_tests.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/new_tests.txt | tail -60; exit 1; }
grep -E "PASS|FAIL|flags|IoU|teacher" $O/new_tests.txt | tail -60
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { tail -30 $O/gpu_suite.txt; exit 1; }
tail -3 $O/gpu_suite.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b32.json 2> $O/bench_b32.err || exit 1
python -c "import json; d=json.load(open('$O/bench_b32.json')); print(d['value'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/bench_dimp.json 2> $O/bench_dimp.err || exit 1
python -c "import json; d=json.load(open('$O/bench_dimp.json')); print(d['value'], d['roofline']['frac'])"
