#!/bin/bash
# Round-3 GPU run 1: the new parity tests first, then the whole GPU suite, the default and one-sequence bench
# lines and a rocprofv3 kernel trace of the default line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh $O \
  "new|900|$PYT tests/test_gpu_benchpath.py tests/test_gpu_f16x3.py tests/test_gpu_parity.py::test_ostrack384_tracker_sequence_matches_reference tests/test_gpu_siamfc.py::test_c1_benchmark_dispatch_100_frames" \
  "suite|1000|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ --deselect tests/test_gpu_benchpath.py --deselect tests/test_gpu_f16x3.py" \
  "bench32|300|python bench.py" \
  "bench1|300|python bench.py --batch 1 --steps 300 --no-cpu-baseline" \
  "prof32|300|TAG=r3_run1/prof32 STEPS=50 bash tools/prof_bench.sh"
