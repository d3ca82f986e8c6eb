#!/bin/bash
# Round-3 GPU run 2: token-kernel fusion (fovea statistics in the consumers, split-K reduces deferred into
# the row kernels): parity suite, bench lines at 32 and 1 sequences, kernel trace at one sequence.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run2
bash tests/gpu_steps.sh $O \
  "suite|900|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/" \
  "bench32|300|python bench.py --no-cpu-baseline" \
  "bench1|300|python bench.py --batch 1 --steps 300 --no-cpu-baseline" \
  "prof1|300|TAG=r3_run2/prof1 STEPS=200 ARGS='--batch 1' bash tests/prof_bench.sh"
