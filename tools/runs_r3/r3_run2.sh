#!/bin/bash
# Round-3 GPU run 2: token-kernel fusion (fovea statistics in the consumers, split-K reduces deferred into
# the row kernels) and the f16x3 DiMP convolutions: new DiMP tests, the GPU suite, bench lines.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run2
bash tools/gpu_steps.sh $O \
  "dimp|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py" \
  "suite|900|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ --deselect tests/test_gpu_dimpnet.py" \
  "bench32|300|python bench.py --no-cpu-baseline" \
  "bench1|300|python bench.py --batch 1 --steps 300 --no-cpu-baseline" \
  "dimp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline" \
  "dimp32fp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline --dimp-precision fp32" \
  "prof1|300|TAG=r3_run2/prof1 STEPS=200 ARGS='--batch 1' bash tools/prof_bench.sh"
