#!/bin/bash
# Round-3 GPU run 3: same-box A/B of the token-kernel fusion (abx/lib_a_base.so = before, lib_b_fused.so = after),
# the f16x3 DiMP conv (K loop unrolled) tests and bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run3
mkdir -p $O
bash tests/gpu_steps.sh $O \
  "dimp|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py" \
  "dimp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline" \
  "ab32|400|LIBDIR=abx ROUNDS=2 STEPS=60 bash tests/ab_bench.sh" \
  "ab1|400|LIBDIR=abx ROUNDS=2 STEPS=300 ARGS='--batch 1' bash tests/ab_bench.sh"
cp gpurun_out/ab.log $O/ab.log 2>/dev/null || true
