#!/bin/bash
# Round-3 GPU run 3: the device-side DiMP tracker + f16x3 convs (DiMP tests, mfDiMP bench lines), then a same-box
# A/B of the ViT token-kernel fusion (abx/lib_a_base.so = before, lib_b_fused.so = after).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run3
mkdir -p $O
bash tests/gpu_steps.sh $O \
  "dimp|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py" \
  "dimp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline" \
  "dimp32fp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline --dimp-precision fp32" \
  "ab32|400|LIBDIR=abx ROUNDS=2 STEPS=60 bash tests/ab_bench.sh" \
  "ab1|400|LIBDIR=abx ROUNDS=2 STEPS=300 ARGS='--batch 1' bash tests/ab_bench.sh"
cp gpurun_out/ab.log $O/ab.log 2>/dev/null || true
