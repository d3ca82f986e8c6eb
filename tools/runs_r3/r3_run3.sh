#!/bin/bash
# Round-3 GPU run 3: the device-side DiMP tracker + f16x3 convs (DiMP tests, mfDiMP bench lines), the fused
# token kernels at 32 / 1 sequences, and an f16x3 GEMM tile sweep.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run3
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "dimp|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp.py" \
  "dimp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline" \
  "dimp32fp32|300|python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --no-cpu-baseline --dimp-precision fp32" \
  "bench32|300|python bench.py --no-cpu-baseline" \
  "bench1|300|python bench.py --batch 1 --steps 300 --no-cpu-baseline" \
  "sweep|600|bash tools/runs_r3/r3_gemmsweep.sh"
