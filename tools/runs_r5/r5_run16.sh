#!/bin/bash
# Round 5, run 16: LayerNorm / deferred-reduce arithmetic spelled out (identical rounding in every kernel), fused CE +
# LN2 back on: the fused-vs-unfused diagnostic, the GPU suite, one-sequence env A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run16
mkdir -p $O
MMT_CE_FUSED=0 timeout -k 10 300 python tools/diag/ce_fused_diag.py $O/unfused.npz > $O/a.txt 2>&1 || { tail -5 $O/a.txt; exit 1; }
MMT_CE_FUSED=2 timeout -k 10 300 python tools/diag/ce_fused_diag.py $O/fused.npz > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r5_run16/unfused.npz"); b = np.load("gpurun_out/r5_run16/fused.npz")
print("fused == unfused on every key:", all(np.array_equal(a[k], b[k]) for k in a.files),
      [k for k in a.files if not np.array_equal(a[k], b[k])][:6])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1 || { grep -E "FAIL|Error" $O/gpu_suite.txt | head; tail -3 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
ROUNDS=3 STEPS=300 ARGS="--batch 1" timeout -k 10 500 bash tools/ab_envs.sh "" "MMT_CE_FUSED=0" > $O/ab_b1.txt 2>&1 || { tail -5 $O/ab_b1.txt; exit 1; }
cat $O/ab_b1.txt
