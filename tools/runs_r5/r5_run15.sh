#!/bin/bash
# Round 5, run 15: the fused CE + LN2 kernel against ce_select + ln_kernel on one sequence (bf16 / f16x3 engines)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run15
mkdir -p $O
MMT_CE_FUSED=0 timeout -k 10 300 python tools/diag/ce_fused_diag.py $O/unfused.npz > $O/a.txt 2>&1 || { tail -5 $O/a.txt; exit 1; }
MMT_CE_FUSED=2 timeout -k 10 300 python tools/diag/ce_fused_diag.py $O/fused.npz > $O/b.txt 2>&1 || { tail -5 $O/b.txt; exit 1; }
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r5_run15/unfused.npz"); b = np.load("gpurun_out/r5_run15/fused.npz")
for k in a.files:
    x, y = a[k], b[k]
    d = np.abs(x.astype(np.float64) - y.astype(np.float64))
    print(f"{k:24s} equal={np.array_equal(x, y)} maxdiff={d.max():.3e} n_diff={(d > 0).sum()}")
PY
