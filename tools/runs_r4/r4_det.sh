cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_det; mkdir -p $O
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so; P=$PWD/abx/libprev.so
for v in new1 new2 prev1 prev2; do
  lib=$L; case $v in prev*) lib=$P;; esac
  MMTRACK_LIB=$lib timeout -k 10 120 python tools/diag/dimp_corr_dump.py $O/$v.npz > $O/$v.txt 2>&1 || { tail -3 $O/$v.txt; exit 1; }
done
python -c "
import numpy as np
d = {v: np.load('$O/%s.npz' % v) for v in ('new1', 'new2', 'prev1', 'prev2')}
for x, y in (('new1', 'new2'), ('prev1', 'prev2'), ('prev1', 'new1')):
    a, b = d[x], d[y]
    print(x, y, {k: float(np.abs(a[k] - b[k]).max()) for k in a.files if not np.array_equal(a[k], b[k])})
"
