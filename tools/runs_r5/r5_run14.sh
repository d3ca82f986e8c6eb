#!/bin/bash
# Round 5, run 14: isolate the bf16 batch-vs-single mismatch (fused CE+LN2 / fused crop geometry), then the suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run14
mkdir -p $O
T="tests/test_gpu_parity.py::test_batch_equals_single"
for v in "X=0" "MMT_CE_FUSED=0" "MMT_GEOM_KERNEL=1" "MMT_CE_FUSED=0 MMT_GEOM_KERNEL=1"; do
  env $v timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "$T" > $O/iso.txt 2>&1
  rc=$?
  echo "[$v] rc=$rc $(tail -1 $O/iso.txt)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # a timeout / abort / fault: nothing more on the GPU
done
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.txt 2>&1
rc=$?
tail -5 $O/gpu_suite.txt
exit $rc
