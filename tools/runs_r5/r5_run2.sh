#!/bin/bash
# Round 5, run 2: DiMP stage localisation (dimp_stages.npz) and the one-sequence GEMM study (cold / warm weights,
# per-block stamps) for the heuristic tile and the pinned 64 x 64 variants
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_run2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_dimp_stages.py > $O/dimp_stages.txt 2>&1
echo "stages rc=$?"; grep -E "^\[(f16x3|fp32)\]" $O/dimp_stages.txt | head -80
for cfg in -1 16 17 19; do
  if [ "$cfg" = "-1" ]; then
    timeout -k 10 120 python tools/b1_gemm_study.py >> $O/b1_gemm.jsonl 2>> $O/b1_gemm.err || exit 1
  else
    MMT_SPLIT_CFG=$cfg timeout -k 10 120 python tools/b1_gemm_study.py >> $O/b1_gemm.jsonl 2>> $O/b1_gemm.err || exit 1
  fi
done
cat $O/b1_gemm.jsonl
