#!/bin/bash
# Round-4 run 19: DiMP conv split-K with the batch-tiled patch kernel: default (256 / 512 slots), no split
# (MMT_CONV_NOSPLIT), 384 / 768-slot targets (MMT_CONV_SLOTS), two rounds of the mfDiMP line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run19
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dimpnet.py tests/test_gpu_dimp_branches.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in default nosplit s384 s768; do
    unset MMT_CONV_NOSPLIT MMT_CONV_SLOTS
    case $v in nosplit) export MMT_CONV_NOSPLIT=1;; s384) export MMT_CONV_SLOTS=384;; s768) export MMT_CONV_SLOTS=768;; esac
    timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "$v r$r: $(python -c "import json; print(json.load(open('$O/dimp_$v$r.json'))['value'])")"
  done
done
