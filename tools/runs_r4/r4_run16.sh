#!/bin/bash
# Round-4 run 16: split-K reduce kernels (DiMP conv_splitk_reduce_kernel, ViT splitk_reduce_kernel) with every slab
# and epilogue operand requested before use, against the previous build (abx/libprev.so): parity tests, one-sequence
# ViT, mfDiMP and ViT 32-sequence lines, two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_run16
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_benchpath.py tests/test_gpu_f16x3.py tests/test_gpu_dimpnet.py > $O/tests.txt 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
L=$PWD/multi-modal-trakcing-bechmark_amd/mmtrack_amd/libmmtrack.so
P=$PWD/abx/libprev.so
for r in 1 2; do
  for v in prev new; do
    lib=$L; [ $v = prev ] && lib=$P
    MMTRACK_LIB=$lib timeout -k 10 200 python bench.py --batch 1 --steps 300 --warmup 30 --no-cpu-baseline --probe none > $O/b1_$v$r.json 2>$O/err.log || exit 1
    MMTRACK_LIB=$lib timeout -k 10 300 python bench.py --workload mfdimp_rgbt --no-cpu-baseline > $O/dimp_$v$r.json 2>$O/err.log || exit 1
    echo "$v r$r: b1 $(python -c "import json; print(json.load(open('$O/b1_$v$r.json'))['value'])") mfdimp $(python -c "import json; print(json.load(open('$O/dimp_$v$r.json'))['value'])")"
  done
done
