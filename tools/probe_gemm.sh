# usage: build probe/lib_<variant>.so from a copy of gemm.hip with -DPROBE_NOLOAD / -DPROBE_NOMFMA hooks, then
# GEMM probe: the persistent kernel with its K-tile loads removed (NOLOAD) or its MFMAs + LDS reads
# removed (NOMFMA), against the unmodified build (base).  Tuning tool, not a test.
for v in ${VARIANTS:-base NOLOAD NOMFMA}; do
  echo "== $v"
  MMTRACK_LIB=$PWD/probe/lib_$v.so NO_TORCH=1 SHAPES=${SHAPES:-qkv,fc1nog,fc1} CFGS=${CFGS:-10} \
    timeout -k 10 100 python tools/bench_gemm.py 2>&1 | grep TFLOP
done
