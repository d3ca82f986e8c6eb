# bf16 statistics of several library builds on one box (tuning tool): LIBS="a b" N=48 bash tools/bisect_libs.sh
for lib in ${LIBS:-lib_b_new lib_c_dpp}; do
  echo "== $lib"
  MMT_STAT_N=${N:-12} MMTRACK_LIB=$PWD/abl/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k "bf16_statistics" --timeout 280 --timeout-method thread 2>&1 | grep -E "argmax agreement|passed|failed"
done
