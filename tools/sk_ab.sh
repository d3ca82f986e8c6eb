# In-launch split-K combine: bitwise / parity tests, then B=1 A/B against the separate reduce launch and with
# split-K widened to more GEMMs (tuning tool; one box, interleaved rounds)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "splitk or gemm_dense or conv3x3" > gpurun_out/sk_t.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sk_p.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_SK_NONE=1" "MMT_SK_INLAUNCH=2" "MMT_SK_INLAUNCH=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/sk_b1.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/sk_b1.json')); print('$v round $r B=1 fps', d['value'])"
  done
done > gpurun_out/sk_ab.log 2>&1
