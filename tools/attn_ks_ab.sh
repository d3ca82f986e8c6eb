# key-split attention for few (sequence, head) pairs: tests, then one-sequence A/B (tuning tool)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "attention or splitk or split_launch" > gpurun_out/ks_t.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ks_p.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_ATTN_NOKS=1" "MMT_NONE=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/ks_b1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ks_b1.json'))
print('$v round $r B=1 fps', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['classes'].items()})"
  done
done > gpurun_out/ks_ab.log 2>&1
