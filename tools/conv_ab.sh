# DiMP stem conv: one tap per load with weights padded to 4 channels (MMT_CONV_W4) vs the per-element path (MMT_CONV_NOW4=1): tests, then mfDiMP A/B (tuning tool)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_dimpnet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/conv_t.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_CONV_NOW4=1" "MMT_NONE=1"; do
    env $v timeout -k 10 200 python bench.py --workload mfdimp_rgbt --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/conv_b.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/conv_b.json'))
print('$v round $r mfdimp fps', d['value'], 'feature', d['roofline']['achieved'], d['roofline']['frac'])"
  done
done > gpurun_out/conv_ab.log 2>&1
