# proj split-K combine fused with LN2 (one sequence): tests, then A/B (tuning tool)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "splitk" > gpurun_out/lf_t.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lf_p.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_NO_LNFUSE=1" "MMT_NONE=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --host-frames 0 > gpurun_out/lf_b1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/lf_b1.json'))
print('$v round $r B=1 fps', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['classes'].items()})"
  done
done > gpurun_out/lf_ab.log 2>&1
