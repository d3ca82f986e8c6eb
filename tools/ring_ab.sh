# ring hand-off (no copy launches per step) vs hipMemcpyAsync of params / results (MMT_RING_COPY=1):
# GPU tests, then one-box A/B at one and 32 sequences (tuning tool)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_workspace.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ring_t.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_RING_COPY=1" "MMT_NONE=1"; do
    env $v timeout -k 10 120 python bench.py --batch 1 --steps 300 --warmup 20 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/ring_b1.json 2>/dev/null || exit 1
    env $v timeout -k 10 150 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --host-frames 0 --probe none > gpurun_out/ring_b32.json 2>/dev/null || exit 1
    python -c "
import json; a=json.load(open('gpurun_out/ring_b1.json')); b=json.load(open('gpurun_out/ring_b32.json'))
print('$v round $r B=1 fps', a['value'], 'B=32 fps', b['value'])"
  done
done > gpurun_out/ring_ab.log 2>&1
