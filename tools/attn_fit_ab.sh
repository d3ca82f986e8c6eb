# f16x3 attention query blocks fitted to the sequence length (8 / 10 / 12 waves) vs 8 waves only
# (MMT_ATTN_FIT=0): tests, batched parity study, then one-box A/B at 32 sequences (tuning tool)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fit_t.log 2>&1 &&
timeout -k 10 300 python -u tools/precision_study.py --n 512 --batch 32 --net deep_rgbt --seed0 51000 --modes fp32 --forced none > gpurun_out/fit_study.txt 2>&1 || exit 1
for r in 1 2 3; do
  for v in "MMT_ATTN_FIT=0" "MMT_NONE=1"; do
    env $v timeout -k 10 150 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --host-frames 0 > gpurun_out/fit_b32.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/fit_b32.json'))
print('$v round $r B=32 fps', d['value'], 'attn us', d['roofline']['classes']['attn']['avg_launch_us'])"
  done
done > gpurun_out/fit_ab.log 2>&1
