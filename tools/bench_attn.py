"""Attention kernel timing on the path's shapes (GPU tuning tool, not a test): B=32, 12 heads,
N = the ViPT joint lengths per CE stage (and OSTrack-384's 720)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
B = int(os.environ.get("B", "32"))
s = torch.cuda.current_stream().cuda_stream
for N in [int(n) for n in os.environ.get("NS", "320,244,190,153,720").split(",")]:
    qkv = (torch.randn(B, N, 3 * 768, device="cuda") * 2.0).bfloat16()
    out = torch.empty(B, N, 768, device="cuda", dtype=torch.bfloat16)
    prob = torch.empty(B, 12, N - 64, device="cuda")  # (OSTrack-384: N = 720)
    run = lambda: lib.mmt_op_attention(qkv.data_ptr(), out.data_ptr(), B, N, 12, 27, 64, prob.data_ptr(), s)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"attn B={B} N={N}: {us:7.1f} us  {4 * B * 12 * N * N * 64 / us / 1e6:7.1f} TFLOP/s", flush=True)
