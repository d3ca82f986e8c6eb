"""GEMM tile-config sweep on the path's shapes (GPU tuning tool, not a test)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-trakcing-bechmark_amd"))
import torch
from mmtrack_amd import _lib
lib = _lib.load()
B = int(os.environ.get("B", "32"))
shapes = {"fc1": (B * 320, 3072, 768, 1), "qkv": (B * 320, 2304, 768, 0), "fc2": (B * 320, 768, 3072, 2),
          "proj": (B * 320, 768, 768, 2), "sq4k": (4096, 4096, 4096, 0), "fc1nog": (B * 320, 3072, 768, 0)}
if os.environ.get("SHAPES"):
    shapes = {k: v for k, v in shapes.items() if k in os.environ["SHAPES"].split(",")}
if os.environ.get("MS"):   # row counts to sweep instead of B * 320 (e.g. the CE-pruned layers' M)
    shapes = {f"{k}@{m}": (m, n, kk, e) for k, (_, n, kk, e) in shapes.items() for m in map(int, os.environ["MS"].split(","))}
CFGS = [int(c) for c in os.environ.get("CFGS", "-1,1,2,3,4,5,6,7,8").split(",")]


def time_it(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
s = torch.cuda.current_stream().cuda_stream
for name, (M, N, K, epi) in shapes.items():
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == 2 else torch.bfloat16)
    ref = None
    # library reference on the same operands (hipBLASLt through torch; bias, no fused epilogue)
    us = 0.0 if os.environ.get("NO_TORCH") else time_it(lambda: torch.nn.functional.linear(A, W, bias.bfloat16()))
    if us > 0:
        print(f"{name:10s} M={M} N={N} K={K} torch/hipBLASLt: {us:8.1f} us  {2*M*N*K/us/1e6:7.1f} TFLOP/s", flush=True)
    for cfg in CFGS:
        lib.mmt_gemm_force_config(cfg)
        def run():
            lib.mmt_op_gemm(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), C.data_ptr(), N,
                            C.data_ptr() if epi == 2 else None, N, M, N, K, epi, 0, 0, 0, s)
        if epi == 2:
            C.zero_()
        run(); torch.cuda.synchronize()
        if epi != 2:
            out = C.float().clone()
            if ref is None: ref = out
            err = (out - ref).abs().max().item()
        else:
            err = 0.0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3): run()
        e0.record()
        n = 20
        for _ in range(n): run()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        print(f"{name:10s} M={M} N={N} K={K} cfg={cfg:2d}: {us:8.1f} us  {2*M*N*K/us/1e6:7.1f} TFLOP/s  maxdiff {err:.2e}", flush=True)
lib.mmt_gemm_force_config(-1)
