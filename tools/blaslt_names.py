"""Which hipBLASLt kernels torch picks for the path's GEMM shapes (tuning tool: run under
rocprofv3 --kernel-trace; the Tensile kernel names carry the macro tile, MFMA shape and pipelining)."""
import torch
import torch.nn.functional as F

shapes = {"fc1": (10240, 3072, 768), "qkv": (10240, 2304, 768), "fc2": (10240, 768, 3072), "proj": (10240, 768, 768),
          "fc1@4896": (4896, 3072, 768)}
for name, (m, n, k) in shapes.items():
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        F.linear(a, w, b)
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push(name) if hasattr(torch.cuda, "nvtx") else None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        F.linear(a, w, b)
    ev1.record()
    torch.cuda.synchronize()
    print(f"{name}: {ev0.elapsed_time(ev1) / 20 * 1e3:.1f} us", flush=True)
