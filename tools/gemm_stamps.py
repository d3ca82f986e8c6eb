"""Per-block phase timing of the GEMM kernels from s_memtime stamps (GPU tuning tool, not a test).
Prints median prologue / main-loop / epilogue cycles and the kernel span per block."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
B = int(os.environ.get("B", "32"))
shapes = {"fc1": (B * 320, 3072, 768, 1), "qkv": (B * 320, 2304, 768, 0), "fc2": (B * 320, 768, 3072, 2),
          "proj": (B * 320, 768, 768, 2), "sq4k": (4096, 4096, 4096, 0)}
s = torch.cuda.current_stream().cuda_stream
for name in os.environ.get("SHAPES", "fc1,qkv,sq4k").split(","):
    M, N, K, epi = shapes[name]
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda")
    C = torch.zeros(M, N, device="cuda", dtype=torch.float32 if epi == 2 else torch.bfloat16)
    st = torch.zeros(200000, dtype=torch.int64, device="cuda")
    for cfg in [int(c) for c in os.environ.get("CFGS", "-1,9").split(",")]:
        lib.mmt_gemm_force_config(cfg)
        run = lambda: lib.mmt_op_gemm(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr(), C.data_ptr(), N,
                                      C.data_ptr() if epi == 2 else None, N, M, N, K, epi, 0, 0, 0, s)
        for _ in range(3):
            run()
        st.zero_()
        lib.mmt_gemm_stamps(st.data_ptr())
        run()
        torch.cuda.synchronize()
        lib.mmt_gemm_stamps(None)
        t = st.view(-1, 4)
        t = t[t[:, 0] > 0].double()
        pro, main, epi_c = (t[:, 1] - t[:, 0]), (t[:, 2] - t[:, 1]), (t[:, 3] - t[:, 2])
        print(f"{name} cfg={cfg:2d} blocks={t.shape[0]:5d}  prologue {pro.median():8.0f}  main {main.median():8.0f}"
              f"  epilogue {epi_c.median():8.0f}  total {(t[:, 3] - t[:, 0]).median():8.0f} cyc (median)", flush=True)
    lib.mmt_gemm_force_config(-1)
