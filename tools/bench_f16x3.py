"""f16x3 GEMM timing on the path's shapes for the tile config pinned by MMT_SPLIT_CFG (GPU tuning tool, not a
test; one process per config because the override is read once).  Prints one JSON line per shape."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
SHAPES = {"fc2": (10240, 768, 3072, 2), "fc2_ce": (4896, 768, 3072, 2), "proj": (10240, 768, 768, 2),
          "fc1": (10240, 3072, 768, 1), "qkv": (10240, 2304, 768, 0), "fc2_half": (5120, 768, 3072, 2),
          # one half's rows after each candidate elimination (16 sequences x 243 / 189 / 152 tokens)
          "fc2_243": (3888, 768, 3072, 2), "fc2_189": (3024, 768, 3072, 2), "fc2_152": (2432, 768, 3072, 2),
          "proj_152": (2432, 768, 768, 2), "proj_half": (5120, 768, 768, 2), "proj_243": (3888, 768, 768, 2),
          "proj_189": (3024, 768, 768, 2), "qkv_half": (5120, 2304, 768, 0), "fc1_half": (5120, 3072, 768, 1),
          "qkv_243": (3888, 2304, 768, 0), "fc1_243": (3888, 3072, 768, 1), "fc1_152": (2432, 3072, 768, 1), "qkv_152": (2432, 2304, 768, 0),
          # the FLOPs of fc2 at 32 sequences as 240 tiles of 256 x 256 over K = 1536 (a two-way K split's round)
          "fc2_sk2_emul": (20480, 768, 1536, 2), "fc2_k1536": (10240, 768, 1536, 2)}
sel = os.environ.get("SHAPES")
s = torch.cuda.current_stream().cuda_stream
for name, (M, N, K, epi) in SHAPES.items():
    if sel and name not in sel.split(","):
        continue
    Ah = torch.randn(M, K, device="cuda").half()
    Al = (torch.randn(M, K, device="cuda") * 1e-3).half()
    Wh = (torch.randn(N, K, device="cuda") * 0.05).half()
    Wl = (torch.randn(N, K, device="cuda") * 5e-5).half()
    bias = torch.randn(N, device="cuda")
    if epi in (0, 1):
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        Cl = torch.empty_like(C)
    else:
        C = torch.zeros(M, N, device="cuda")
        Cl = None

    def run():
        lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh.data_ptr(), Wl.data_ptr(), K, bias.data_ptr(),
                              C.data_ptr(), Cl.data_ptr() if Cl is not None else None, N,
                              C.data_ptr() if epi == 2 else None, N if epi == 2 else 0, M, N, K, epi, 1e-3, 1.0, 0, 0, s)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    tf = 2 * M * N * K / us / 1e6
    print(json.dumps({"cfg": os.environ.get("MMT_SPLIT_CFG", "-1"), "shape": name, "M": M, "N": N, "K": K, "us": round(us, 2),
                      "tflops": round(tf, 1), "frac_f16x3": round(tf / (2500 / 3), 4)}), flush=True)
