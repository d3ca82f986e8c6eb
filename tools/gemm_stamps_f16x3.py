"""Per-block prologue / main-loop / epilogue cycles (s_memtime stamps, mmt_gemm_stamps) of the f16x3 GEMM launches
of one shape list (GPU tuning tool, not a test): the heuristic's tile for each shape, one launch stamped after a
warm-up; prints the medians and the launch time."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
SHAPES = {"fc2_half": (5120, 768, 3072, 2), "proj_half": (5120, 768, 768, 2), "fc2_153": (2448, 768, 3072, 2),
          "qkv_half": (5120, 2304, 768, 0), "fc1_half": (5120, 3072, 768, 1), "qkv_b1": (320, 2304, 768, 0),
          "fc1_b1": (320, 3072, 768, 1), "fc1_b8": (2560, 3072, 768, 1), "qkv_b8": (2560, 2304, 768, 0),
          "fc2_full": (10240, 768, 3072, 2), "proj_full": (10240, 768, 768, 2), "fc2_244": (7808, 768, 3072, 2)}
# MMT_FORCE: pin the tile (mmt_gemm_force_config: 128 = the 128 x 256 two-group kernel, 256 = 256 x 256)
s = torch.cuda.current_stream().cuda_stream
if os.environ.get("MMT_FORCE"):
    lib.mmt_gemm_force_config(int(os.environ["MMT_FORCE"]))
st = torch.zeros(65536 + 256 * 2 * 288, dtype=torch.int64, device="cuda")
for name in os.environ.get("SHAPES", ",".join(SHAPES)).split(","):
    M, N, K, epi = SHAPES[name]
    Ah = torch.randn(M, K, device="cuda").half()
    Al = (torch.randn(M, K, device="cuda") * 1e-3).half()
    Wh = (torch.randn(N, K, device="cuda") * 0.05).half()
    Wl = (torch.randn(N, K, device="cuda") * 5e-5).half()
    bias = torch.randn(N, device="cuda")
    if epi in (0, 1):
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        Cl = torch.empty_like(C)
    else:
        C = torch.randn(M, N, device="cuda")
        Cl = None

    def run():
        lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh.data_ptr(), Wl.data_ptr(), K, bias.data_ptr(),
                              C.data_ptr(), Cl.data_ptr() if Cl is not None else None, N,
                              C.data_ptr() if epi == 2 else None, N if epi == 2 else 0, M, N, K, epi, 1e-3, 1.0, 0, 0, s)
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    st.zero_()
    lib.mmt_gemm_stamps(st.data_ptr())
    run()
    torch.cuda.synchronize()
    lib.mmt_gemm_stamps(None)
    t = st[:65536].view(-1, 4)
    t = t[t[:, 0] > 0].double()
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": round(us, 2),
                      "tflops": round(2 * M * N * K / us / 1e6, 1), "blocks": int(t.shape[0]),
                      "prologue": float((t[:, 1] - t[:, 0]).median()), "loop": float((t[:, 2] - t[:, 1]).median()),
                      "epilogue": float((t[:, 3] - t[:, 2]).median()),
                      "block": float((t[:, 3] - t[:, 0]).median())}), flush=True)
