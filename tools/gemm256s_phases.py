"""Per-phase timing of the f16x3 256 x 256 GEMM (gemm256s_kernel) from in-kernel s_memtime stamps (GPU tuning tool,
not a test).  Needs a library built with -DGEMM_PHASE_STAMPS (tools/build_variant.sh phase "-DGEMM_PHASE_STAMPS",
then MMTRACK_LIB=abx/libphase.so).  Per phase and wave group (waves 0-3 / 4-7) three stamps: before the counted
vmcnt wait (fragment reads issued), after the first barrier (MFMA start), after the second barrier (phase end).
Prints, per shape, the median cycles of: wait + load issue + barrier, MFMA + barrier, fragment reads, over the
steady phases of the first 256 blocks, and the loop's share spent in each."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
PS = 3 * 96
SHAPES = {"qkv_half": (5120, 2304, 768, 0), "fc1_half": (5120, 3072, 768, 1), "qkv": (10240, 2304, 768, 0),
          "fc1": (10240, 3072, 768, 1)}
s = torch.cuda.current_stream().cuda_stream
st = torch.zeros(65536 + 256 * 2 * PS, dtype=torch.int64, device="cuda")
for name in os.environ.get("SHAPES", "qkv_half,fc1_half,qkv,fc1").split(","):
    M, N, K, epi = SHAPES[name]
    Ah = torch.randn(M, K, device="cuda").half()
    Al = (torch.randn(M, K, device="cuda") * 1e-3).half()
    Wh = (torch.randn(N, K, device="cuda") * 0.05).half()
    Wl = (torch.randn(N, K, device="cuda") * 5e-5).half()
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    Cl = torch.empty_like(C)

    def run():
        lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh.data_ptr(), Wl.data_ptr(), K, bias.data_ptr(),
                              C.data_ptr(), Cl.data_ptr(), N, None, 0, M, N, K, epi, 1e-3, 1.0, 0, 0, s)
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
    k4 = st[:65536].view(-1, 4)
    k4 = k4[k4[:, 0] > 0].double()
    ph = st[65536:].view(256, 2, PS).double()
    nph = 4 * (K // 32)
    rows = []
    for g in range(2):
        t = ph[:, g, :3 * nph].view(256, nph, 3)
        ok = t[:, :, 0] > 0
        wait = (t[:, :, 1] - t[:, :, 0])[:, 1:-2]
        mfma = (t[:, :, 2] - t[:, :, 1])[:, 1:-2]
        reads = (t[:, 1:, 0] - t[:, :-1, 2])[:, 1:-1]
        per_phase = (t[:, 1:, 2] - t[:, :-1, 2])[:, 1:-1]
        rows.append({"group": g, "blocks": int(ok[:, 0].sum()),
                     "wait_issue_barrier": float(wait.median()), "mfma_barrier": float(mfma.median()),
                     "reads": float(reads.median()), "phase": float(per_phase.median()),
                     "phase_p90": float(per_phase.quantile(0.9)) if per_phase.numel() < 16_000_000 else None})
    rec = {"shape": name, "M": M, "N": N, "K": K, "us": round(us, 2), "tflops": round(2 * M * N * K / us / 1e6, 1),
           "kernel_cycles_median": float((k4[:, 3] - k4[:, 0]).median()),
           "prologue": float((k4[:, 1] - k4[:, 0]).median()), "loop": float((k4[:, 2] - k4[:, 1]).median()),
           "epilogue": float((k4[:, 3] - k4[:, 2]).median()), "groups": rows,
           "mfma_cycles_ideal_per_phase": 24 * 16}
    print(json.dumps(rec), flush=True)
