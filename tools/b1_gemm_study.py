"""One-sequence GEMM study (GPU tuning tool, not a test): the f16x3 GEMMs of a one-sequence frame (M = 320 rows)
timed with their weights cold (cycled through distinct copies totalling > 256 MB, as a frame finds them: the
372 MB of hi + lo weights do not fit the Infinity Cache) and warm (the same copy again), with per-block
s_memtime stamps (prologue = first K-tile landed, main loop, epilogue).  The tile config is the heuristic's
unless MMT_SPLIT_CFG pins one (read once per process).  One JSON line per (shape, mode)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib  # noqa: E402

lib = _lib.load()
M = int(os.environ.get("M", "320"))
SHAPES = {"qkv": (2304, 768, 0), "fc1": (3072, 768, 1), "fc2": (768, 3072, 2), "proj": (768, 768, 2)}
s = torch.cuda.current_stream().cuda_stream
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
for name in os.environ.get("SHAPES", "qkv,fc1,fc2,proj").split(","):
    N, K, epi = SHAPES[name]
    Ah = torch.randn(M, K, device="cuda").half()
    Al = (torch.randn(M, K, device="cuda") * 1e-3).half()
    wbytes = N * K * 4
    ncopy = max(2, (300 << 20) // wbytes + 1)
    Wh = [(torch.randn(N, K, device="cuda") * 0.05).half() for _ in range(ncopy)]
    Wl = [(torch.randn(N, K, device="cuda") * 5e-5).half() for _ in range(ncopy)]
    bias = torch.randn(N, device="cuda")
    if epi in (0, 1):
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        Cl = torch.empty_like(C)
    else:
        C = torch.zeros(M, N, device="cuda")
        Cl = None

    def run(k):
        lib.mmt_op_gemm_f16x3(Ah.data_ptr(), Al.data_ptr(), K, Wh[k].data_ptr(), Wl[k].data_ptr(), K,
                              bias.data_ptr(), C.data_ptr(), Cl.data_ptr() if Cl is not None else None, N,
                              C.data_ptr() if epi == 2 else None, N if epi == 2 else 0, M, N, K, epi, 1e-3, 1.0,
                              0, 0, s)
    st = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
    scratch = torch.empty(2, device="cuda")
    # "mall": each launch's weight copy read by another kernel (torch.sum, its own XCD placement) just before the
    # GEMM, which then finds it in the Infinity Cache and mostly not in its XCD's L2 -- what a prefetch of the next
    # GEMM's weights on a side stream would give; timed per launch with events around the GEMM alone
    for mode in ("mall",):
        for k in range(ncopy):
            run(k)
        flush.fill_(1)
        ts = []
        for i in range(2 * ncopy):
            k = i % ncopy
            scratch[0] = torch.sum(Wh[k], dtype=torch.float32)
            scratch[1] = torch.sum(Wl[k], dtype=torch.float32)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(k)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "mode": mode,
                          "cfg": os.environ.get("MMT_SPLIT_CFG", "-1"), "us_median": round(us[len(us) // 2], 2),
                          "us_min": round(us[0], 2)}), flush=True)
        # the same single-launch event timing in the cold and warm states, for comparison
        for sub in ("cold", "warm"):
            ts = []
            for i in range(2 * ncopy):
                k = i % ncopy if sub == "cold" else 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(k)
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
            print(json.dumps({"shape": name, "mode": sub + "_single", "us_median": round(us[len(us) // 2], 2),
                              "us_min": round(us[0], 2)}), flush=True)
    for mode in ("cold", "warm"):
        for k in range(ncopy):
            run(k)
        flush.fill_(1)
        n = 3 * ncopy if mode == "cold" else 40
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            run(i % ncopy if mode == "cold" else 0)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        # stamps of one launch in the same state
        run(0 if mode == "warm" else 1)
        flush.fill_(2) if mode == "cold" else None
        st.zero_()
        lib.mmt_gemm_stamps(st.data_ptr())
        run(0 if mode == "warm" else 2)
        torch.cuda.synchronize()
        lib.mmt_gemm_stamps(None)
        t = st.view(-1, 4)
        t = t[t[:, 0] > 0].double()
        rec = {"shape": name, "M": M, "N": N, "K": K, "mode": mode, "cfg": os.environ.get("MMT_SPLIT_CFG", "-1"),
               "us_per_launch": round(us, 2), "weight_copies": ncopy}
        if t.shape[0]:
            t0 = t[:, 0].min()
            rec.update({"blocks": int(t.shape[0]), "prologue_cyc": float((t[:, 1] - t[:, 0]).median()),
                        "main_cyc": float((t[:, 2] - t[:, 1]).median()),
                        "epilogue_cyc": float((t[:, 3] - t[:, 2]).median()),
                        "block_span_cyc": float((t[:, 3] - t[:, 0]).median()),
                        "start_spread_cyc": float(t[:, 0].max() - t0), "kernel_span_cyc": float(t[:, 3].max() - t0)})
        print(json.dumps(rec), flush=True)
