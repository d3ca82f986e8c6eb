"""f16x3 conv timing on the DiMP feature net's shapes (GPU tuning tool, not a test; the tuning knobs
MMT_CONV_SLOTS / MMT_CONV_PREFER64 / MMT_CONV_NOSPLIT are read once per process, so one process per setting).
Prints one JSON line per shape: microseconds per launch, algorithmic TF/s and the fraction of 833 TF/s."""
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multi-modal-trakcing-bechmark_amd"))
import torch  # noqa: E402

from mmtrack_amd import _lib, dimpnet  # noqa: E402

# name: (N images, groups, Cin, H, W, Cout, k, stride, pad)
SHAPES = {"clf": (32, 1, 1024, 18, 18, 512, 3, 1, 1), "l3_c2": (32, 2, 256, 18, 18, 256, 3, 1, 1),
          "l3_c1": (32, 2, 1024, 18, 18, 256, 1, 1, 0), "l3_c3": (32, 2, 256, 18, 18, 1024, 1, 1, 0),
          "l2_c2": (32, 2, 128, 36, 36, 128, 3, 1, 1), "l1_c2": (32, 2, 64, 72, 72, 64, 3, 1, 1),
          "l1_c3": (32, 2, 64, 72, 72, 256, 1, 1, 0)}
sel = os.environ.get("SHAPES")
lib = _lib.load()
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for name, (N, G, C, H, W, Co, k, s, p) in SHAPES.items():
    if sel and name not in sel.split(","):
        continue
    g = torch.Generator().manual_seed(1)
    convs = [dimpnet._Conv(torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k),
                           bias=torch.randn(Co, generator=g) * 0.1, stride=s, pad=p, dev="cuda", f16x3=True)
             for _ in range(G)]
    Ho, Wo = convs[0].out_hw(H, W)
    xs = [torch.randn(N, H, W, C, device="cuda") for _ in range(G)]
    outs = [torch.empty(N, Ho, Wo, Co, device="cuda") for _ in range(G)]
    groups = [convs[i].group(xs[i], outs[i], relu=True, x_scale=dimpnet.range_scale(5.0)) for i in range(G)]
    bufs = {}

    def wsf(n):
        if n not in bufs:
            bufs[n] = torch.empty((n + 3) // 4, device="cuda")
        return bufs[n]

    def run():
        dimpnet.run_f16x3(lib, convs[0], groups, N, H, W, wsf, stream)
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
    fl = 2.0 * G * N * Ho * Wo * Co * C * k * k
    print(json.dumps({"env": " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("MMT_CONV")),
                      "shape": name, "us": round(us, 2), "tflops": round(fl / us / 1e6, 1),
                      "frac_f16x3": round(fl / us / 1e6 / (2500 / 3), 4)}), flush=True)
