"""Measurement of the SURVEY §8 rows outside the headline path (GPU tool, not a test).

One JSON line per row, each with the kernel time measured with HIP events on the stream the op runs
on, the algorithmic bytes (or FLOPs) per call, the roofline fraction against the MI355X peak, and
the CPU restatement (oracle/) timed on the same inputs on the host cores (a reported baseline):

* f1   ``mmt_rgbd_assemble``   get_rgbd_frame (depth_utils.py:7-58) at DepthTrack's 640 x 360:
       algorithmic bytes per frame = rgb 3 + depth 2 (median histogram) + depth 2 (min/max + map)
       + frame 6 = 13 B per pixel.
* A19  ``mmt_dimp_optimize``   DiMPSteepestDescentGN (optimizer.py:85-170) at the DiMP tracker's
       update shapes (sample memory 50, 8 sequences, 512 x 18 x 18 features, 4 x 4 filter,
       net_opt_update_iter 2): per Gauss-Newton iteration the features are read three times
       (scores, filter gradient, J g) = 3 x I x S x C x H x W x 4 B.
* A18  ``mmt_xcorr_nhwc``      SiamFC correlation of 3 scales (AlexNet-5 [256, 6, 6] exemplar over
       [256, 22, 22] instances -> 3 x 17 x 17): 2 C hz wz ho wo FLOP per scale; plus the whole
       SiamFC update (HIP crop, HIP AlexNet, HIP xcorr, HIP cubic response) in frames/s.

usage: python tools/bench_rows.py [--rows f1,A19,A18] [--cpu-seconds 4]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0
PEAK_FP32_TFLOPS = 157.3   # vector / f32-MFMA peak (MI355X_MICROARCH.md)


def gpu_time_us(fn, n=50, warm=5):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def cpu_time_s(fn, seconds):
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n, n


def row_rgbd(cpu_seconds):
    from mmtrack_amd.frames import assemble_rgbd
    from oracle import frames as of
    H, W = 360, 640
    rng = np.random.Generator(np.random.PCG64(3))
    rgb = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    depth = rng.integers(0, 12000, size=(H, W), dtype=np.uint16)
    depth[rng.random((H, W)) < 0.05] = 0
    r_d = torch.from_numpy(rgb).cuda()
    d_d = torch.from_numpy(depth.view(np.int16)).cuda()
    out = torch.empty(H, W, 6, dtype=torch.uint8, device="cuda")
    us = gpu_time_us(lambda: assemble_rgbd(r_d, d_d, out=out), n=200)
    ok = np.array_equal(out.cpu().numpy(), of.rgbd_frame(rgb, depth))
    nbytes = 13.0 * H * W
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    ct, n = cpu_time_s(lambda: of.rgbd_frame(rgb, depth), cpu_seconds)
    gbs = nbytes / us / 1e3
    return {"row": "f1", "op": "mmt_rgbd_assemble", "shape": f"{H}x{W} rgb + uint16 depth -> {H}x{W}x6",
            "us_per_call": round(us, 2), "frames_per_s": round(1e6 / us, 1), "bit_exact_vs_oracle": bool(ok),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_call": nbytes},
            "cpu_baseline": {"value": round(1.0 / ct, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                             "sample": f"{n} frames through oracle/frames.py rgbd_frame (numpy)"}}


def row_dimp(cpu_seconds):
    from mmtrack_amd.dimp import DiMPSteepestDescentGN
    from oracle import dimp as od
    I, S, C, H, W, it = 50, 8, 512, 18, 18, 2
    g = torch.Generator().manual_seed(0)
    sd = {"log_step_length": torch.tensor([0.0]), "filter_reg": torch.tensor([0.1]),
          "label_map_predictor.weight": torch.linspace(1.0, -0.2, 10).view(1, 10, 1, 1),
          "target_mask_predictor.0.weight": torch.linspace(3.0, -3.0, 10).view(1, 10, 1, 1),
          "spatial_weight_predictor.weight": torch.ones(1, 10, 1, 1)}
    feat = torch.randn(I, S, C, H, W, generator=g) * 0.3
    bb = torch.tensor([[[128.0, 128.0, 40.0, 30.0]] * S] * I)
    w0 = torch.randn(S, C, 4, 4, generator=g) * 0.01
    opt = DiMPSteepestDescentGN(sd, num_iter=it)
    fd, wd = feat.cuda(), w0.cuda()
    us = gpu_time_us(lambda: opt.optimize(wd, fd, bb, num_iter=it), n=30)
    wg = opt.optimize(wd, fd, bb, num_iter=it).cpu()
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    ref, _, _ = od.steepest_descent_gn(w0.clone(), feat, bb, sd, it)
    err = float((wg - ref).abs().max() / ref.abs().max())
    ct, n = cpu_time_s(lambda: od.steepest_descent_gn(w0.clone(), feat, bb, sd, it), cpu_seconds)
    nbytes = 3.0 * it * I * S * C * H * W * 4
    gbs = nbytes / us / 1e3
    return {"row": "A19", "op": "mmt_dimp_optimize", "shape": f"I={I} S={S} C={C} {H}x{W}, 4x4 filter, {it} GN iters",
            "us_per_call": round(us, 2), "updates_per_s": round(S * 1e6 / us, 1), "max_rel_err_vs_oracle": err,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_call": nbytes},
            "cpu_baseline": {"value": round(S / ct, 2), "unit": "sequence-updates/s", "cores": threads, "kind": "port",
                             "sample": f"{n} calls of oracle/dimp.py steepest_descent_gn (torch {threads} threads)"}}


def row_siamfc(cpu_seconds):
    import ctypes
    from mmtrack_amd import _lib, synth
    from mmtrack_amd.siamfc import TrackerSiamFC
    from oracle import siamfc as osf
    lib = _lib.load()
    n, C, hz, hx = 3, 256, 6, 22
    ho = hx - hz + 1
    g = torch.Generator().manual_seed(1)
    z = torch.randn(1, C, hz, hz, generator=g)          # one exemplar, three scales of the instance
    x = torch.randn(n, C, hx, hx, generator=g)
    zd, xd = z.expand(n, C, hz, hz).contiguous().cuda(), x.cuda()
    out = torch.empty(n, 1, ho, ho, device="cuda")
    s = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    us = gpu_time_us(lambda: lib.mmt_xcorr(zd.data_ptr(), xd.data_ptr(), out.data_ptr(), n, C, hz, hz, hx, hx,
                                           ctypes.c_float(0.001), ctypes.c_float(0.0), s()), n=200)
    ref = osf.xcorr(z, x)
    err = float((out.cpu() - ref).abs().max())
    # the NHWC correlation the tracker runs since the backbone is on the HIP conv (one exemplar for 3 scales)
    zn, xn = z[0].permute(1, 2, 0).contiguous().cuda(), x.permute(0, 2, 3, 1).contiguous().cuda()
    out2 = torch.empty(n, 1, ho, ho, device="cuda")
    us_nhwc = gpu_time_us(lambda: lib.mmt_xcorr_nhwc(zn.data_ptr(), 0, xn.data_ptr(), out2.data_ptr(), n, C, hz, hz,
                                                     hx, hx, ctypes.c_float(0.001), ctypes.c_float(0.0), s()), n=200)
    err_nhwc = float((out2.cpu() - ref).abs().max())
    flops = 2.0 * n * C * hz * hz * ho * ho
    tfs = flops / us_nhwc / 1e6   # the roofline line is the NHWC kernel the tracker runs
    # the whole SiamFC update step (C1 config, here on the GPU)
    frames, gt = synth.make_frames(7, 12, 360, 640, 3, box=(300.0, 160.0, 40.0, 30.0))
    tr = TrackerSiamFC(state_dict=synth.make_siamfc_state_dict(0))
    tr.init(frames[0], gt[0])
    fdev = [torch.from_numpy(f).cuda() for f in frames]
    for f in fdev[1:4]:
        tr.update(f)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(60):
        tr.update(fdev[1 + k % (len(fdev) - 1)])
    torch.cuda.synchronize()
    upd = 60 / (time.perf_counter() - t0)
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    ct, cn = cpu_time_s(lambda: osf.xcorr(z, x), cpu_seconds)
    return {"row": "A18", "op": "mmt_xcorr_nhwc (the tracker's; NCHW mmt_xcorr beside it)",
            "shape": f"{n} x [{C},{hz},{hz}] * [{C},{hx},{hx}] -> {n}x{ho}x{ho}",
            "us_per_call": round(us_nhwc, 2), "max_abs_err_vs_oracle": err_nhwc,
            "nchw_us_per_call": round(us, 2), "nchw_max_abs_err_vs_oracle": err,
            "siamfc_update_frames_per_s": round(upd, 1),
            "roofline": {"bound": "fp32 VALU (latency-bound at this size)", "achieved": round(tfs, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tfs / PEAK_FP32_TFLOPS, 5),
                         "flop_per_call": flops},
            "cpu_baseline": {"value": round(1e6 * ct, 1), "unit": "us/call", "cores": threads, "kind": "port",
                             "sample": f"{cn} calls of oracle/siamfc.py xcorr (torch conv2d, {threads} threads)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="f1,A19,A18")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    a = ap.parse_args()
    assert torch.cuda.is_available(), "bench_rows.py needs an MI355X"
    torch.cuda.set_device(0)
    fns = {"f1": row_rgbd, "A19": row_dimp, "A18": row_siamfc}
    for r in a.rows.split(","):
        print(json.dumps(fns[r](a.cpu_seconds)), flush=True)


if __name__ == "__main__":
    main()
