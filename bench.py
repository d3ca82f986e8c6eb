"""Headline benchmark: tracked frames/sec/GPU, ViPT-deep ViT-B, 128^2 template / 256^2 search, bf16.

One "step" = one tracking step of B independent sequences on each GPU (mmt_track_batch_submit +
_fetch, frames pipelined LAG deep; --sync: blocking mmt_track_batch): crop geometry from the last box +
normalise from the HBM-resident frame, dual patch-embed, 12 ViT-B blocks with deep prompts and CE,
CENTER head, windowed argmax decode, box back-mapping.  Frames are synthetic 640x480x6 uint8
(RGB + thermal-like aux) already resident in HBM; weights are the seeded synthetic law of
mmtrack_amd.synth (no checkpoint ships with the reference).

Multi-GPU: one process per GPU (torchrun), sequences sharded per rank, no data-path collective
(the reference shards sequences over a Pool, test_rgbt_mgpus.py:180-184); a gloo barrier and a
max-over-ranks of the timed region only.
"""
import argparse
import collections
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
LAG = 2   # frames a sequence may have in flight ahead of its fetched boxes (pipelined mode)

WORKLOADS = {
    # name: (engine kwargs, synth shape kwargs, frame H, W, C, published-config description)
    "vipt_deep_rgbt": (dict(), dict(kind="vipt", prompt_type="vipt_deep"), 480, 640, 6,
                       "ViPT-deep RGB-T, ViT-B/16, template 128 / search 256 (BASELINE configs[1])"),
    "vipt_deep_rgbd": (dict(), dict(kind="vipt", prompt_type="vipt_deep"), 360, 640, 6,
                       "ViPT-deep RGB-D (DepthTrack shapes 640x360) (BASELINE configs[2])"),
    "ostrack384": (dict(model="ostrack", prompt_type="none", in_chans=3, template_size=192, search_size=384,
                        search_factor=5.0), dict(kind="ostrack", search_size=384, template_size=192), 480, 640, 3,
                   "OSTrack RGB ViT-B, template 192 / search 384 (BASELINE configs[3])"),
}
GFLOP_PER_FRAME = {"vipt_deep_rgbt": 45.80, "vipt_deep_rgbd": 45.80, "ostrack384": 109.34}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(workload, frames_np, gts, seconds=12.0):
    """The fp32 CPU oracle tracker (oracle/tracker.py) on the same synthetic frames, bounded sample."""
    from mmtrack_amd import synth
    from oracle import tracker as otracker
    from oracle import vipt as ov
    ekw, skw, H, W, C, _ = WORKLOADS[workload]
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = synth.make_state_dict(0, **skw)
    cfg = ov.NetCfg(kind=skw["kind"], prompt_type=skw.get("prompt_type", "vipt_deep"),
                    search_size=skw.get("search_size", 256), template_size=skw.get("template_size", 128))
    tr = otracker.OracleTracker(sd, cfg, search_factor=ekw.get("search_factor", 4.0))
    tr.initialize(frames_np[0], {"init_bbox": list(gts[0])})
    tr.track(frames_np[1])  # warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        tr.track(frames_np[2 + n % (len(frames_np) - 2)])
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames of one sequence through the fp32 CPU oracle tracker "
                      f"(crop+net+decode, torch {threads} threads, {dt:.1f}s)"}


def pmc_traffic(probe, path=None):
    """HBM bytes per launch of the probed kernel class from the committed PMC summary
    (tests/pmc_bench.sh + tests/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 passes)."""
    import glob
    import re
    epi = {"fc1": 1, "qkv": 0, "fc2": 2, "proj": 2}.get(probe)
    files = [path] if path else sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic*.json")))
    if epi is None or not files or not os.path.exists(files[-1]):
        return None, None
    ks = json.load(open(files[-1]))["kernels"]
    best = None
    for name, d in ks.items():
        m = (re.match(r"gemm_kernel<\d+, \d+, \d+, \d+, (\d+), 0, false", name) or re.match(r"gemm256_kernel<(\d+)>", name)
             or re.match(r"gemm_persist_kernel<\d+, \d+, \d+, \d+, (\d+)>", name))
        if m and int(m.group(1)) == epi and "traffic_bytes_per_dispatch" in d:
            if best is None or d["dispatches"] > best[1]["dispatches"]:
                best = (name, d)
    if best is None:
        return None, None
    return best[1]["traffic_bytes_per_dispatch"], os.path.relpath(files[-1], REPO) + ":" + best[0]


def aggregate_throughput(batch, steps, elapsed):
    """(whole-job frames/s, max-over-ranks elapsed): every rank tracked batch x steps frames."""
    from mmtrack_amd.sharding import max_over_ranks, rank_world
    _, world = rank_world()
    elapsed = max_over_ranks(elapsed)
    return world * batch * steps / elapsed, elapsed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="sequences tracked per GPU per step")
    ap.add_argument("--workload", default="vipt_deep_rgbt", choices=list(WORKLOADS))
    ap.add_argument("--frames", type=int, default=8, help="distinct synthetic frames per sequence (cycled)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--sync", action="store_true", help="blocking per-frame calls (no frame pipelining)")
    ap.add_argument("--probe", default="fc1", help="kernel class timed with HIP events for the roofline ('none': off)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(local)

    from mmtrack_amd import Engine, EngineConfig, synth
    ekw, skw, H, W, C, desc = WORKLOADS[args.workload]
    B = args.batch
    cfg = EngineConfig(max_batch=B, use_graphs=not args.no_graphs, **ekw)
    sd = synth.make_state_dict(0, **skw)
    eng = Engine(cfg, sd, device=local)

    # synthetic video, HBM-resident; every sequence tracks its own target box in it
    video_np, gts = synth.make_frames(1000 + rank, args.frames + 1, H, W, C)
    video = torch.from_numpy(video_np).cuda()
    boxes0 = [[60.0 + (37 * i) % (W - 160), 40.0 + (23 * i) % (H - 120), 30.0 + (i % 5) * 6, 24.0 + (i % 3) * 8]
              for i in range(B)]
    for i in range(B):
        eng.initialize(i, video[0], boxes0[i])
    torch.cuda.synchronize()
    frame_lists = [[video[1 + t]] * B for t in range(args.frames)]

    def step(k):
        eng.track_batch(0, frame_lists[k % args.frames])

    def run(k0, count):
        """`count` frames of every sequence.  Pipelined (default): the tracker state lives on the device,
        so frame k+1 is submitted before frame k's boxes are fetched (at most LAG frames in flight);
        every frame's boxes reach the host before this returns.  --sync: one blocking call per frame."""
        if args.sync:
            for k in range(k0, k0 + count):
                step(k)
            return
        pend = collections.deque()
        for k in range(k0, k0 + count):
            pend.append(eng.track_batch_submit(0, frame_lists[k % args.frames]))
            if len(pend) > LAG:
                eng.track_batch_fetch(pend.popleft())
        while pend:
            eng.track_batch_fetch(pend.popleft())

    run(0, max(args.warmup, 2))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    value, elapsed = aggregate_throughput(B, args.steps, t1 - t0)

    # roofline probe: the same steps again, launched eagerly (HIP cannot time event nodes captured in a
    # graph), with HIP events on the engine stream around every launch of the dominant kernel class
    roof = None
    if args.probe and args.probe != "none":
        eng.timing_enable(args.probe)
        for k in range(min(args.steps, 20)):
            step(args.warmup + k)
        tr = eng.timing_read()
        eng.timing_enable(None)
        if tr["launches"]:
            avg_ms = tr["total_ms"] / tr["launches"]
            fl = tr["flops"] / tr["launches"]
            achieved = fl / (avg_ms * 1e-3) / 1e12
            traffic, src = pmc_traffic(args.probe) if B == 32 and args.workload == "vipt_deep_rgbt" else (None, None)
            roof = {"bound": "mfma", "kernel": f"gemm[{args.probe}]", "achieved": round(achieved, 1),
                    "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                    "traffic": round(traffic) if traffic else None, "traffic_unit": "bytes/launch (HBM, PMC)",
                    "traffic_source": src, "algorithmic_bytes_per_launch": tr["bytes"] / tr["launches"],
                    "avg_launch_us": round(avg_ms * 1e3, 2), "flop_per_launch": fl, "launches": tr["launches"]}

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.workload, video_np, gts, args.cpu_seconds)
        gf = GFLOP_PER_FRAME[args.workload]
        line = {
            "metric": "tracked frames/sec/GPU, ViPT ViT-B 256² search bf16, at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": args.workload, "description": desc, "sequences_per_gpu": B,
                       "global_batch": B * world, "frame": f"{W}x{H}x{C} uint8 (HBM-resident)",
                       "template": cfg.template_size, "search": cfg.search_size, "parallelism": f"seq-shard x{world}",
                       "graphs": cfg.use_graphs, "pipelined_frames": 0 if args.sync else LAG,
                       "weights": "synthetic seeded (no checkpoint ships)"},
            "per_gpu_fps": round(value / world, 2),
            "model_tflops": round(value * gf / 1e3, 1),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
