"""Headline benchmark: tracked frames/sec/GPU, ViPT-deep ViT-B, 128^2 template / 256^2 search.

One "step" = one tracking step of B independent sequences on each GPU (mmt_track_batch_submit +
_fetch, frames pipelined LAG deep; --sync: blocking mmt_track_batch): crop geometry from the last box +
normalise from the HBM-resident frame, dual patch-embed, 12 ViT-B blocks with deep prompts and CE,
CENTER head, windowed argmax decode, box back-mapping.  Frames are synthetic 640x480x6 uint8
(RGB + thermal-like aux) already resident in HBM; weights are the seeded synthetic law of
mmtrack_amd.synth (no checkpoint ships with the reference).

Precision (--precision): "fp32" (default) is the parity mode -- every MFMA operand split into fp16
hi/lo halves of range-scaled values (Wh*Ah + Wl*Ah + Wh*Al, "f16x3"), which reproduces the fp32 reference's candidate-
elimination decisions and windowed argmax (tests/test_gpu_parity.py); "bf16" is plain bf16 operands,
faster, but its CE decisions flip against the reference.

Multi-GPU: one process per GPU, sequences sharded per rank, no data-path collective (the reference
shards sequences over a Pool, test_rgbt_mgpus.py:180-184); a gloo barrier and a max-over-ranks of the
timed region only.  `--gpus N` without a torchrun environment spawns the N rank processes itself
(before anything touches a GPU); under torchrun WORLD_SIZE must equal --gpus.
"""
import argparse
import collections
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
LAG = 2   # frames a sequence may have in flight ahead of its fetched boxes (pipelined mode)
METRIC = "tracked frames/sec/GPU, ViPT ViT-B 256² search bf16, at 1/2/4/8 MI355X"

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
PEAK_FP32_MATRIX_TFLOPS = 157.3   # MI355X dense fp32 MFMA (v_mfma_f32_*_f32), MI355X_MICROARCH.md
DIMP_WORKLOAD = "mfdimp_rgbt"     # BASELINE configs[4]: mfDiMP RGB-T, ResNet-50 features + DiMP inner loop
PROBE_CLASSES = ("qkv", "proj", "fc1", "fc2", "attn", "conv1", "patch")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_quota():
    """CPUs this process may use: the cgroup quota (the GPU box's share) capped by the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(workload, frames_np, gts, seconds=4.0):
    """The fp32 CPU oracle tracker (oracle/tracker.py) on the same synthetic frames, bounded samples:
    full track (crop + network + decode) and network only, at the box's CPU share and at 1 thread."""
    from mmtrack_amd import synth
    from oracle import crop as ocrop
    from oracle import tracker as otracker
    from oracle import vipt as ov
    ekw, skw, H, W, C, _ = WORKLOADS[workload]
    sd = synth.make_state_dict(0, **skw)
    cfg = ov.NetCfg(kind=skw["kind"], prompt_type=skw.get("prompt_type", "vipt_deep"),
                    search_size=skw.get("search_size", 256), template_size=skw.get("template_size", 128))
    quota = cpu_quota()
    variants = []
    for threads in (quota, 1):
        torch.set_num_threads(threads)
        tr = otracker.OracleTracker(sd, cfg, search_factor=ekw.get("search_factor", 4.0))
        tr.initialize(frames_np[0], {"init_bbox": list(gts[0])})
        tr.track(frames_np[1])  # warm
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            tr.track(frames_np[2 + n % (len(frames_np) - 2)])
            n += 1
        dt = time.perf_counter() - t0
        variants.append({"part": "track", "threads": threads, "value": round(n / dt, 3), "frames": n,
                         "seconds": round(dt, 2)})
        # network only: the oracle forward on a fixed pre-cropped pair
        z = ocrop.preprocess(synth.make_patch(1, cfg.template_size, C))
        x = ocrop.preprocess(synth.make_patch(2, cfg.search_size, C))
        mask = ov.ce_template_mask(cfg)
        ov.forward(sd, z, x, cfg, mask)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            ov.forward(sd, z, x, cfg, mask)
            n += 1
        dt = time.perf_counter() - t0
        variants.append({"part": "network", "threads": threads, "value": round(n / dt, 3), "frames": n,
                         "seconds": round(dt, 2)})
    head = variants[0]
    return {"value": head["value"], "unit": "frames/s", "cores": quota, "kind": "port",
            "machine_cpus": os.cpu_count(), "variants": variants,
            "sample": f"{head['frames']} frames of one sequence through the fp32 CPU oracle tracker (crop + "
                      f"network + decode, {quota} torch threads = the box's CPU share, {head['seconds']} s); "
                      f"'variants' adds network-only and 1-thread samples of ~{seconds:.0f} s each"}


def dimp_traffic(batch, path=None):
    """HBM bytes per feature-net batch of the mfDiMP line from the committed PMC summary
    (tools/pmc_dimp_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE over the feature net's kernels, 32 images per batch)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic_dimp*.json"))) if path is None else [path]
    if not files or batch != 32:
        return None
    d = json.load(open(files[-1]))
    return {"bytes": d["bytes_per_batch"], "algorithmic_bytes": d.get("algorithmic_bytes_per_batch"),
            "ratio": d.get("ratio_to_algorithmic"), "source": os.path.relpath(files[-1], REPO),
            "build": d.get("build"), "note": "committed PMC summary (tools/pmc_dimp_traffic.sh), not measured by this run"}


def pmc_traffic(cls, precision, path=None):
    """HBM bytes per launch of the probed kernel class from the committed PMC summary
    (tools/pmc_bench.sh + tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 passes)."""
    import glob
    pat = f"*pmc_traffic_{precision}*.json"
    files = [path] if path else sorted(glob.glob(os.path.join(REPO, "profiles", pat)))
    if not files or not os.path.exists(files[-1]):
        return None, None
    d = json.load(open(files[-1]))
    c = d.get("classes", {}).get(cls)
    if not c or "traffic_bytes_per_dispatch" not in c:
        return None, None
    return c["traffic_bytes_per_dispatch"], os.path.relpath(files[-1], REPO) + ":" + cls


# C3 per GPU (one sequence), C4 and C5 as short samples after nothing has touched the GPU: each in a fresh child
# process (its own HIP context), so the default invocation's JSON line carries every single-GPU configuration of
# BASELINE.json, timed under the driver's clock.  name -> extra argv
EXTRAS = {
    "vipt_deep_rgbt_b1": ["--workload", "vipt_deep_rgbt", "--batch", "1", "--steps", "300", "--warmup", "30"],
    "ostrack384": ["--workload", "ostrack384", "--steps", "20", "--warmup", "5"],
    "mfdimp_rgbt": ["--workload", DIMP_WORKLOAD, "--steps", "30", "--warmup", "10"],
}


def run_extras(timeout=150):
    """The EXTRAS samples, one child process each (run before this process touches a GPU); per workload the
    child's own JSON line reduced to its rate, step time and roofline fraction."""
    out = {}
    for name, argv in EXTRAS.items():
        cmd = [sys.executable, os.path.abspath(__file__), "--no-extras", "--no-cpu-baseline", "--host-frames", "0"] + argv
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
            rc, text, err = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired:
            rc, text, err = "timeout", "", ""
        rec = {"rc": rc, "seconds": round(time.perf_counter() - t0, 1), "argv": " ".join(argv)}
        lines = [ln for ln in text.splitlines() if ln.startswith("{")]
        if rc == 0 and lines:
            d = json.loads(lines[-1])
            roof = d.get("roofline") or {}
            rec.update({"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps": d["steps"],
                        "warmup": d["warmup"], "sequences_per_gpu": d["config"]["sequences_per_gpu"],
                        "dtype": d["dtype"], "frac": roof.get("frac"), "roofline_kernel": roof.get("kernel"),
                        "roofline_achieved": roof.get("achieved"), "roofline_peak": roof.get("peak"),
                        "frac_of_layer_roofline": roof.get("frac_of_layer_roofline"),
                        "step_frac_of_peak": d.get("step_frac_of_peak"), "description": d["config"]["description"]})
        else:
            rec["stderr_tail"] = err[-600:]
        log(f"bench extra {name}: {rec.get('value')} frames/s ({rec['seconds']} s, rc {rc})")
        out[name] = rec
    return out


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """One child process per GPU with the torchrun environment; rank 0 prints the JSON line.  Called
    before this process touches any GPU (no HIP context to inherit)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def aggregate_throughput(batch, steps, elapsed):
    """(whole-job frames/s, max-over-ranks elapsed, world): every rank tracked batch x steps frames.

    `value` is this whole-job rate, as the driver's bench contract defines it (it derives the scaling
    efficiency from the per-N values itself); the per-GPU rate the metric's name quotes is `per_gpu_fps`."""
    from mmtrack_amd.sharding import max_over_ranks, rank_world
    _, world = rank_world()
    elapsed = max_over_ranks(elapsed)
    return world * batch * steps / elapsed, elapsed, world


def probe_classes(eng, step, k0, nsteps, precision):
    """HIP-event timing of every launch of each kernel class on the engine stream (eager replays of the
    same steps: HIP cannot time event nodes captured in a graph)."""
    out = {}
    for cls in PROBE_CLASSES:
        eng.timing_enable(cls)
        for k in range(nsteps):
            step(k0 + k)
        tr = eng.timing_read()
        eng.timing_enable(None)
        if not tr["launches"]:
            continue
        avg_ms = tr["total_ms"] / tr["launches"]
        fl = tr["flops"] / tr["launches"]
        by = tr["bytes"] / tr["launches"]
        out[cls] = {"launches": tr["launches"], "avg_launch_us": round(avg_ms * 1e3, 2),
                    "ms_per_step": round(tr["total_ms"] / nsteps, 4), "flop_per_launch": fl,
                    "algorithmic_bytes_per_launch": by,
                    "achieved_tflops": round(fl / (avg_ms * 1e-3) / 1e12, 1),
                    "achieved_gbs": round(by / (avg_ms * 1e-3) / 1e9, 1)}
    return out


def roofline_from(classes, precision, workload, batch):
    """The dominant class (most time per step) as the roofline line; every class kept beside it."""
    if not classes:
        return None
    dom = max(classes, key=lambda c: classes[c]["ms_per_step"])
    c = classes[dom]
    split = precision == "fp32"
    # f16x3: three fp16 MFMAs (bf16 rate) per product, so the arithmetic's dense peak is the bf16 peak / 3
    peak = PEAK_BF16_TFLOPS / 3 if split else PEAK_BF16_TFLOPS
    traffic, src = pmc_traffic(dom, precision) if (batch == 32 and workload == "vipt_deep_rgbt") else (None, None)
    for k, v in classes.items():
        v["frac_of_peak"] = round(v["achieved_tflops"] / peak, 4)
    return {"bound": "mfma", "kernel": dom, "achieved": c["achieved_tflops"], "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(c["achieved_tflops"] / peak, 4),
            "traffic": round(traffic) if traffic else None, "traffic_unit": "bytes/launch (HBM, PMC)",
            "traffic_source": src,
            "traffic_note": ("from the committed PMC pass of this build (tools/pmc_bench.sh, FETCH_SIZE x2 + WRITE_SIZE, halves "
                             "off as the probe runs), not measured by this run") if src else None,
            "algorithmic_bytes_per_launch": c["algorithmic_bytes_per_launch"],
            "avg_launch_us": c["avg_launch_us"], "flop_per_launch": c["flop_per_launch"],
            "launches": c["launches"],
            "peak_note": ("f16x3 split products (Wh*Ah + Wl*Ah + Wh*Al, fp16 MFMA at the bf16 rate): dense 2500 TF/s / 3; achieved counts "
                          "algorithmic 2MNK flops, the MFMA pipe issues 3x that") if split else "dense bf16",
            "mfma_pipe_frac": round(c["achieved_tflops"] * (3 if split else 1) / PEAK_BF16_TFLOPS, 4),
            "probe_config": ("eager launches of the timed steps' kernels with the two-stream halves off (HIP cannot "
                             "time kernels inside a captured graph, and the halves would overlap the classes): "
                             "each class's own duration, not its share of the overlapped step"),
            "classes": classes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="sequences tracked per GPU per step (default 32)")
    ap.add_argument("--workload", default="vipt_deep_rgbt", choices=list(WORKLOADS) + [DIMP_WORKLOAD])
    ap.add_argument("--precision", default="fp32", choices=("fp32", "bf16"),
                    help="fp32: parity mode (f16x3 split products); bf16: plain bf16 operands")
    ap.add_argument("--frames", type=int, default=8, help="distinct synthetic frames per sequence (cycled)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--sync", action="store_true", help="blocking per-frame calls (no frame pipelining)")
    ap.add_argument("--probe", default="all", help="'all': time every kernel class for the roofline; 'none': off")
    ap.add_argument("--host-frames", type=int, default=10,
                    help="steps of an extra PCIe-inclusive pass with frames in pinned host memory (0: off)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="per CPU-baseline sample (4 samples)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry", action="store_true", help="no GPU: sleep for the step (tests the multi-rank plumbing)")
    ap.add_argument("--dimp-groups", type=int, default=1, help="mfdimp: PipelinedBatch groups of sequences")
    ap.add_argument("--dimp-precision", default="f16x3", choices=("f16x3", "fp32"),
                    help="mfdimp_rgbt: ResNet-50 convs on fp32-faithful f16x3 split products (default) or fp32 MFMA")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the one-sequence / OSTrack-384 / mfDiMP samples the default 1-GPU line carries")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
    if args.batch is None:   # LasHeR's 245 test sequences over 8 GPUs (ViPT); over C5's 4 GPUs, 61
        args.batch = 32
    if args.dry:
        return dry_main(args, rank, world, dist)
    extras = None
    if (world == 1 and "WORLD_SIZE" not in os.environ and not args.no_extras and args.workload == "vipt_deep_rgbt"
            and args.batch == 32 and args.precision == "fp32"):
        extras = run_extras()   # children first: this process has not touched the GPU yet
    torch.cuda.set_device(local)
    if args.workload == DIMP_WORKLOAD:
        return dimp_main(args, rank, world, dist)

    from mmtrack_amd import Engine, EngineConfig, synth
    ekw, skw, H, W, C, desc = WORKLOADS[args.workload]
    B = args.batch
    cfg = EngineConfig(max_batch=B, use_graphs=not args.no_graphs, precision=args.precision, **ekw)
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

    def step(k, lists=frame_lists):
        eng.track_batch(0, lists[k % args.frames])

    def run(k0, count, lists=frame_lists):
        """`count` frames of every sequence.  Pipelined (default): the tracker state lives on the device,
        so frame k+1 is submitted before frame k's boxes are fetched (at most LAG frames in flight);
        every frame's boxes reach the host before this returns.  --sync: one blocking call per frame."""
        if args.sync:
            for k in range(k0, k0 + count):
                step(k, lists)
            return
        pend = collections.deque()
        for k in range(k0, k0 + count):
            pend.append(eng.track_batch_submit(0, lists[k % args.frames]))
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
    value, elapsed, world = aggregate_throughput(B, args.steps, t1 - t0)

    # PCIe-inclusive rate: the same steps with every frame handed over as a host array in pinned memory
    # (the reference's per-frame call receives a host np.ndarray); copies run on the engine's copy stream
    host_fps = None
    if args.host_frames > 0:
        pinned = [torch.from_numpy(video_np[1 + t]).pin_memory().numpy() for t in range(args.frames)]
        host_lists = [[pinned[t]] * B for t in range(args.frames)]
        run(0, 2, host_lists)
        torch.cuda.synchronize()
        th = time.perf_counter()
        run(0, args.host_frames, host_lists)
        torch.cuda.synchronize()
        host_fps = B * args.host_frames / (time.perf_counter() - th)

    roof = None
    if args.probe and args.probe != "none":
        classes = probe_classes(eng, step, args.warmup, min(args.steps, 10), args.precision)
        roof = roofline_from(classes, args.precision, args.workload, B)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.workload, video_np, gts, args.cpu_seconds)
        gf = GFLOP_PER_FRAME[args.workload]
        line = {
            "metric": METRIC,
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "f16x3" if args.precision == "fp32" else "bf16", "data": "synthetic",
            "config": {"workload": args.workload, "description": desc, "sequences_per_gpu": B,
                       "global_batch": B * world, "frame": f"{W}x{H}x{C} uint8 (HBM-resident)",
                       "template": cfg.template_size, "search": cfg.search_size, "parallelism": f"seq-shard x{world}",
                       "precision": args.precision, "parity_mode": args.precision == "fp32",
                       "graphs": cfg.use_graphs, "pipelined_frames": 0 if args.sync else LAG,
                       "weights": "synthetic seeded (no checkpoint ships)"},
            "per_gpu_fps": round(value / world, 2),
            "host_frames_fps_rank0": round(host_fps, 2) if host_fps else None,
            "model_tflops": round(value * gf / 1e3, 1),
            "roofline": roof,
            # the whole timed step (graph replays, halves on) against the same dense peak: algorithmic
            # FLOPs of every kernel of the step / ms_per_step, per GPU
            "step_frac_of_peak": round(value / world * gf / 1e3 / (PEAK_BF16_TFLOPS / (3 if args.precision == "fp32"
                                                                                         else 1)), 4),
            "cpu_baseline": cpu,
        }
        if extras is not None:
            line["extra_workloads"] = extras
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


def dimp_main(args, rank, world, dist):
    """C5: DeT/mfDiMP DiMP-50 tracking of B synthetic RGB-T sequences per GPU (mmtrack_amd.dimp_tracker):
    a step = one frame of every sequence (patch sampling, two ResNet-50 backbones + clf features for the
    batch, grouped filter application, per-sequence localisation / memory / Gauss-Newton updates)."""
    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, parameters, track_batch
    from mmtrack_amd.dimpnet import DiMPNet
    B, H, W, C = args.batch, 480, 640, 6
    sd = synth.make_dimp_state_dict(0)
    net = DiMPNet(sd, precision=args.dimp_precision)
    video_np, gts = synth.make_frames(1000 + rank, args.frames + 1, H, W, C)
    video = torch.from_numpy(video_np).cuda()
    pool = DimpPool(net, B, parameters())   # the trackers' device-resident state, one slot each
    trackers = [DiMP(parameters(), net=net, pool=pool) for _ in range(B)]
    torch.manual_seed(rank)
    for i, t in enumerate(trackers):
        t.initialize(video[0], {"init_bbox": [60.0 + (37 * i) % (W - 160), 40.0 + (23 * i) % (H - 120),
                                               40.0 + (i % 5) * 6, 32.0 + (i % 3) * 8]})
    torch.cuda.synchronize()

    from mmtrack_amd.dimp_tracker import PipelinedBatch
    pipe = PipelinedBatch(trackers, groups=args.dimp_groups) if not args.sync else None

    def run(k0, n):
        """n frames of every sequence, all results on the host before returning (--sync: track_batch per
        frame; default: PipelinedBatch over --dimp-groups groups of sequences -- with 2, the host updates of
        one group run under the other's network; 1, the whole batch per launch, is faster on MI355X since the
        grouped split-K convs want the larger M)."""
        for k in range(k0, k0 + n):
            frames = [video[1 + k % args.frames]] * B
            if pipe is None:
                track_batch(trackers, frames)
            else:
                pipe.step(frames)
        if pipe is not None:
            pipe.flush()

    run(0, max(args.warmup, 2))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    value, elapsed, world = aggregate_throughput(B, args.steps, t1 - t0)
    # roofline: the feature net (fp32 MFMA convs, >99 % of the step's FLOPs) timed with HIP events on the
    # stream its kernels run on (torch's current stream)
    patches = torch.rand(B, 6, 288, 288, device="cuda") * 255
    net.extract_classification_feat(net.extract_backbone(patches))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    ev0.record()
    for _ in range(reps):
        net.extract_classification_feat(net.extract_backbone(patches))
    ev1.record()
    torch.cuda.synchronize()
    feat_ms = ev0.elapsed_time(ev1) / reps
    flops = net.flops() * B
    achieved = flops / (feat_ms * 1e-3) / 1e12
    f16 = args.dimp_precision == "f16x3"
    peak = PEAK_BF16_TFLOPS / 3 if f16 else PEAK_FP32_MATRIX_TFLOPS
    tr = dimp_traffic(B) if f16 else None
    roof = {"bound": "mfma", "kernel": ("f16x3 convs: conv_f16x3_deep_kernel, conv3x3_patch_f16x3_kernel, "
                                        "conv_stem_pool_f16x3_kernel" if f16 else "conv_f32_kernel") +
            " (2 x ResNet-50 to layer3 + clf conv, per batch)",
            "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": None,
            # no PMC pass runs inside bench.py: the committed summary's figure, named as such
            "traffic_committed": tr,
            "traffic_unit": "bytes per 32-image feature-net batch (FETCH_SIZE x2 + WRITE_SIZE, PMC)",
            "flop_per_launch_group": flops, "avg_batch_ms": round(feat_ms, 4),
            # the feature net is partly HBM-bound (fp32 activations, 1x1 convs of K = 64..256): its per-layer
            # roofline (sum over layers of max(FLOPs / peak, min bytes / 8 TB/s)) and the fraction of it reached
            "layer_roofline_ms": round(net.roofline_ms(B, peak, PEAK_HBM_GBS / 1e3), 4),
            "frac_of_layer_roofline": round(net.roofline_ms(B, peak, PEAK_HBM_GBS / 1e3) / feat_ms, 4),
            "peak_note": ("f16x3 split products (Wh*Ah + Wl*Ah + Wh*Al, fp16 MFMA at the bf16 rate): dense 2500 TF/s / 3 "
                          "of algorithmic FLOPs, fp32-faithful (the reference runs fp32)") if f16 else
                         "dense fp32 matrix (v_mfma_f32_16x16x4_f32): the DiMP path runs at the reference's fp32"}
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            from oracle import dimp as od
            from oracle import dimpnet as odn
            torch.set_num_threads(cpu_quota())
            im = torch.rand(1, 6, 288, 288) * 255
            filt = torch.randn(1, 512, 4, 4) * 0.01
            n, tc = 0, time.perf_counter()
            with torch.no_grad():
                while time.perf_counter() - tc < args.cpu_seconds or n == 0:
                    f = odn.clf_features(odn.backbone(odn.preprocess(im), sd), sd)
                    od.apply_filter(f.unsqueeze(1), filt)
                    n += 1
            dt = time.perf_counter() - tc
            cpu = {"value": round(n / dt, 3), "unit": "frames/s", "cores": cpu_quota(), "kind": "port",
                   "sample": f"{n} frames of the fp32 CPU oracle DiMP-50 feature net + classifier "
                             f"(oracle/dimpnet.py, {cpu_quota()} threads, {dt:.1f} s)"}
        line = {"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f16x3" if f16 else "f32", "data": "synthetic",
                "config": {"workload": DIMP_WORKLOAD, "description": "mfDiMP RGB-T (DeT DiMP-50, merge max): "
                           "ResNet-50 x2 features + DiMP online optimiser (BASELINE configs[4])",
                           "sequences_per_gpu": B, "global_batch": B * world, "frame": f"{W}x{H}x{C} uint8 (HBM)",
                           "image_sample_size": 288, "parallelism": f"seq-shard x{world}",
                           "conv_precision": args.dimp_precision, "iou_net": "off (fixed-size boxes, as the golden)",
                           "weights": "synthetic seeded (no checkpoint ships)"},
                "per_gpu_fps": round(value / world, 2), "model_tflops": round(value * net.flops() / 1e12, 2),
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def dry_main(args, rank, world, dist):
    """The multi-rank plumbing without a GPU: each 'step' sleeps 1 ms per sequence."""
    def run(n):
        for _ in range(n):
            time.sleep(1e-3 * args.batch / 32)
    run(args.warmup)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.steps)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    value, elapsed, w = aggregate_throughput(args.batch, args.steps, t1 - t0)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": w,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "dry": True,
                          "per_gpu_fps": round(value / w, 2),
                          "config": {"sequences_per_gpu": args.batch, "global_batch": args.batch * w}}), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
