"""Bitwise comparison of two builds of libmmtrack.so on the tracking path (GPU tuning tool, not a test): each build
tracks the same synthetic sequences for some frames in its own child process (MMTRACK_LIB selects the build) and
the boxes and scores of every frame are compared bit for bit -- for a change meant to keep the arithmetic.
usage: python tools/lib_bitwise.py <libA.so> <libB.so> [batch] [frames] [workload]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child_dimp(out, batch, frames):
    """mfdimp_rgbt: bench.py's DiMP trackers (synthetic weights and frames), track_batch per frame; boxes and
    confidences of every frame"""
    import numpy as np
    import torch

    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, parameters, track_batch
    from mmtrack_amd.dimpnet import DiMPNet
    H, W, C = 480, 640, 6
    net = DiMPNet(synth.make_dimp_state_dict(0), precision="f16x3")
    video_np, _ = synth.make_frames(1000, frames + 1, H, W, C)
    video = torch.from_numpy(video_np).cuda()
    pool = DimpPool(net, batch, parameters())
    trackers = [DiMP(parameters(), net=net, pool=pool) for _ in range(batch)]
    torch.manual_seed(0)
    for i, t in enumerate(trackers):
        t.initialize(video[0], {"init_bbox": [60.0 + (37 * i) % (W - 160), 40.0 + (23 * i) % (H - 120),
                                               40.0 + (i % 5) * 6, 32.0 + (i % 3) * 8]})
    boxes, scores = [], []
    for t in range(frames):
        outs = track_batch(trackers, [video[1 + t]] * batch)
        boxes.append([o["target_bbox"] for o in outs])
        scores.append([o["confidence"] for o in outs])
    np.savez(out, boxes=np.array(boxes, dtype=np.float64), scores=np.array(scores, dtype=np.float64))


def child(out, batch, frames, workload):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "multi-modal-trakcing-bechmark_amd"))
    import numpy as np
    import torch
    if workload == "mfdimp_rgbt":
        return child_dimp(out, batch, frames)

    import bench
    from mmtrack_amd import Engine, EngineConfig, synth
    ekw, skw, H, W, C, _ = bench.WORKLOADS[workload]
    eng = Engine(EngineConfig(max_batch=batch, use_graphs=True, precision="fp32", **ekw),
                 synth.make_state_dict(0, **skw), device=0)
    video_np, _ = synth.make_frames(1000, frames + 1, H, W, C)
    video = torch.from_numpy(video_np).cuda()
    for i in range(batch):
        eng.initialize(i, video[0], [60.0 + (37 * i) % (W - 160), 40.0 + (23 * i) % (H - 120), 30.0 + (i % 5) * 6,
                                     24.0 + (i % 3) * 8])
    boxes, scores = [], []
    for t in range(frames):
        bx, sc = eng.track_batch(0, [video[1 + t]] * batch)
        boxes.append(bx)
        scores.append(sc.astype(np.float64))
    np.savez(out, boxes=np.array(boxes, dtype=np.float64), scores=np.array(scores, dtype=np.float64))


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    import numpy as np
    a, b = sys.argv[1], sys.argv[2]
    batch = sys.argv[3] if len(sys.argv) > 3 else "32"
    frames = sys.argv[4] if len(sys.argv) > 4 else "20"
    workload = sys.argv[5] if len(sys.argv) > 5 else "vipt_deep_rgbt"
    res = []
    with tempfile.TemporaryDirectory() as d:
        for i, lib in enumerate((a, b)):
            out = os.path.join(d, f"{i}.npz")
            env = dict(os.environ, MMTRACK_LIB=os.path.abspath(lib))
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", out, batch, frames, workload],
                           env=env, check=True)
            res.append(np.load(out))
    same = all(np.array_equal(res[0][k].view(np.uint64), res[1][k].view(np.uint64)) for k in ("boxes", "scores"))
    dmax = float(np.abs(res[0]["scores"] - res[1]["scores"]).max())
    print(f"{workload} batch {batch} x {frames} frames: bitwise {'IDENTICAL' if same else 'DIFFERENT'} "
          f"(max |d score| {dmax:.3e})")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
