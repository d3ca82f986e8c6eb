"""SiamFC on RGB-E sequences (the command RGBE/benchmark.py dispatches: ``cd models/siamfc && python test.py``).

Tracks the RGB half of each sequence with mmtrack_amd.siamfc.TrackerSiamFC (HIP crop / xcorr / response
on the GPU) and writes one result file per sequence in the RGB-E format ('%.14f', comma-separated,
test_rgbe_mgpus.py:83). Without --seq_home it runs seeded synthetic sequences (BASELINE configs[0]:
one 100-frame sequence) with seeded AlexNet weights unless --net_path is given.
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.normpath(os.path.join(HERE, "..", "..", "..")))

import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--net_path", default=None)
    ap.add_argument("--seq_home", default="")
    ap.add_argument("--dataset_name", default="VisEvent")
    ap.add_argument("--synthetic", type=int, default=1)
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--out_root", default=os.path.join(HERE, "results"))
    args = ap.parse_args(argv)
    from mmtrack_amd import synth
    from mmtrack_amd.sharding import rank_world, shard_indices
    from mmtrack_amd.siamfc import TrackerSiamFC
    from mmtrack_amd.workspace import gen_config, save_result, synthetic_sequences
    sd = None if args.net_path else synth.make_siamfc_state_dict(0)
    tracker = TrackerSiamFC(net_path=args.net_path, state_dict=sd)
    if args.seq_home:
        from lib.train.dataset.depth_utils import get_x_frame
        names = sorted(d for d in os.listdir(args.seq_home) if os.path.isdir(os.path.join(args.seq_home, d)))
        seqs = []
        for nm in names:
            rgb, aux, gt = gen_config(os.path.join(args.seq_home, nm), args.dataset_name)
            seqs.append((nm, [get_x_frame(r, None, dtype="color") for r in rgb], gt))
    else:
        seqs = synthetic_sequences(args.synthetic, args.frames, C=3)
    rank, world = rank_world()
    os.makedirs(os.path.join(args.out_root, args.dataset_name, "siamfc"), exist_ok=True)
    total_frames, total_time = 0, 0.0
    for i in shard_indices(len(seqs), rank, world):
        name, frames, gt = seqs[i]
        t0 = time.time()
        boxes, times = tracker.track(frames, list(gt[0]))
        dt = time.time() - t0
        save_result(os.path.join(args.out_root, args.dataset_name, "siamfc", name + ".txt"), boxes, "rgbe")
        print(f"{name} , fps:{(len(frames) - 1) / max(times[1:].sum(), 1e-9):.1f}")
        total_frames += len(frames)
        total_time += dt
    print(f"siamfc: {total_frames} frames in {total_time:.2f}s")


if __name__ == "__main__":
    main()
