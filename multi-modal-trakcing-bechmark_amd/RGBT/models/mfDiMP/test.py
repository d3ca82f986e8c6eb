"""mfDiMP RGB-T tracking (the RGBT/benchmark.py 'mfDiMP' entry) on the MI355X path.

The reference's mfDiMP source is an empty submodule (RGBT/models/end2end_rgbt_tracking/); the in-tree
multi-modal DiMP is DeT's DiMP-50 (two ResNet-50 backbones, 'max' feature merge, DiMP classifier), which
this build runs as HIP kernels (mmtrack_amd.dimpnet / dimp / dimp_tracker).  This driver tracks seeded
synthetic RGB-T sequences -- or a LasHeR / RGBT234 / GTOT folder with --seq_home and a checkpoint
(--net_path; --synthetic_weights runs the seeded network there, into a separately named result folder) -- one sequence per
tracker, several sequences per GPU per launch (dimp_tracker.track_batch), sequences sharded over ranks
(torchrun: sequence i on rank i % world, no collective), and writes one result file per sequence in the
RGB-T workspace format (np.savetxt, test_rgbt_mgpus.py:116).

    python RGBT/models/mfDiMP/test.py --synthetic 8 --frames 100 --batch 8
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 RGBT/models/mfDiMP/test.py --synthetic 32
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PRJ = os.path.normpath(os.path.join(HERE, "..", "..", ".."))
sys.path.insert(0, PRJ)


def main(argv=None):
    import numpy as np
    import torch

    from mmtrack_amd import synth
    from mmtrack_amd.dimp_tracker import DiMP, DimpPool, parameters, track_batch
    from mmtrack_amd.dimpnet import DiMPNet
    from mmtrack_amd.sharding import rank_world, shard_indices
    from mmtrack_amd.workspace import frame_getter, gen_config, sequence_list
    ap = argparse.ArgumentParser()
    ap.add_argument("--synthetic", type=int, default=8, help="seeded synthetic sequences (0: use --seq_home)")
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--seq_home", default="")
    ap.add_argument("--dataset_name", default="LasHeR")
    ap.add_argument("--batch", type=int, default=8, help="sequences tracked per launch")
    ap.add_argument("--out_root", default=".")
    ap.add_argument("--net_path", default="", help="DiMPnet_DeT checkpoint (a state_dict, or pytracking's "
                    "{'net': state_dict}), loaded with torch.load(weights_only=True)")
    ap.add_argument("--synthetic_weights", action="store_true",
                    help="seeded synthetic weights on a --seq_home dataset (results land in mfDiMP_synthetic_weights)")
    args = ap.parse_args(argv)
    if not args.synthetic and not args.net_path and not args.synthetic_weights:
        # random weights would produce result files that look like real benchmark outputs
        raise SystemExit("--seq_home needs real weights (--net_path); pass --synthetic_weights to run the "
                         "seeded synthetic network on it anyway")
    rank, world = rank_world()
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
    if args.synthetic:
        seqs = []
        for i in range(args.synthetic):
            box = (150.0 + 31 * (i % 9), 100.0 + 17 * (i % 7), 40.0 + 4 * (i % 5), 32.0 + 3 * (i % 4))
            fr, gt = synth.make_frames(i, args.frames, 480, 640, 6, box=box)
            seqs.append((f"synthetic_{i:03d}", len(fr), (lambda f: (lambda k: f[k]))(fr), gt))
    else:
        seqs = []
        for name in sequence_list(args.seq_home, args.dataset_name):
            rgb, aux, gt = gen_config(os.path.join(args.seq_home, name), args.dataset_name)
            seqs.append((name, len(rgb), frame_getter(rgb, aux, 'rgbrgb'), gt))
    mine = [seqs[i] for i in shard_indices(len(seqs), rank, world)]
    if args.net_path:
        ck = torch.load(args.net_path, map_location="cpu", weights_only=True)
        net = DiMPNet(ck["net"] if isinstance(ck, dict) and "net" in ck else ck)
        tag = "mfDiMP"
    else:
        net = DiMPNet(synth.make_dimp_state_dict(0))
        tag = "mfDiMP" if args.synthetic else "mfDiMP_synthetic_weights"
    out_dir = os.path.join(args.out_root, "RGBT_workspace", "results", args.dataset_name, tag)
    os.makedirs(out_dir, exist_ok=True)
    t0, tracked = time.perf_counter(), 0
    for b0 in range(0, len(mine), args.batch):
        group = mine[b0:b0 + args.batch]
        pool = DimpPool(net, len(group), parameters())
        trackers = [DiMP(parameters(), net=net, pool=pool) for _ in group]
        results = [np.zeros((n, 4)) for _, n, _, _ in group]
        for tr, (name, n, get, gt), res in zip(trackers, group, results):
            tr.initialize(get(0), {"init_bbox": list(np.asarray(gt[0], dtype=np.float64))})
            res[0] = gt[0]
        for k in range(1, max(n for _, n, _, _ in group)):
            live = [i for i, (_, n, _, _) in enumerate(group) if k < n]
            outs = track_batch([trackers[i] for i in live], [group[i][2](k) for i in live])
            for i, o in zip(live, outs):
                results[i][k] = o["target_bbox"]
            tracked += len(live)
        for (name, _, _, _), res in zip(group, results):
            np.savetxt(os.path.join(out_dir, name + ".txt"), res)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"mfDiMP rank {rank}/{world}: {len(mine)} sequences, {tracked} tracked frames in {dt:.2f}s -> "
          f"{tracked / max(dt, 1e-9):.1f} frames/s (init included)")


if __name__ == "__main__":
    main()
