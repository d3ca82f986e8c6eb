"""mfDiMP classifier inner loop on RGB-T features (the RGBT/benchmark.py 'mfDiMP' entry).

The reference's mfDiMP source is an empty submodule (RGBT/models/end2end_rgbt_tracking/); what this
build provides is DiMP's target-classifier optimiser (DeT's ltr filter.py / optimizer.py restated as
HIP, mmtrack_amd.dimp). This driver times that inner loop at the DiMP tracker's shapes
(pytracking/parameter/dimp/DeT_DiMP50_Max.py:10-28: 512-d clf features, 18x18 at 288^2 input,
4x4 filter, sample memory 50, net_opt_iter 10 at init / 2 per update), with seeded fused RGB-T
features standing in for the ResNet-50 layer3 + clf-feature extractor (not built this round).
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.normpath(os.path.join(HERE, "..", "..", "..")))


def main(argv=None):
    import torch
    from mmtrack_amd.dimp import DiMPSteepestDescentGN, apply_filter
    ap = argparse.ArgumentParser()
    ap.add_argument("--sequences", type=int, default=8, help="sequences optimised together (S)")
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--memory", type=int, default=50)
    args = ap.parse_args(argv)
    g = torch.Generator().manual_seed(0)
    S, C, H, W = args.sequences, 512, 18, 18
    sd = {"log_step_length": torch.tensor([0.0]), "filter_reg": torch.tensor([0.1]),
          "label_map_predictor.weight": torch.linspace(1.0, -0.2, 10).view(1, 10, 1, 1),
          "target_mask_predictor.0.weight": torch.linspace(3.0, -3.0, 10).view(1, 10, 1, 1),
          "spatial_weight_predictor.weight": torch.ones(1, 10, 1, 1)}
    opt = DiMPSteepestDescentGN(sd, num_iter=2)
    dev = torch.device("cuda")
    feat = (torch.randn(args.memory, S, C, H, W, generator=g) * 0.3).to(dev)
    bb = torch.tensor([[[128.0, 128.0, 40.0, 30.0]] * S] * args.memory)
    w = torch.zeros(S, C, 4, 4, device=dev)
    w = opt.optimize(w, feat[:15], bb[:15], num_iter=10)          # initial filter (15 augmented samples)
    torch.cuda.synchronize()
    t0 = time.time()
    for f in range(1, args.frames):
        test = feat[f % args.memory].unsqueeze(0)
        scores = apply_filter(test, w)                           # classify the new frame
        w = opt.optimize(w, feat, bb, num_iter=2)                 # update_classifier
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"mfDiMP classifier: {S} sequences x {args.frames - 1} frames in {dt:.3f}s -> "
          f"{S * (args.frames - 1) / dt:.1f} frame-updates/s (scores {tuple(scores.shape)})")


if __name__ == "__main__":
    main()
