"""CPU restatement of the DiMP target-classifier inner loop (TEST ORACLE).

mfDiMP's own source is absent (RGBT/models/end2end_rgbt_tracking/ is an empty un-vendored
submodule); its classifier is DiMP's, whose in-tree copy is DeT's:
* ``apply_filter``            RGBD/models/DeT/ltr/models/layers/filter.py:5-54
* ``apply_feat_transpose``    filter.py:57-148 (the filter gradient of apply_filter)
* ``DistanceMap``             ltr/models/layers/distance.py:6-39
* ``LeakyReluPar(+Deriv)``    ltr/models/layers/activation.py:32-44
* ``DiMPSteepestDescentGN``   ltr/models/target_classifier/optimizer.py:85-170
Pinned by tests/golden/dimp.npz (produced by importing the DeT code itself).
"""
import math

import torch
import torch.nn.functional as F


def apply_filter(feat, filt):
    """feat [I, S, C, H, W], filt [S, C, fh, fw] -> scores [I, S, Ho, Wo] (pad fh//2, groups = S)."""
    I, S = feat.shape[0], feat.shape[1]
    pad = (filt.shape[-2] // 2, filt.shape[-1] // 2)
    sc = F.conv2d(feat.reshape(I, -1, feat.shape[-2], feat.shape[-1]), filt, padding=pad, groups=S)
    return sc.view(I, S, sc.shape[-2], sc.shape[-1])


def apply_feat_transpose(feat, inp, filter_ksz):
    """d/dw of sum(inp * apply_filter(feat, w)) (filter.py:95-121, v2 path) -> [S, C, fh, fw]."""
    I, S = feat.shape[0], feat.shape[1]
    trans_pad = [(k - 1) // 2 for k in filter_ksz]
    g = F.conv2d(inp.reshape(1, -1, inp.shape[-2], inp.shape[-1]),
                 feat.reshape(-1, 1, feat.shape[-2], feat.shape[-1]), padding=trans_pad, groups=I * S)
    return g.view(I, S, -1, g.shape[-2], g.shape[-1]).sum(dim=0).flip((2, 3))


def distance_map(center, output_sz, num_bins, bin_displacement):
    """distance.py:17-39."""
    center = center.view(-1, 2)
    bin_centers = torch.arange(num_bins, dtype=torch.float32).view(1, -1, 1, 1)
    k0 = torch.arange(output_sz[0], dtype=torch.float32).view(1, 1, -1, 1)
    k1 = torch.arange(output_sz[1], dtype=torch.float32).view(1, 1, 1, -1)
    d0 = k0 - center[:, 0].view(-1, 1, 1, 1)
    d1 = k1 - center[:, 1].view(-1, 1, 1, 1)
    dist = torch.sqrt(d0 * d0 + d1 * d1)
    bin_diff = dist / bin_displacement - bin_centers
    return torch.cat((F.relu(1.0 - torch.abs(bin_diff[:, :-1])), (1.0 + bin_diff[:, -1:]).clamp(0, 1)), dim=1)


def steepest_descent_gn(weights, feat, bb, sd, num_iter, feat_stride=16, min_filter_reg=1e-3, alpha_eps=0.0,
                        num_dist_bins=10, bin_displacement=0.5, sample_weight=None):
    """DiMPSteepestDescentGN.forward (optimizer.py:85-170), relu score activation, sigmoid mask.
    sd: the optimizer's state_dict tensors (log_step_length, filter_reg, *_predictor weights)."""
    num_images, num_sequences = feat.shape[0], feat.shape[1]
    filter_sz = (weights.shape[-2], weights.shape[-1])
    output_sz = (feat.shape[-2] + (weights.shape[-2] + 1) % 2, feat.shape[-1] + (weights.shape[-1] + 1) % 2)
    step_length_factor = torch.exp(sd["log_step_length"])
    reg_weight = (sd["filter_reg"] * sd["filter_reg"]).clamp(min=min_filter_reg ** 2)
    dmap_offset = (torch.Tensor(filter_sz) % 2) / 2.0
    center = ((bb[..., :2] + bb[..., 2:] / 2) / feat_stride).reshape(-1, 2).flip((1,)) - dmap_offset
    dist_map = distance_map(center, output_sz, num_dist_bins, bin_displacement)
    label_map = F.conv2d(dist_map, sd["label_map_predictor.weight"]).reshape(num_images, num_sequences, *output_sz)
    target_mask = torch.sigmoid(F.conv2d(dist_map, sd["target_mask_predictor.0.weight"])).reshape(
        num_images, num_sequences, *output_sz)
    spatial_weight = F.conv2d(dist_map, sd["spatial_weight_predictor.weight"]).reshape(
        num_images, num_sequences, *output_sz)
    if sample_weight is None:
        sample_weight = math.sqrt(1.0 / num_images) * spatial_weight
    else:
        sample_weight = sample_weight.sqrt().reshape(num_images, num_sequences, 1, 1) * spatial_weight

    def act(x, a):
        return (1.0 - a) / 2.0 * torch.abs(x) + (1.0 + a) / 2.0 * x

    def dact(x, a):
        return (1.0 - a) / 2.0 * torch.sign(x) + (1.0 + a) / 2.0

    iterates, losses = [weights], []
    for _ in range(num_iter):
        scores = apply_filter(feat, weights)
        scores_act = act(scores, target_mask)
        score_mask = dact(scores, target_mask)
        residuals = sample_weight * (scores_act - label_map)
        losses.append(((residuals ** 2).sum() + reg_weight * (weights ** 2).sum()) / num_sequences)
        residuals_mapped = score_mask * (sample_weight * residuals)
        weights_grad = apply_feat_transpose(feat, residuals_mapped, filter_sz) + reg_weight * weights
        scores_grad = apply_filter(feat, weights_grad)
        scores_grad = sample_weight * (score_mask * scores_grad)
        alpha_num = (weights_grad * weights_grad).sum(dim=(1, 2, 3))
        alpha_den = ((scores_grad * scores_grad).reshape(num_images, num_sequences, -1).sum(dim=(0, 2))
                     + (reg_weight + alpha_eps) * alpha_num).clamp(1e-8)
        alpha = alpha_num / alpha_den
        weights = weights - (step_length_factor * alpha.reshape(-1, 1, 1, 1)) * weights_grad
        iterates.append(weights)
    scores = act(apply_filter(feat, weights), target_mask)
    losses.append((((sample_weight * (scores - label_map)) ** 2).sum() + reg_weight * (weights ** 2).sum())
                  / num_sequences)
    return weights, iterates, losses
