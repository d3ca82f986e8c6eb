"""CPU restatement of the DiMP tracker's per-frame decisions (TEST ORACLE; imported only by tests/).

The step the device state machine (csrc/dimptrack.hip dimp_localize_kernel) runs per frame, restated from DeT's
pytracking tracker (RGBD/models/DeT/pytracking/tracker/dimp/dimp.py) with the DeT_DiMP50_Max parameters and
use_iou_net = False:
* ``get_sample_location``      dimp.py:179-184
* ``localize_advanced``        dimp.py:239-302 (one scale, no output window)
* ``update_state``             dimp.py:488-497
* ``update_classifier``        dimp.py:607-625 (the memory update and the Gauss-Newton iteration count)
* ``update_memory``            dimp.py:432-444, ``update_sample_weights`` dimp.py:447-486
in torch float32 where the reference computes on tensors and Python doubles where it calls .item() or
compares Python floats.  Pinned by the decision records of tests/golden/tracker_dimp_branches.npz (the reference's
state before every frame, the score map it localised on and its state after it; make_golden_dimp.py).
"""
import math

import torch

FLAGS = ("normal", "not_found", "uncertain", "hard_negative")


def _max2d(a):
    """dcf.max2d on one [H, W] map: the maximum and its (row, col), first index on ties (torch.max)."""
    v, i = torch.max(a.reshape(-1), dim=0)
    return v, torch.tensor([int(i) // a.shape[-1], int(i) % a.shape[-1]])


def update_sample_weights(sw, prev_ind, num_samp, num_init, lr, init_min_weight):
    """dimp.py:447-486 on one memory's weights (in place); returns the replaced index."""
    init_w = None if init_min_weight == 0 else init_min_weight
    s_ind = 0 if init_w is None else num_init
    if num_samp == 0 or lr == 1:
        sw[:] = 0
        sw[0] = 1
        r_ind = 0
    else:
        if num_samp < sw.shape[0]:
            r_ind = num_samp
        else:
            _, r = torch.min(sw[s_ind:], 0)
            r_ind = int(r) + s_ind
        if prev_ind is None:
            sw /= 1 - lr
            sw[r_ind] = lr
        else:
            sw[r_ind] = sw[prev_ind] / (1 - lr)
    sw /= sw.sum()
    if init_w is not None and sw[:num_init].sum() < init_w:
        sw /= init_w + sw[num_init:].sum()
        sw[:num_init] = init_w / num_init
    return r_ind


def decide(st, scores, coords, p, img_sample_sz=(288.0, 288.0), kernel_size=(4.0, 4.0)):
    """One frame's decisions.  st: dict with pos, target_sz, base_target_sz, image_sz (float32 [2] tensors),
    target_scale, min_scale_factor, max_scale_factor (float32 scalars), frame_num, num_init, num_stored,
    prev_replace (None or int), sample_weights ([50] float32), target_boxes ([50, 4] float32) -- updated in place;
    scores: the raw [H, W] score map; coords: the sample's [4] coordinates; p: the tracker parameters (an object
    with the DeT_DiMP50_Max attributes).  Returns (flag, num_iter, replace_ind or -1, output box [4])."""
    g = lambda name, default=None: getattr(p, name, default)
    img_sample_sz = torch.tensor(img_sample_sz)
    kernel_size = torch.tensor(kernel_size)
    st["frame_num"] += 1
    # get_sample_location
    sc = coords.float().view(1, 4)
    sample_pos = 0.5 * (sc[:, :2] + sc[:, 2:] - 1)
    sample_scales = ((sc[:, 2:] - sc[:, :2]) / img_sample_sz).prod(dim=1).sqrt()
    # localize_advanced (one scale)
    sz = scores.shape[-2:]
    score_sz = torch.Tensor(list(sz))
    output_sz = score_sz - (kernel_size + 1) % 2
    score_center = (score_sz - 1) / 2
    max_score1, max_disp1 = _max2d(scores)
    sample_scale = sample_scales[0]
    max_disp1 = max_disp1.float()
    target_disp1 = max_disp1 - score_center
    tv1 = target_disp1 * (img_sample_sz / output_sz) * sample_scale
    tv, flag = tv1, None
    if max_score1.item() < g("target_not_found_threshold"):
        flag = "not_found"
    elif max_score1.item() < g("uncertain_threshold", -float("inf")):
        flag = "uncertain"
    elif max_score1.item() < g("hard_sample_threshold", -float("inf")):
        flag = "hard_negative"
    else:
        tns = g("target_neighborhood_scale") * (st["target_sz"] / sample_scale) * (output_sz / img_sample_sz)
        top = max(round(max_disp1[0].item() - tns[0].item() / 2), 0)
        bottom = min(round(max_disp1[0].item() + tns[0].item() / 2 + 1), sz[0])
        left = max(round(max_disp1[1].item() - tns[1].item() / 2), 0)
        right = min(round(max_disp1[1].item() + tns[1].item() / 2 + 1), sz[1])
        masked = scores.clone()
        masked[top:bottom, left:right] = 0
        max_score2, max_disp2 = _max2d(masked)
        target_disp2 = max_disp2.float() - score_center
        tv2 = target_disp2 * (img_sample_sz / output_sz) * sample_scale
        prev_vec = (st["pos"] - sample_pos[0]) / ((img_sample_sz / output_sz) * sample_scale)
        if max_score2 > g("distractor_threshold") * max_score1:
            n1 = torch.sqrt(torch.sum((target_disp1 - prev_vec) ** 2))
            n2 = torch.sqrt(torch.sum((target_disp2 - prev_vec) ** 2))
            thr = g("dispalcement_scale") * math.sqrt(sz[0] * sz[1]) / 2
            if n2 > thr and n1 < thr:
                flag = "hard_negative"
            elif n2 < thr and n1 > thr:
                flag, tv = "hard_negative", tv2
            else:
                flag = "uncertain"
        elif max_score2 > g("hard_negative_threshold") * max_score1 and max_score2 > g("target_not_found_threshold"):
            flag = "hard_negative"
        else:
            flag = "normal"
    new_pos = sample_pos[0] + tv
    # update_state (use_iou_net False: the sample scale becomes the target scale)
    if flag != "not_found":
        st["target_scale"] = sample_scales[0].clamp(st["min_scale_factor"], st["max_scale_factor"])
        st["target_sz"] = st["base_target_sz"] * st["target_scale"]
        off = (g("target_inside_ratio", 0.2) - 0.5) * st["target_sz"]
        st["pos"] = torch.max(torch.min(new_pos, st["image_sz"] - off), off)
    # update_classifier: memory and iteration count
    num_iter, r_ind = 0, -1
    if flag not in ("not_found", "uncertain") and g("update_classifier", False):
        hard = flag == "hard_negative"
        lr = g("hard_negative_learning_rate") if hard else g("learning_rate")
        box_center = (st["pos"] - sample_pos[0]) / sample_scales[0] + (img_sample_sz - 1) / 2
        box_sz = st["target_sz"] / sample_scales[0]
        target_ul = box_center - (box_sz - 1) / 2
        target_box = torch.cat([target_ul.flip((0,)), box_sz.flip((0,))])
        if hard or st["frame_num"] % g("train_sample_interval", 1) == 0:
            r_ind = update_sample_weights(st["sample_weights"], st["prev_replace"], st["num_stored"], st["num_init"], lr,
                                          g("init_samples_minimum_weight", None) or 0)
            st["prev_replace"] = r_ind
            st["target_boxes"][r_ind, :] = target_box
            st["num_stored"] += 1
        low = g("low_score_opt_threshold", None)
        if hard:
            num_iter = g("net_opt_hn_iter", None)
        elif low is not None and low > scores.max().item():
            num_iter = g("net_opt_low_iter", None)
        elif (st["frame_num"] - 1) % g("train_skipping") == 0:
            num_iter = g("net_opt_update_iter", None)
    box = torch.cat((st["pos"][[1, 0]] - (st["target_sz"][[1, 0]] - 1) / 2, st["target_sz"][[1, 0]]))
    return flag, int(num_iter or 0), r_ind, box
