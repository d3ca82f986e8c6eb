"""mfDiMP / DeT-DiMP tracker on the MI355X path.

``DiMP`` keeps the reference tracker's contract and cadence (RGBD/models/DeT/pytracking/tracker/dimp/
dimp.py: ``initialize(image, info)`` :24-82, ``track(image)`` :85-166, advanced localisation :232-301,
init augmentation :322-385, classifier init / memory / update :399-504 and :538-607), restated over the
device path:

* patch sampling, init augmentations, the two ResNet-50 backbones + max merge, the clf features, the
  filter initialiser (PrRoIPool) run as HIP kernels (mmtrack_amd.dimpnet, csrc/dimpnet.hip);
* the steepest-descent Gauss-Newton filter optimiser and the classifier (apply_filter) run as HIP
  kernels (mmtrack_amd.dimp, csrc/dimp.hip);
* the host keeps the tracker's scalar state (position, scale, sample weights and boxes) in float32 CPU
  tensors with the reference's own arithmetic, and the 19 x 19 score map comes back once per frame.

IoU-Net box refinement (AtomIoUNet + PrRoIPool gradients, dimp.py:609-700) is not part of this path:
``parameters()`` sets ``use_iou_net = False``, the reference's switch for it (dimp.py:76-78, 123-130), so
position comes from the classifier and the size follows the sample scale.  Random init augmentation shifts
and the dropout masks draw from the host torch generator in the reference's order, so a seeded run matches
the reference run with the same seed.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from .dimp import DiMPSteepestDescentGN
from .dimpnet import DiMPNet, patch_transform_device, sample_patch_device


class TrackerParams:
    def get(self, name, *default):
        return getattr(self, name, default[0] if default else None)

    def has(self, name):
        return hasattr(self, name)


def parameters():
    """pytracking/parameter/dimp/DeT_DiMP50_Max.py:4-62 with use_iou_net = False (no IoU-Net refinement)."""
    p = TrackerParams()
    p.debug = 0
    p.visualization = False
    p.use_gpu = True
    p.image_sample_size = 18 * 16
    p.search_area_scale = 5
    p.sample_memory_size = 50
    p.learning_rate = 0.01
    p.init_samples_minimum_weight = 0.25
    p.train_skipping = 20
    p.update_classifier = True
    p.net_opt_iter = 10
    p.net_opt_update_iter = 2
    p.net_opt_hn_iter = 1
    p.window_output = False
    p.use_augmentation = True
    p.augmentation = {'fliplr': True, 'rotate': [10, -10, 45, -45], 'blur': [(3, 1), (1, 3), (2, 2)],
                      'relativeshift': [(0.6, 0.6), (-0.6, 0.6), (0.6, -0.6), (-0.6, -0.6)], 'dropout': (2, 0.2)}
    p.augmentation_expansion_factor = 2
    p.random_shift_factor = 1 / 3
    p.advanced_localization = True
    p.target_not_found_threshold = 0.25
    p.distractor_threshold = 0.8
    p.hard_negative_threshold = 0.5
    p.target_neighborhood_scale = 2.2
    p.dispalcement_scale = 0.8
    p.hard_negative_learning_rate = 0.02
    p.update_scale_when_uncertain = True
    p.merge_type = 'max'
    p.use_iou_net = False
    return p


# ---------------------------------------------------------------------------------------- init augmentations
def _crop_offsets(out_sz, in_sz, shift):
    """augmentation.py crop_to_output: (pad_top, pad_left)."""
    pad_h = (out_sz[0] - in_sz[0]) / 2
    pad_w = (out_sz[1] - in_sz[1]) / 2
    return math.floor(pad_h) + shift[0], math.floor(pad_w) + shift[1]


class _Tf:
    def __init__(self, kind, output_sz, shift=None, **kw):
        self.kind = kind
        self.output_sz = output_sz
        self.shift = (0, 0) if shift is None else tuple(shift)
        self.kw = kw

    def c_struct(self, in_sz):
        t = _lib.MmtPatchTf()
        t.kind = self.kind
        t.top, t.left = _crop_offsets(self.output_sz, in_sz, self.shift)
        if self.kind == 2:   # Blur (augmentation.py Blur.__init__: taps exp(-x^2 / 2 s^2), normalised)
            sig = self.kw['sigma']
            sig = (sig, sig) if isinstance(sig, (int, float)) else sig
            fsz = [math.ceil(2 * s) for s in sig]
            taps = []
            for sz, s in zip(fsz, sig):
                x = torch.arange(-sz, sz + 1, dtype=torch.float32)
                f = torch.exp(-(x ** 2) / (2 * s ** 2))
                taps.append(f / f.sum())
            t.blur_ry, t.blur_rx = fsz
            for i, v in enumerate(taps[0].tolist()):
                t.blur_fy[i] = v
            for i, v in enumerate(taps[1].tolist()):
                t.blur_fx[i] = v
        elif self.kind == 3:   # Rotate: H = [R | c - R c] (augmentation.py Rotate), inverted as cv2.warpAffine does
            a = math.pi * self.kw['angle'] / 180
            c = (np.array(in_sz, dtype=np.float64).reshape(2, 1) - 1) / 2
            R = np.array([[math.cos(a), math.sin(a)], [-math.sin(a), math.cos(a)]])
            M = np.concatenate([R, c - R @ c], 1).reshape(-1).tolist()
            D = M[0] * M[4] - M[1] * M[3]
            D = 1.0 / D if D != 0 else 0.0
            A11, A22 = M[4] * D, M[0] * D
            M[0], M[1], M[3], M[4] = A11, M[1] * -D, M[3] * -D, A22
            b1 = -M[0] * M[2] - M[1] * M[5]
            b2 = -M[3] * M[2] - M[4] * M[5]
            M[2], M[5] = b1, b2
            for i in range(6):
                t.affine[i] = M[i]
        return t


class DiMP:
    multiobj_mode = 'parallel'

    def __init__(self, params, state_dict=None, device=None, net=None):
        self.params = params
        if net is None:
            sd = state_dict if state_dict is not None else getattr(params, 'state_dict', None)
            if sd is None:
                raise ValueError("DiMP needs the network weights (params.state_dict or state_dict=)")
            net = DiMPNet(sd, device=device)
        self.net = net
        self.dev = self.net.dev
        self.optimizer = DiMPSteepestDescentGN(self.net.sd_opt, num_iter=5, feat_stride=16,
                                               num_dist_bins=self.net.sd_opt["label_map_predictor.weight"].numel(),
                                               bin_displacement=getattr(params, 'bin_displacement', 0.1))
        self.debug_info = {}

    # ------------------------------------------------------------------ image helpers
    def _frame(self, image):
        if isinstance(image, torch.Tensor):
            return image.to(self.dev).contiguous()
        return torch.from_numpy(np.ascontiguousarray(image)).to(self.dev)

    def _sample_patch(self, frame, pos, sample_sz, output_sz):
        """preprocessing.py sample_patch (mode 'replicate'): the integer geometry on the host with the
        reference's tensor arithmetic, the pixels on the device -> (patch [1, C, oh, ow], coord [1, 4])."""
        posl = pos.long().clone()
        resize_factor = torch.min(sample_sz.float() / output_sz.float()).item()
        df = int(max(int(resize_factor - 0.1), 1))
        sz = sample_sz.float() / df
        os_ = torch.zeros(2, dtype=torch.long)
        if df > 1:
            os_ = posl % df
            posl = (posl - os_) // df
        szl = torch.max(sz.round(), torch.Tensor([2])).long()
        tl = posl - (szl - 1) // 2
        br = posl + szl // 2 + 1
        geom = [df, int(os_[0]), int(os_[1]), int(tl[0]), int(tl[1]), int(szl[0]), int(szl[1])]
        patch = sample_patch_device(frame, geom, output_sz.long().tolist())
        return patch, df * torch.cat((tl, br)).view(1, 4)

    # ------------------------------------------------------------------ reference API
    def initialize(self, image, info: dict) -> dict:
        self.frame_num = 1
        frame = self._frame(image)
        state = info['init_bbox']
        self.pos = torch.Tensor([state[1] + (state[3] - 1) / 2, state[0] + (state[2] - 1) / 2])
        self.target_sz = torch.Tensor([state[3], state[2]])
        self.image_sz = torch.Tensor([frame.shape[0], frame.shape[1]])
        sz = self.params.image_sample_size
        sz = torch.Tensor([sz, sz] if isinstance(sz, int) else sz)
        self.img_sample_sz = sz
        self.img_support_sz = self.img_sample_sz
        search_area = torch.prod(self.target_sz * self.params.search_area_scale).item()
        self.target_scale = math.sqrt(search_area) / self.img_sample_sz.prod().sqrt()
        self.base_target_sz = self.target_sz / self.target_scale
        self.scale_factors = torch.ones(1)
        self.min_scale_factor = torch.max(10 / self.base_target_sz)
        self.max_scale_factor = torch.min(self.image_sz / self.base_target_sz)
        init_backbone_feat = self.generate_init_samples(frame)
        self.init_classifier(init_backbone_feat)
        return {}

    def generate_init_samples(self, frame):
        self.init_sample_scale = self.target_scale
        global_shift = torch.zeros(2)
        self.init_sample_pos = self.pos.round()
        aug_expansion_factor = self.params.get('augmentation_expansion_factor', None)
        aug_expansion_sz = self.img_sample_sz.clone()
        aug_output_sz = None
        if aug_expansion_factor is not None and aug_expansion_factor != 1:
            aug_expansion_sz = (self.img_sample_sz * aug_expansion_factor).long()
            aug_expansion_sz += (aug_expansion_sz - self.img_sample_sz.long()) % 2
            aug_expansion_sz = aug_expansion_sz.float()
            aug_output_sz = self.img_sample_sz.long().tolist()
        random_shift_factor = self.params.get('random_shift_factor', 0)

        def rand_shift():
            if random_shift_factor > 0:
                return ((torch.rand(2) - 0.5) * self.img_sample_sz * random_shift_factor + global_shift).long().tolist()
            return None
        out_sz = aug_output_sz if aug_output_sz is not None else self.img_sample_sz.long().tolist()
        gs = global_shift.long().tolist()
        self.transforms = [_Tf(0, out_sz, gs)]
        augs = self.params.augmentation if self.params.get('use_augmentation', True) else {}
        if 'shift' in augs:
            self.transforms.extend([_Tf(0, out_sz, (gs[0] + s[0], gs[1] + s[1])) for s in augs['shift']])
        if 'relativeshift' in augs:
            for s in augs['relativeshift']:
                a = (torch.Tensor(s) * self.img_sample_sz / 2).long().tolist()
                self.transforms.append(_Tf(0, out_sz, (gs[0] + a[0], gs[1] + a[1])))
        if 'fliplr' in augs and augs['fliplr']:
            self.transforms.append(_Tf(1, out_sz, rand_shift()))
        if 'blur' in augs:
            self.transforms.extend([_Tf(2, out_sz, rand_shift(), sigma=s) for s in augs['blur']])
        if 'scale' in augs:
            raise NotImplementedError("the 'scale' init augmentation is not used by the DiMP-50 settings")
        if 'rotate' in augs:
            self.transforms.extend([_Tf(3, out_sz, rand_shift(), angle=a) for a in augs['rotate']])
        patch, _ = self._sample_patch(frame, self.init_sample_pos, self.init_sample_scale * aug_expansion_sz,
                                      aug_expansion_sz)
        in_sz = (patch.shape[2], patch.shape[3])
        patches = torch.cat([patch_transform_device(patch, T.c_struct(in_sz), out_sz) for T in self.transforms])
        return self.net.extract_backbone(patches)

    def init_classifier(self, init_backbone_feat):
        x, x_nhwc = self.net.extract_classification_feat(init_backbone_feat, nhwc=True)
        if 'dropout' in self.params.augmentation and self.params.get('use_augmentation', True):
            num, prob = self.params.augmentation['dropout']
            self.transforms.extend(self.transforms[:1] * num)
            # F.dropout2d's channel mask drawn from the host generator as the reference's CPU run draws it
            mask = F.dropout2d(torch.ones(num, x.shape[1], 1, 1), p=prob, training=True).to(self.dev)
            drop = x[0:1].expand(num, -1, -1, -1) * mask
            x = torch.cat([x, drop])
            x_nhwc = torch.cat([x_nhwc, drop.permute(0, 2, 3, 1)])
        self.feature_sz = torch.Tensor(list(x.shape[-2:]))
        ksz = self.net.filter_size
        self.kernel_size = torch.Tensor([ksz, ksz])
        self.output_sz = self.feature_sz + (self.kernel_size + 1) % 2
        self.output_window = None
        target_boxes = self.init_target_boxes()
        w = self.net.init_filter(x_nhwc.contiguous(), target_boxes)
        num_iter = self.params.get('net_opt_iter', None)
        self.target_filter = self.optimizer.optimize(w, x.unsqueeze(1).contiguous(), target_boxes.view(-1, 1, 4),
                                                     num_iter=num_iter)
        self.init_memory(x)

    def init_target_boxes(self):
        self.classifier_target_box = self.get_iounet_box(self.pos, self.target_sz, self.init_sample_pos,
                                                         self.init_sample_scale)
        init_target_boxes = torch.stack([self.classifier_target_box + torch.Tensor([T.shift[1], T.shift[0], 0, 0])
                                         for T in self.transforms])
        self.target_boxes = init_target_boxes.new_zeros(self.params.sample_memory_size, 4)
        self.target_boxes[:init_target_boxes.shape[0], :] = init_target_boxes
        return init_target_boxes

    def init_memory(self, x):
        self.num_init_samples = x.shape[0]
        self.num_stored_samples = self.num_init_samples
        self.previous_replace_ind = None
        self.sample_weights = torch.zeros(self.params.sample_memory_size)
        self.sample_weights[:self.num_init_samples] = torch.ones(1) / x.shape[0]
        self.training_samples = x.new_zeros(self.params.sample_memory_size, *x.shape[1:])
        self.training_samples[:x.shape[0]] = x

    def track(self, image, info: dict = None) -> dict:
        patch, coords = self.track_sample(image)
        test_x = self.net.extract_classification_feat(self.net.extract_backbone(patch))
        scores = self.net.classify(self.target_filter, test_x).squeeze(1).cpu()
        return self.track_update(test_x, scores, coords)

    # the per-frame step in two halves so that track_batch can run the network once for many sequences
    def track_sample(self, image, out=None):
        """dimp.py:85-99 up to the patch: frame counter, the centred sample position, the search patch
        (written into ``out`` when given) -> (patch [1, 6, 288, 288], sample_coords [1, 4])."""
        self.debug_info = {}
        self.frame_num += 1
        frame = self._frame(image)
        sample_pos_c = self.pos + ((self.feature_sz + self.kernel_size) % 2) * self.target_scale * \
            self.img_support_sz / (2 * self.feature_sz)
        patch, coords = self._sample_patch(frame, sample_pos_c, self.target_scale * self.scale_factors[0] *
                                           self.img_sample_sz, self.img_sample_sz)
        if out is not None:
            out.copy_(patch[0])
        return patch, coords

    def track_update(self, test_x, scores, sample_coords):
        """dimp.py:101-166 after the classifier: localisation, state update, memory / filter update, output.
        test_x: this sequence's clf features [1, 512, 18, 18] (device); scores: [1, 19, 19] (host)."""
        sample_pos, sample_scales = self.get_sample_location(sample_coords)
        translation_vec, scale_ind, s, flag = self.localize_advanced(scores, sample_pos, sample_scales)
        new_pos = sample_pos[scale_ind, :] + translation_vec
        if flag != 'not_found':
            self.update_state(new_pos, sample_scales[scale_ind])
        update_flag = flag not in ['not_found', 'uncertain']
        hard_negative = flag == 'hard_negative'
        learning_rate = self.params.get('hard_negative_learning_rate', None) if hard_negative else None
        if update_flag and self.params.get('update_classifier', False):
            train_x = test_x[scale_ind:scale_ind + 1, ...]
            target_box = self.get_iounet_box(self.pos, self.target_sz, sample_pos[scale_ind, :],
                                             sample_scales[scale_ind])
            self.update_classifier(train_x, target_box, learning_rate, s[scale_ind, ...])
        score_map = s[scale_ind, ...]
        max_score = torch.max(score_map).item()
        self.debug_info['flag'] = flag
        self.debug_info['max_score'] = max_score
        self.debug_info['score_map'] = score_map
        new_state = torch.cat((self.pos[[1, 0]] - (self.target_sz[[1, 0]] - 1) / 2, self.target_sz[[1, 0]]))
        return {'target_bbox': new_state.tolist(), 'confidence': max_score}

    def get_sample_location(self, sample_coord):
        sample_coord = sample_coord.float()
        sample_pos = 0.5 * (sample_coord[:, :2] + sample_coord[:, 2:] - 1)
        sample_scales = ((sample_coord[:, 2:] - sample_coord[:, :2]) / self.img_sample_sz).prod(dim=1).sqrt()
        return sample_pos, sample_scales

    @staticmethod
    def max2d(a):
        """pytracking dcf.max2d: maximum and (row, col) argmax over the last two dims."""
        max_val_row, argmax_row = torch.max(a, dim=-2)
        max_val, argmax_col = torch.max(max_val_row, dim=-1)
        argmax_row = argmax_row.view(argmax_col.numel(), -1)[torch.arange(argmax_col.numel()), argmax_col.view(-1)]
        argmax_row = argmax_row.reshape(argmax_col.shape)
        return max_val, torch.cat((argmax_row.unsqueeze(-1), argmax_col.unsqueeze(-1)), -1)

    def localize_advanced(self, scores, sample_pos, sample_scales):
        sz = scores.shape[-2:]
        score_sz = torch.Tensor(list(sz))
        output_sz = score_sz - (self.kernel_size + 1) % 2
        score_center = (score_sz - 1) / 2
        scores_hn = scores
        max_score1, max_disp1 = self.max2d(scores)
        _, scale_ind = torch.max(max_score1, dim=0)
        sample_scale = sample_scales[scale_ind]
        max_score1 = max_score1[scale_ind]
        max_disp1 = max_disp1[scale_ind, ...].float().view(-1)
        target_disp1 = max_disp1 - score_center
        translation_vec1 = target_disp1 * (self.img_support_sz / output_sz) * sample_scale
        p = self.params
        if max_score1.item() < p.target_not_found_threshold:
            return translation_vec1, scale_ind, scores_hn, 'not_found'
        if max_score1.item() < p.get('uncertain_threshold', -float('inf')):
            return translation_vec1, scale_ind, scores_hn, 'uncertain'
        if max_score1.item() < p.get('hard_sample_threshold', -float('inf')):
            return translation_vec1, scale_ind, scores_hn, 'hard_negative'
        target_neigh_sz = p.target_neighborhood_scale * (self.target_sz / sample_scale) * (output_sz /
                                                                                           self.img_support_sz)
        top = max(round(max_disp1[0].item() - target_neigh_sz[0].item() / 2), 0)
        bottom = min(round(max_disp1[0].item() + target_neigh_sz[0].item() / 2 + 1), sz[0])
        left = max(round(max_disp1[1].item() - target_neigh_sz[1].item() / 2), 0)
        right = min(round(max_disp1[1].item() + target_neigh_sz[1].item() / 2 + 1), sz[1])
        scores_masked = scores_hn[scale_ind:scale_ind + 1, ...].clone()
        scores_masked[..., top:bottom, left:right] = 0
        max_score2, max_disp2 = self.max2d(scores_masked)
        max_disp2 = max_disp2.float().view(-1)
        target_disp2 = max_disp2 - score_center
        translation_vec2 = target_disp2 * (self.img_support_sz / output_sz) * sample_scale
        prev_target_vec = (self.pos - sample_pos[scale_ind, :]) / ((self.img_support_sz / output_sz) * sample_scale)
        if max_score2 > p.distractor_threshold * max_score1:
            disp_norm1 = torch.sqrt(torch.sum((target_disp1 - prev_target_vec) ** 2))
            disp_norm2 = torch.sqrt(torch.sum((target_disp2 - prev_target_vec) ** 2))
            disp_threshold = p.dispalcement_scale * math.sqrt(sz[0] * sz[1]) / 2
            if disp_norm2 > disp_threshold and disp_norm1 < disp_threshold:
                return translation_vec1, scale_ind, scores_hn, 'hard_negative'
            if disp_norm2 < disp_threshold and disp_norm1 > disp_threshold:
                return translation_vec2, scale_ind, scores_hn, 'hard_negative'
            if disp_norm2 > disp_threshold and disp_norm1 > disp_threshold:
                return translation_vec1, scale_ind, scores_hn, 'uncertain'
            return translation_vec1, scale_ind, scores_hn, 'uncertain'
        if max_score2 > p.hard_negative_threshold * max_score1 and max_score2 > p.target_not_found_threshold:
            return translation_vec1, scale_ind, scores_hn, 'hard_negative'
        return translation_vec1, scale_ind, scores_hn, 'normal'

    def update_state(self, new_pos, new_scale=None):
        if new_scale is not None:
            self.target_scale = new_scale.clamp(self.min_scale_factor, self.max_scale_factor)
            self.target_sz = self.base_target_sz * self.target_scale
        inside_offset = (self.params.get('target_inside_ratio', 0.2) - 0.5) * self.target_sz
        self.pos = torch.max(torch.min(new_pos, self.image_sz - inside_offset), inside_offset)

    def get_iounet_box(self, pos, sz, sample_pos, sample_scale):
        box_center = (pos - sample_pos) / sample_scale + (self.img_sample_sz - 1) / 2
        box_sz = sz / sample_scale
        target_ul = box_center - (box_sz - 1) / 2
        return torch.cat([target_ul.flip((0,)), box_sz.flip((0,))])

    def update_classifier(self, train_x, target_box, learning_rate=None, scores=None):
        hard_negative_flag = learning_rate is not None
        if learning_rate is None:
            learning_rate = self.params.learning_rate
        if hard_negative_flag or self.frame_num % self.params.get('train_sample_interval', 1) == 0:
            self.update_memory(train_x, target_box, learning_rate)
        num_iter = 0
        low_score_th = self.params.get('low_score_opt_threshold', None)
        if hard_negative_flag:
            num_iter = self.params.get('net_opt_hn_iter', None)
        elif low_score_th is not None and low_score_th > scores.max().item():
            num_iter = self.params.get('net_opt_low_iter', None)
        elif (self.frame_num - 1) % self.params.train_skipping == 0:
            num_iter = self.params.get('net_opt_update_iter', None)
        if num_iter > 0:
            n = min(self.num_stored_samples, self.params.sample_memory_size)
            samples = self.training_samples[:n].unsqueeze(1).contiguous()
            self.target_filter = self.optimizer.optimize(self.target_filter, samples,
                                                         self.target_boxes[:n].clone().view(-1, 1, 4),
                                                         sample_weight=self.sample_weights[:n].view(-1, 1),
                                                         num_iter=num_iter)

    def update_memory(self, sample_x, target_box, learning_rate=None):
        replace_ind = self.update_sample_weights(learning_rate)
        self.previous_replace_ind = replace_ind
        self.training_samples[replace_ind:replace_ind + 1, ...] = sample_x
        self.target_boxes[replace_ind, :] = target_box
        self.num_stored_samples += 1

    def update_sample_weights(self, learning_rate=None):
        sw, prev_ind = self.sample_weights, self.previous_replace_ind
        num_samp, num_init = self.num_stored_samples, self.num_init_samples
        lr = learning_rate if learning_rate is not None else self.params.learning_rate
        init_samp_weight = self.params.get('init_samples_minimum_weight', None)
        if init_samp_weight == 0:
            init_samp_weight = None
        s_ind = 0 if init_samp_weight is None else num_init
        if num_samp == 0 or lr == 1:
            sw[:] = 0
            sw[0] = 1
            r_ind = 0
        else:
            if num_samp < sw.shape[0]:
                r_ind = num_samp
            else:
                _, r_ind = torch.min(sw[s_ind:], 0)
                r_ind = r_ind.item() + s_ind
            if prev_ind is None:
                sw /= 1 - lr
                sw[r_ind] = lr
            else:
                sw[r_ind] = sw[prev_ind] / (1 - lr)
        sw /= sw.sum()
        if init_samp_weight is not None and sw[:num_init].sum() < init_samp_weight:
            sw /= init_samp_weight + sw[num_init:].sum()
            sw[:num_init] = init_samp_weight / num_init
        return r_ind


def track_batch(trackers, frames):
    """One frame for each of several DiMP trackers sharing one DiMPNet: the search patches are sampled
    into one batch, the two backbones + clf features run once over it, every sequence's filter is applied
    in one grouped launch (apply_filter with S = len(trackers)), then each tracker localises and updates
    on its own (the reference runs one tracker per process, test_rgbt_mgpus.py:178-186).  Returns the
    per-tracker outputs of DiMP.track."""
    net = trackers[0].net
    n = len(trackers)
    if any(t.net is not net for t in trackers):
        raise ValueError("track_batch needs trackers that share one DiMPNet")
    sz = trackers[0].img_sample_sz.long().tolist()
    patches = torch.empty(n, 6, sz[0], sz[1], dtype=torch.float32, device=net.dev)
    coords = [t.track_sample(f, out=patches[i])[1] for i, (t, f) in enumerate(zip(trackers, frames))]
    test_x = net.extract_classification_feat(net.extract_backbone(patches))
    filters = torch.cat([t.target_filter for t in trackers])
    from .dimp import apply_filter
    scores = apply_filter(test_x.unsqueeze(0), filters)[0].cpu()          # [n, 19, 19]
    return [t.track_update(test_x[i:i + 1], scores[i:i + 1], c) for i, (t, c) in enumerate(zip(trackers, coords))]


class PipelinedBatch:
    """track_batch with the host half of one group of sequences overlapped with the device half of the other:
    the trackers are split into two groups; group g's frame k is sampled and its network launched
    (asynchronously, its scores copied to pinned host memory behind an event) while the host localises and
    updates group 1 - g from frame k - 1.  Per-sequence results are identical to track_batch (each tracker
    still sees its frames in order; only the interleaving of different sequences' host work changes)."""

    def __init__(self, trackers, groups=2):
        self.trackers = trackers
        n = len(trackers)
        bounds = [round(i * n / groups) for i in range(groups + 1)]
        self.groups = [list(range(bounds[i], bounds[i + 1])) for i in range(groups) if bounds[i + 1] > bounds[i]]
        self.pending = [None] * len(self.groups)

    def _start(self, g, frames):
        idx = self.groups[g]
        trs = [self.trackers[i] for i in idx]
        net = trs[0].net
        sz = trs[0].img_sample_sz.long().tolist()
        patches = torch.empty(len(idx), 6, sz[0], sz[1], dtype=torch.float32, device=net.dev)
        coords = [t.track_sample(frames[i], out=patches[j])[1] for j, (i, t) in enumerate(zip(idx, trs))]
        test_x = net.extract_classification_feat(net.extract_backbone(patches))
        from .dimp import apply_filter
        scores = apply_filter(test_x.unsqueeze(0), torch.cat([t.target_filter for t in trs]))[0]
        host = torch.empty(scores.shape, dtype=torch.float32, pin_memory=True)
        host.copy_(scores, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending[g] = (idx, test_x, host, ev, coords)

    def _finish(self, g, outs):
        idx, test_x, host, ev, coords = self.pending[g]
        self.pending[g] = None
        ev.synchronize()
        for j, i in enumerate(idx):
            outs[i] = self.trackers[i].track_update(test_x[j:j + 1], host[j:j + 1], coords[j])

    def step(self, frames):
        """Submit frame k for every sequence; returns the outputs of frame k - 1 (None on the first call)."""
        outs = [None] * len(self.trackers)
        had = self.pending[0] is not None
        for g in range(len(self.groups)):
            if self.pending[g] is not None:
                self._finish(g, outs)
            self._start(g, frames)
        return outs if had else None

    def flush(self):
        outs = [None] * len(self.trackers)
        for g in range(len(self.groups)):
            if self.pending[g] is not None:
                self._finish(g, outs)
        return outs


__all__ = ["DiMP", "parameters", "TrackerParams", "track_batch", "PipelinedBatch"]
