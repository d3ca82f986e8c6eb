"""mfDiMP / DeT-DiMP tracker on the MI355X path.

``DiMP`` keeps the reference tracker's contract and cadence (RGBD/models/DeT/pytracking/tracker/dimp/
dimp.py: ``initialize(image, info)`` :24-82, ``track(image)`` :85-166, advanced localisation :232-301,
init augmentation :322-385, classifier init / memory / update :399-504 and :538-607), restated over the
device path:

* patch sampling, init augmentations, the two ResNet-50 backbones + max merge, the clf features, the
  filter initialiser (PrRoIPool) run as HIP kernels (mmtrack_amd.dimpnet, csrc/dimpnet.hip, dimpconv.hip);
* the steepest-descent Gauss-Newton filter optimiser and the classifier (apply_filter) run as HIP
  kernels (mmtrack_amd.dimp, csrc/dimp.hip);
* the per-frame state machine -- sample geometry from the tracked position and scale, localize_advanced,
  update_state, the sample memory's weights / boxes / slots and the choice of Gauss-Newton iterations --
  runs on the device over every sequence of a batch at once (csrc/dimptrack.hip): the tracker state lives
  in device memory (``DimpPool``), and per frame only a small result record per sequence (box, score, flag,
  iterations) comes back to the host, which launches the filter updates the records ask for.
  Initialisation (augmented samples, initial filter, 10 Gauss-Newton steps) is host-orchestrated, once.

IoU-Net box refinement (AtomIoUNet + PrRoIPool gradients, dimp.py:609-700) is not part of this path:
``parameters()`` sets ``use_iou_net = False``, the reference's switch for it (dimp.py:76-78, 123-130), so
position comes from the classifier and the size follows the sample scale (the tracker golden was made with
the same setting; parity with the reference's default IoU-Net configuration is not claimed).  Random init
augmentation shifts and the dropout masks draw from the host torch generator in the reference's order, so a
seeded run matches the reference run with the same seed.
"""
from __future__ import annotations

import ctypes
import math
import os

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

    def __init__(self, params, state_dict=None, device=None, net=None, pool=None):
        self.params = params
        if net is None:
            sd = state_dict if state_dict is not None else getattr(params, 'state_dict', None)
            if sd is None:
                raise ValueError("DiMP needs the network weights (params.state_dict or state_dict=)")
            net = DiMPNet(sd, device=device)
        self.net = net
        self.dev = self.net.dev
        # the device-resident per-frame state: a slot of a shared pool (batched trackers) or a pool of its own
        self.pool = pool if pool is not None else DimpPool(net, 1, params)
        if self.pool.net is not net:
            raise ValueError("the pool belongs to another DiMPNet")
        self.slot = self.pool.alloc()
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
        w = self.optimizer.optimize(w, x.unsqueeze(1).contiguous(), target_boxes.view(-1, 1, 4), num_iter=num_iter)
        # the filter lives in the pool's filter array (one row per slot), so a batch's filters apply and update
        # in place without gathering
        self.target_filter = self.pool.write_filter(self.slot, w)
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
        """init_memory (dimp.py:505-536): the sample memory and the tracker state into the device slot."""
        self.num_init_samples = x.shape[0]
        sw = torch.zeros(self.params.sample_memory_size)
        sw[:self.num_init_samples] = torch.ones(1) / x.shape[0]
        st = _lib.MmtDimpState()
        for name in ("pos", "target_sz", "base_target_sz", "image_sz"):
            v = getattr(self, name).float()
            getattr(st, name)[0], getattr(st, name)[1] = float(v[0]), float(v[1])
        st.target_scale = float(torch.as_tensor(self.target_scale, dtype=torch.float32))
        st.min_scale_factor = float(self.min_scale_factor)
        st.max_scale_factor = float(self.max_scale_factor)
        st.frame_num = self.frame_num
        st.num_init = st.num_stored = self.num_init_samples
        st.prev_replace = -1
        for k in range(self.params.sample_memory_size):
            st.sample_weights[k] = float(sw[k])
            for j in range(4):
                st.target_boxes[k][j] = float(self.target_boxes[k, j])
        self.pool.write_state(self.slot, st, x)

    def get_iounet_box(self, pos, sz, sample_pos, sample_scale):
        """dimp.py:468-475 (the initial target boxes; per frame the device restates it)."""
        box_center = (pos - sample_pos) / sample_scale + (self.img_sample_sz - 1) / 2
        box_sz = sz / sample_scale
        target_ul = box_center - (box_sz - 1) / 2
        return torch.cat([target_ul.flip((0,)), box_sz.flip((0,))])

    def track(self, image, info: dict = None) -> dict:
        """track (dimp.py:85-166): one frame through the device state machine (a batch of one)."""
        return track_batch([self], [image])[0]

    def _output(self, res):
        flag = FLAGS[res.flag]
        self.debug_info = {'flag': flag, 'max_score': float(res.max_score)}
        return {'target_bbox': [float(v) for v in res.box], 'confidence': float(res.max_score)}

FLAGS = ('normal', 'not_found', 'uncertain', 'hard_negative')
# f16x3 pools sample 6-channel frames straight into the backbones' normalised 4-channel inputs
# (mmt_dimp_track_sample_norm4); MMT_DIMP_FUSED_SAMPLE=0 (tuning A/B, stage tests): the NCHW patch + normalise
FUSED_SAMPLE = os.environ.get("MMT_DIMP_FUSED_SAMPLE", "1") != "0"


class DimpPool:
    """Device-resident state of up to ``capacity`` DiMP trackers sharing one DiMPNet: one mmt_dimp_state per
    slot (position, scale, sample weights and boxes), the sample memory [capacity][50][512][18][18] fp32, and
    the per-frame result records (pinned host copy).  Trackers of one pool whose slots are consecutive are
    advanced together by track_batch."""

    def __init__(self, net, capacity, params):
        self.net, self.cap, self.dev = net, capacity, net.dev
        self.lib = _lib.load()
        self.sbytes = self.lib.mmt_dimp_state_bytes()
        if self.sbytes != ctypes.sizeof(_lib.MmtDimpState):
            raise RuntimeError("libmmtrack.so's mmt_dimp_state does not match the binding")
        self.states = torch.zeros(capacity * self.sbytes, dtype=torch.uint8, device=self.dev)
        self.rbytes = ctypes.sizeof(_lib.MmtDimpResult)
        self.results = torch.zeros(capacity * self.rbytes, dtype=torch.uint8, device=self.dev)
        self.memory = None   # [capacity][50][C][h][w], allocated with the first sample shape
        self.filters = None  # [capacity][C][fh][fw]: every slot's target filter
        self.next = 0
        p = _lib.MmtDimpTrackParams()
        sz = params.image_sample_size
        sz = (sz, sz) if isinstance(sz, int) else tuple(sz)
        fsz = (sz[0] // net.feat_stride, sz[1] // net.feat_stride)
        for d in range(2):
            p.img_sample_sz[d], p.feature_sz[d], p.kernel_size[d] = float(sz[d]), float(fsz[d]), float(net.filter_size)
        g = params.get
        inf = float('inf')
        p.target_not_found_threshold = g('target_not_found_threshold')
        p.uncertain_threshold = g('uncertain_threshold', -inf)
        p.hard_sample_threshold = g('hard_sample_threshold', -inf)
        p.distractor_threshold = g('distractor_threshold')
        p.hard_negative_threshold = g('hard_negative_threshold')
        p.target_neighborhood_scale = g('target_neighborhood_scale')
        p.dispalcement_scale = g('dispalcement_scale')
        p.target_inside_ratio = g('target_inside_ratio', 0.2)
        low = g('low_score_opt_threshold', None)
        p.low_score_opt_threshold = float('nan') if low is None else low
        p.learning_rate = g('learning_rate')
        p.hard_negative_learning_rate = g('hard_negative_learning_rate', None) or g('learning_rate')
        p.init_samples_minimum_weight = g('init_samples_minimum_weight', None) or 0.0
        p.sample_memory_size = g('sample_memory_size')
        p.train_sample_interval = g('train_sample_interval', 1)
        p.train_skipping = g('train_skipping')
        p.net_opt_update_iter = g('net_opt_update_iter', None) or 0
        p.net_opt_hn_iter = g('net_opt_hn_iter', None) or 0
        p.net_opt_low_iter = g('net_opt_low_iter', None) or 0
        p.update_classifier = int(bool(g('update_classifier', False)))
        if not g('advanced_localization', False) or g('use_iou_net', True) or g('window_output', False):
            raise NotImplementedError("the device DiMP path restates advanced localisation without IoU-Net / window")
        if p.sample_memory_size != _lib.MMT_DIMP_MEMORY:
            raise ValueError(f"sample_memory_size must be {_lib.MMT_DIMP_MEMORY}")
        self.tparams = p
        # frame descriptors: one pinned host copy per record parity, copied to the device without a stream sync;
        # a parity's pinned rows (descriptors and staged host frames) are rewritten only after the copies of its
        # previous launch have run (its event, normally long complete when the host is one frame behind)
        # frame descriptors and result records in mapped, coherent pinned memory (mmt_host_alloc) that the kernels
        # read and write in place: no copy launches (the sampler reads a launch's descriptors, the localisation
        # kernel writes its records); two parities, so frame k + 1 may be launched before frame k's records are read
        fb = ctypes.sizeof(_lib.MmtDimpFrame)
        self._host_ptrs = []

        def host_buffer(nbytes):
            ptr = self.lib.mmt_host_alloc(nbytes)
            if not ptr:
                raise RuntimeError("mmt_host_alloc failed")
            self._host_ptrs.append(ptr)
            return torch.frombuffer((ctypes.c_uint8 * nbytes).from_address(ptr), dtype=torch.uint8)
        self.desc_host = [host_buffer(capacity * fb) for _ in range(2)]
        self._stage = {}      # (slot, parity) -> pinned host staging of a numpy frame
        self._copy_ev = {}    # (first slot, parity) -> event after the launch's reads of its descriptors / staging
        self.res_host = [host_buffer(capacity * self.rbytes) for _ in range(2)]
        self._parity = {}   # per first slot: the record buffer its next launch uses
        self.max_iter = max(p.net_opt_update_iter, p.net_opt_hn_iter, p.net_opt_low_iter) if p.update_classifier else 0
        self._opt_ws = None

    def alloc(self):
        if self.next >= self.cap:
            raise RuntimeError(f"DimpPool: all {self.cap} slots are in use")
        self.next += 1
        return self.next - 1

    def state_ptr(self, slot):
        return self.states.data_ptr() + slot * self.sbytes

    def boxes_ptr(self, slot):
        return self.state_ptr(slot) + _lib.MmtDimpState.target_boxes.offset

    def weights_ptr(self, slot):
        return self.state_ptr(slot) + _lib.MmtDimpState.sample_weights.offset

    def write_state(self, slot, st, x):
        raw = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8)
        self.states[slot * self.sbytes:(slot + 1) * self.sbytes].copy_(raw)
        if self.memory is None:
            self.memory = torch.zeros(self.cap, _lib.MMT_DIMP_MEMORY, *x.shape[1:], dtype=torch.float32, device=self.dev)
        self.memory[slot, :x.shape[0]] = x
        self.memory[slot, x.shape[0]:] = 0

    def write_filter(self, slot, w):
        """Store slot's filter [1, C, fh, fw]; returns the slot's row (a view the tracker keeps)."""
        if self.filters is None:
            self.filters = torch.zeros(self.cap, *w.shape[1:], dtype=torch.float32, device=self.dev)
        self.filters[slot] = w[0]
        return self.filters[slot:slot + 1]

    def result(self, slot, buf=0):
        return _lib.MmtDimpResult.from_buffer_copy(bytes(self.res_host[buf][slot * self.rbytes:(slot + 1) * self.rbytes]
                                                         .numpy()))

    def launch(self, trackers, frames, first):
        """Sample, network, classifier and the device state update for trackers in slots [first, first + n);
        the result records go to pinned host memory behind the returned event."""
        lib, n, net = self.lib, len(trackers), self.net
        buf = self._parity.get(first, 0)
        prev = self._copy_ev.get((first, buf))
        if prev is not None:
            prev.synchronize()   # this parity's pinned rows are still being read by the launch two frames back
        fr = [self._device_frame(first + i, buf, f) for i, f in enumerate(frames)]
        fb = ctypes.sizeof(_lib.MmtDimpFrame)
        desc_ptr = self.desc_host[buf].data_ptr() + first * fb
        desc = (_lib.MmtDimpFrame * n).from_address(desc_ptr)
        for i, f in enumerate(fr):
            d = desc[i]
            d.data, d.stride, d.H, d.W, d.C = f.data_ptr(), f.stride(0), f.shape[0], f.shape[1], f.shape[2]
        sz = [int(v) for v in self.tparams.img_sample_sz]
        C = fr[0].shape[2]
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        if net.precision == "f16x3" and C == 6 and FUSED_SAMPLE:
            # the sampler writes the backbones' normalised 4-channel halves itself (same bits as sample + normalise)
            # (and clears the backbones' max words: no fill launch)
            xa, xb = net.norm4_buffers(n, sz[0], sz[1])
            words = net.max_words()
            rc = lib.mmt_dimp_track_sample_norm4(ctypes.c_void_p(self.state_ptr(first)), ctypes.c_void_p(desc_ptr), n,
                                                 ctypes.byref(self.tparams), sz[0], sz[1], net._mean, net._std,
                                                 ctypes.c_void_p(xa.data_ptr()), ctypes.c_void_p(xb.data_ptr()),
                                                 ctypes.c_void_p(words.data_ptr()), words.numel(), stream)
            if rc != 0:
                raise RuntimeError(f"mmt_dimp_track_sample_norm4 failed ({rc})")
            self._descriptors_read(first, buf)
            layer3 = net.extract_backbone_norm4(n, sz[0], sz[1], words_cleared=True)
        else:
            patches = torch.empty(n, C, sz[0], sz[1], dtype=torch.float32, device=self.dev)
            rc = lib.mmt_dimp_track_sample(ctypes.c_void_p(self.state_ptr(first)), ctypes.c_void_p(desc_ptr), n,
                                           ctypes.byref(self.tparams), sz[0], sz[1],
                                           ctypes.c_void_p(patches.data_ptr()), stream)
            if rc != 0:
                raise RuntimeError(f"mmt_dimp_track_sample failed ({rc})")
            self._descriptors_read(first, buf)
            layer3 = net.extract_backbone(patches)
        test_x = net.extract_classification_feat(layer3)
        from .dimp import apply_filter
        scores = apply_filter(test_x.unsqueeze(0), self.filters[first:first + n])[0].contiguous()
        F_ = test_x[0].numel()
        rc = lib.mmt_dimp_track_update_pinned(ctypes.c_void_p(self.state_ptr(first)), n,
                                              ctypes.c_void_p(scores.data_ptr()), scores.shape[-2], scores.shape[-1],
                                              ctypes.byref(self.tparams), ctypes.c_void_p(test_x.data_ptr()), F_,
                                              ctypes.c_void_p(self.memory[first].data_ptr()),
                                              ctypes.c_void_p(self.results.data_ptr() + first * self.rbytes),
                                              ctypes.c_void_p(self.res_host[buf].data_ptr() + first * self.rbytes),
                                              stream)
        if rc != 0:
            raise RuntimeError(f"mmt_dimp_track_update_pinned failed ({rc})")
        # update_classifier's Gauss-Newton steps where the records ask for them (dimp.py:555-570), decided on
        # the device: one launch sequence over the batch, no host round trip
        if self.max_iter > 0:
            opt = trackers[0].optimizer
            C, h, w = self.memory.shape[2:]
            fh, fw = self.filters.shape[-2:]
            nbytes = lib.mmt_dimp_track_optimize_ws_bytes(n, C, h, w, fh, fw, self.max_iter)
            if self._opt_ws is None or self._opt_ws.numel() < nbytes:
                self._opt_ws = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
            rc = lib.mmt_dimp_track_optimize(ctypes.c_void_p(self.state_ptr(first)), n,
                                             ctypes.c_void_p(self.results.data_ptr() + first * self.rbytes),
                                             ctypes.c_void_p(self.memory[first].data_ptr()), C, h, w,
                                             ctypes.c_void_p(self.filters[first].data_ptr()), fh, fw,
                                             ctypes.byref(opt.params), self.max_iter,
                                             ctypes.c_void_p(self._opt_ws.data_ptr()), nbytes, stream)
            if rc != 0:
                raise RuntimeError(f"mmt_dimp_track_optimize failed ({rc})")
        self._parity[first] = buf ^ 1
        ev = torch.cuda.Event()
        ev.record()
        return ev, buf

    def _descriptors_read(self, first, buf):
        """An event behind the kernel that read this parity's descriptors (and host-staged frames): they are
        rewritten two frames later only once it has passed."""
        cev = torch.cuda.Event()
        cev.record()
        self._copy_ev[(first, buf)] = cev

    def __del__(self):
        for p in getattr(self, "_host_ptrs", []):
            try:
                self.lib.mmt_host_free(p)
            except Exception:
                pass
        self._host_ptrs = []

    def _device_frame(self, slot, buf, image):
        """A frame on the device without a blocking copy: device tensors as they are, host frames through a
        pinned staging buffer of (slot, parity) and an asynchronous copy."""
        if isinstance(image, torch.Tensor) and image.is_cuda:
            return image.to(self.dev).contiguous()
        src = image if isinstance(image, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(image))
        st = self._stage.get((slot, buf))
        if st is None or st.shape != src.shape or st.dtype != src.dtype:
            st = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            self._stage[(slot, buf)] = st
        st.copy_(src)
        return st.to(self.dev, non_blocking=True)

    def finish(self, trackers, first, ticket):
        """Wait for a launch's records (its filter updates are already queued on the device) and return the
        per-tracker outputs."""
        ev, buf = ticket
        ev.synchronize()
        return [t._output(self.result(first + i, buf)) for i, t in enumerate(trackers)]


def _slots(trackers):
    pool = trackers[0].pool
    first = trackers[0].slot
    if any(t.pool is not pool for t in trackers) or [t.slot for t in trackers] != list(range(first, first + len(trackers))):
        raise ValueError("track_batch needs trackers of one DimpPool in consecutive slots")
    return pool, first


def track_batch(trackers, frames):
    """One frame for each of several DiMP trackers of one DimpPool (consecutive slots): the search patches
    are sampled into one batch from the device state, the two backbones + clf features run once over it, every
    sequence's filter is applied in one grouped launch, the device state machine advances every sequence, and
    the filter updates the result records ask for follow (the reference runs one tracker per process,
    test_rgbt_mgpus.py:178-186).  Returns the per-tracker outputs of DiMP.track."""
    runs, i = [], 0   # runs of trackers in consecutive slots of one pool, each one batch
    while i < len(trackers):
        j = i + 1
        while j < len(trackers) and trackers[j].pool is trackers[i].pool and trackers[j].slot == trackers[j - 1].slot + 1:
            j += 1
        runs.append((i, j))
        i = j
    launched = [(a, b, trackers[a].pool.launch(trackers[a:b], frames[a:b], trackers[a].slot)) for a, b in runs]
    outs = []
    for a, b, ticket in launched:
        outs.extend(trackers[a].pool.finish(trackers[a:b], trackers[a].slot, ticket))
    return outs


class PipelinedBatch:
    """track_batch with the host one frame behind the device: frame k of every group of sequences is launched
    (asynchronously -- the state machine and the filter updates run on the device, the result records are
    copied to pinned host memory behind an event) before the host reads frame k - 1's records, so the device
    always has the next frame queued.  groups > 1 splits the sequences into launches of their own.
    Per-sequence results are identical to track_batch (each tracker sees its frames in order; only the
    interleaving of different sequences' work changes)."""

    def __init__(self, trackers, groups=1):
        self.trackers = trackers
        n = len(trackers)
        bounds = [round(i * n / groups) for i in range(groups + 1)]
        self.groups = [list(range(bounds[i], bounds[i + 1])) for i in range(groups) if bounds[i + 1] > bounds[i]]
        self.pending = [None] * len(self.groups)
        _slots(trackers)

    def _start(self, g, frames):
        idx = self.groups[g]
        trs = [self.trackers[i] for i in idx]
        pool, first = _slots(trs)
        self.pending[g] = pool.launch(trs, [frames[i] for i in idx], first)

    def _finish(self, g, ticket, outs):
        idx = self.groups[g]
        trs = [self.trackers[i] for i in idx]
        pool, first = _slots(trs)
        for i, o in zip(idx, pool.finish(trs, first, ticket)):
            outs[i] = o

    def step(self, frames):
        """Submit frame k for every sequence; returns the outputs of frame k - 1 (None on the first call)."""
        outs = [None] * len(self.trackers)
        had = self.pending[0] is not None
        for g in range(len(self.groups)):
            prev = self.pending[g]
            self._start(g, frames)
            if prev is not None:
                self._finish(g, prev, outs)
        return outs if had else None

    def flush(self):
        outs = [None] * len(self.trackers)
        for g in range(len(self.groups)):
            if self.pending[g] is not None:
                self._finish(g, self.pending[g], outs)
                self.pending[g] = None
        return outs


__all__ = ["DiMP", "DimpPool", "parameters", "TrackerParams", "track_batch", "PipelinedBatch"]
