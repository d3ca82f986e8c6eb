"""DeT / mfDiMP DiMP-50 classification path on the HIP kernels (mmt_conv2d_f32 & co, include/mmtrack.h).

``DiMPNet`` is DiMPnet_DeT with merge_type 'max' (RGBD/models/DeT/ltr/models/tracking/dimpnet.py:15-156,
built by dimp50_DeT, :421-476) as the DiMP tracker uses it (pytracking/tracker/dimp/dimp.py):

* ``extract_backbone(patches)``      NetWithBackbone.extract_backbone (net_wrappers.py:81-85): normalise
  each 3-channel half, two ResNet-50 backbones to layer3 (resnet.py), torch.max merge (dimpnet.py:103);
* ``extract_classification_feat``    the clf feature block (features.py:47-66: 3x3 conv 1024 -> 512 without
  bias, InstanceL2Norm) -> [N, 512, 18, 18] fp32 (NCHW, what the DiMP optimiser reads);
* ``init_filter(feat, bb)``          FilterInitializerLinear (initializer.py:118-170): 3x3 conv, PrRoIPool2D
  4 x 4 of the target box at 1/16, mean over the samples;
* ``classify``                       LinearFilter.classify (linear_filter.py:78-83) = dimp.apply_filter.

Weights load from the reference state_dict keys (load_state_dict strict on the keys this path reads;
IoU-Net ``bb_regressor.*``, ``layer4`` and ``fc`` keys are accepted and unused).  BatchNorm (eval) is
folded into each conv in float64 on the host.  Precision (``precision``): "f16x3" (default) runs every
convolution on the fp16 matrix cores with fp32-faithful split products (mmt_conv2d_f16x3, csrc/dimpconv.hip:
fp16 hi / lo halves of power-of-two range-scaled operands, Wh*Ah + Wl*Ah + Wh*Al with fp32 accumulation; the
activation scales come from each producing conv's max|y|, kept on the device); "fp32" keeps the plain fp32
MFMA kernel (mmt_conv2d_f32).  Everything else is fp32.  There is no CPU fallback: a missing libmmtrack.so
raises ImportError.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from .synth import RESNET50_LAYERS, dimp_shapes

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def _rc(rc, what):
    if rc == -1:
        raise ValueError(f"{what}: invalid argument")
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def range_scale(m):
    """engine.cpp range_scale: the power of two s with m * s <= 2^14 (m > 0)."""
    return 2.0 ** (14 - math.ceil(math.log2(m))) if m > 0 else 1.0


MAX_WORDS = 64 * 32   # sharded max|y| words per tensor (mmt_conv_max_words)
# f16x3: the stem writes the max-pooled map directly (MMT_CONV_POOL); MMT_DIMP_STEMPOOL=0 (tuning A/B): the stem map
# and a separate max-pool launch
STEM_POOL = os.environ.get("MMT_DIMP_STEMPOOL", "1") != "0"


class _Conv:
    """One conv (+ folded BN): weight [Cout][kh][kw][Cin] and bias [Cout] fp32 on the device; with f16x3 the
    weights also as the fp16 halves of w * s_w, [Cout][Kp] (the stem: 4 channels per tap, K padded to 32)."""

    def __init__(self, w, bn=None, bias=None, stride=1, pad=0, dev=None, w4=True, f16x3=False):
        w = w.detach().double()
        co = w.shape[0]
        b = bias.detach().double() if bias is not None else torch.zeros(co, dtype=torch.float64)
        if bn is not None:
            g, beta, mean, var = (t.detach().double() for t in bn)
            s = g / torch.sqrt(var + 1e-5)
            w = w * s.view(-1, 1, 1, 1)
            b = (b - mean) * s + beta
        wk = w.permute(0, 2, 3, 1)
        # the 3-channel stem: weights padded to 4 channels per tap (MMT_CONV_W4, one float4 per tap)
        self.w4 = w4 and w.shape[1] == 3 and not os.environ.get("MMT_CONV_NOW4")   # (env: tuning A/B)
        if self.w4:
            wk = torch.nn.functional.pad(wk, (0, 1))
        self.w = wk.contiguous().float().to(dev)
        self.b = b.float().to(dev) if (bn is not None or bias is not None) else None
        self.cout, self.cin, self.kh, self.kw = co, w.shape[1], w.shape[2], w.shape[3]
        self.stride, self.pad = stride, pad
        self.f16x3 = f16x3
        if f16x3:
            wq = w.permute(0, 2, 3, 1)
            if self.cin == 3:
                wq = torch.nn.functional.pad(wq, (0, 1))
            wq = wq.reshape(co, -1).float()
            kp = (wq.shape[1] + 31) // 32 * 32
            wq = torch.nn.functional.pad(wq, (0, kp - wq.shape[1]))
            self.w_scale = range_scale(float(wq.abs().max()))
            v = wq * self.w_scale
            hi = v.half()
            lo = (v - hi.float()).half()
            self.wh, self.wl, self.kp = hi.contiguous().to(dev), lo.contiguous().to(dev), kp

    def out_hw(self, H, W):
        return (H + 2 * self.pad - self.kh) // self.stride + 1, (W + 2 * self.pad - self.kw) // self.stride + 1

    def group(self, x, out, relu=False, resid=None, merge_max=False, x_max=None, x_scale=0.0, y_max=None,
              pool=False):
        """This conv's operands as one mmt_conv_group of an f16x3 launch (pool: the stem with the 3 x 3 / stride-2
        max-pool fused, MMT_CONV_POOL; out is then the pooled map)."""
        flags = (1 if relu else 0) | (2 if merge_max else 0) | (8 if pool else 0)
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        return _lib.MmtConvGroup(x.data_ptr(), self.wh.data_ptr(), self.wl.data_ptr(), self.w_scale, ptr(self.b),
                                 ptr(resid), out.data_ptr(), ptr(x_max), float(x_scale), ptr(y_max), flags)

    def __call__(self, lib, x, N, H, W, out, stream, relu=False, resid=None, merge_max=False, x_max=None,
                 x_scale=0.0, y_max=None, ws=None):
        """f16x3: x_max = the input's sharded max words (or x_scale, a static power-of-two input scale), y_max =
        the output's (accumulated by the epilogue; None: not tracked); ws(nbytes) -> a device buffer for split-K
        partials (None: no split)."""
        if self.f16x3:
            run_f16x3(lib, self, [self.group(x, out, relu, resid, merge_max, x_max, x_scale, y_max)], N, H, W, ws,
                      stream)
            return out
        flags = (1 if relu else 0) | (2 if merge_max else 0) | (4 if self.w4 else 0)
        _rc(lib.mmt_conv2d_f32(_p(x), N, H, W, self.cin, _p(self.w), _p(self.b), self.cout, self.kh, self.kw,
                               self.stride, self.pad, _p(resid), _p(out), flags, stream), "mmt_conv2d_f32")
        return out


class _ConvDs:
    """A Bottleneck's conv3 (1 x 1) and its downsample (1 x 1 / stride) as one f16x3 GEMM over concatenated K
    (mmt_conv2d_f16x3_ds_groups, resnet.py:76-95): weights [Cout][Cin3 + Cin_d] -- conv3's BN-folded K then the
    downsample's -- split at one common scale, bias b3 + b_d; the downsample's output is never materialised."""

    def __init__(self, c3, ds, dev):
        w3 = c3.w.double().reshape(c3.cout, -1)     # [Cout][1][1][Cin] fp32 (BN folded) -> [Cout][Cin]
        wd = ds.w.double().reshape(ds.cout, -1)
        wq = torch.cat([w3, wd], dim=1).float()
        self.cout, self.cin3, self.cin_d, self.stride = c3.cout, c3.cin, ds.cin, ds.stride
        self.kp = wq.shape[1]
        self.w_scale = range_scale(float(wq.abs().max()))
        v = wq.to(dev) * self.w_scale
        hi = v.half()
        self.wh, self.wl = hi.contiguous(), (v - hi.float()).half().contiguous()
        self.b = (c3.b.double() + ds.b.double()).float().to(dev)

    def group(self, x, out, relu=True, x_max=None, y_max=None):
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        return _lib.MmtConvGroup(x.data_ptr(), self.wh.data_ptr(), self.wl.data_ptr(), self.w_scale, ptr(self.b),
                                 None, out.data_ptr(), ptr(x_max), 0.0, ptr(y_max), 1 if relu else 0)

    def run(self, lib, groups, ds, N, H, W, H2, W2, ws, stream):
        """groups: conv3's operands per backbone (x = conv2's output [N][H][W][Cin3]); ds: (x2 = the block input
        [N][H2][W2][Cin_d], its max words) per backbone."""
        G = len(groups)
        need = lib.mmt_conv2d_f16x3_ws_bytes(N, H, W, self.kp, self.cout, 1, 1, 1, 0, G)
        buf = ws(need) if (need and ws is not None) else None
        arr = (_lib.MmtConvGroup * G)(*groups)
        darr = (_lib.MmtConvDs * G)(*[_lib.MmtConvDs(x2.data_ptr(), x2m.data_ptr() if x2m is not None else None, 0.0)
                                      for x2, x2m in ds])
        _rc(lib.mmt_conv2d_f16x3_ds_groups(arr, darr, G, N, H, W, self.cin3, H2, W2, self.cin_d, self.stride, self.kp,
                                           self.cout, _p(buf), need if buf is not None else 0, stream),
            "mmt_conv2d_f16x3_ds_groups")


# f16x3: each stage's first Bottleneck runs conv3 + downsample as one GEMM (_ConvDs); MMT_DIMP_DSFUSE=0 (tuning A/B):
# the downsample conv writes its map and conv3 adds it as a residual
DS_FUSE = os.environ.get("MMT_DIMP_DSFUSE", "1") != "0"


def run_f16x3(lib, conv, groups, N, H, W, ws, stream, cin=None):
    """One mmt_conv2d_f16x3_groups launch of conv's shape over groups (the twin layers of the two backbones, or
    one); split-K partials in ws(nbytes) when the library asks for a split.  cin=4: the stem over an image
    padded to 4 channels (mmt_image_normalize4)."""
    G = len(groups)
    cin = conv.cin if cin is None else cin
    need = lib.mmt_conv2d_f16x3_ws_bytes(N, H, W, cin, conv.cout, conv.kh, conv.kw, conv.stride, conv.pad, G)
    buf = ws(need) if (need and ws is not None) else None
    arr = (_lib.MmtConvGroup * G)(*groups)
    _rc(lib.mmt_conv2d_f16x3_groups(arr, G, N, H, W, cin, conv.kp, conv.cout, conv.kh, conv.kw, conv.stride,
                                    conv.pad, _p(buf), need if buf is not None else 0, stream),
        "mmt_conv2d_f16x3_groups")


class DiMPNet:
    def __init__(self, state_dict, device=None, out_dim=512, filter_size=4, feat_stride=16, precision="f16x3"):
        if precision not in ("f16x3", "fp32"):
            raise ValueError(f"precision must be 'f16x3' or 'fp32', got {precision!r}")
        self.precision = precision
        f16 = precision == "f16x3"
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("DiMPNet needs an MI355X (HIP device); there is no CPU path")
        self.dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        missing = [k for k in dimp_shapes() if not k.endswith("num_batches_tracked") and k not in state_dict]
        if missing:
            raise RuntimeError("Error(s) in loading state_dict: missing keys " + ", ".join(missing[:8]))
        for k, shp in dimp_shapes().items():
            if k in state_dict and tuple(state_dict[k].shape) != tuple(shp) and not k.endswith("predictor.weight") \
                    and not k.endswith("predictor.0.weight"):
                raise RuntimeError(f"Error(s) in loading state_dict: size mismatch for {k}: "
                                   f"{tuple(state_dict[k].shape)} vs {tuple(shp)}")
        sd = {k: torch.as_tensor(v) for k, v in state_dict.items()}
        self.sd_opt = {k[len("classifier.filter_optimizer."):]: v for k, v in sd.items()
                       if k.startswith("classifier.filter_optimizer.")}
        self.out_dim, self.filter_size, self.feat_stride = out_dim, filter_size, feat_stride
        self.norm_scale = math.sqrt(1.0 / (out_dim * filter_size * filter_size))

        def bn(pre):
            return [sd[pre + s] for s in (".weight", ".bias", ".running_mean", ".running_var")]
        self.backbones = []
        for fe in ("feature_extractor", "feature_extractor_depth"):
            stem = _Conv(sd[fe + ".conv1.weight"], bn(fe + ".bn1"), stride=2, pad=3, dev=self.dev, f16x3=f16)
            blocks = []
            for li, (planes, nb, stride) in enumerate(RESNET50_LAYERS):
                for b in range(nb):
                    pre = f"{fe}.layer{li + 1}.{b}"
                    s = stride if b == 0 else 1
                    c1 = _Conv(sd[pre + ".conv1.weight"], bn(pre + ".bn1"), dev=self.dev, f16x3=f16)
                    c2 = _Conv(sd[pre + ".conv2.weight"], bn(pre + ".bn2"), stride=s, pad=1, dev=self.dev, f16x3=f16)
                    c3 = _Conv(sd[pre + ".conv3.weight"], bn(pre + ".bn3"), dev=self.dev, f16x3=f16)
                    ds = _Conv(sd[pre + ".downsample.0.weight"], bn(pre + ".downsample.1"), stride=s, dev=self.dev,
                               f16x3=f16) if b == 0 else None
                    blocks.append((c1, c2, c3, ds, _ConvDs(c3, ds, self.dev) if (f16 and ds is not None) else None))
            self.backbones.append((stem, blocks))
        self.clf = _Conv(sd["classifier.feature_extractor.0.weight"], pad=1, dev=self.dev, f16x3=f16)
        self.fconv = _Conv(sd["classifier.filter_initializer.filter_conv.weight"], pad=1,
                           bias=sd["classifier.filter_initializer.filter_conv.bias"], dev=self.dev, f16x3=f16)
        # f16x3 activation range: sharded max|y| words per produced tensor, zeroed once per extract_backbone;
        # the normalised image and the InstanceL2Norm output have static bounds
        self._max_words = torch.zeros(128 * MAX_WORDS, dtype=torch.float32, device=self.dev) if f16 else None
        self._nslot = 0
        self.image_scale = range_scale(max((1 - m) / s for m, s in zip(MEAN, STD)))
        self.l2_scale = lambda L: range_scale(self.norm_scale * math.sqrt(L))
        self._mean = (ctypes.c_float * 3)(*MEAN)
        self._std = (ctypes.c_float * 3)(*STD)
        self._bufs = {}

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _buf(self, name, n):
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = self._bufs[name] = torch.empty(n, dtype=torch.float32, device=self.dev)
        return b[:n]

    def _slot(self):
        """The next tensor's sharded max words (f16x3), or None in fp32 mode."""
        if self._max_words is None:
            return None
        k = self._nslot
        self._nslot += 1
        if (k + 1) * MAX_WORDS > self._max_words.numel():
            raise RuntimeError("DiMPNet: out of max-word slots")
        return self._max_words[k * MAX_WORDS:(k + 1) * MAX_WORDS]

    def _ws(self, nbytes):
        return self._buf("splitk", (nbytes + 3) // 4)

    def _layer(self, convs, kws, N, H, W, s, cin=None):
        """The same layer of each backbone: f16x3 runs the twins as one grouped launch (unless one merges into
        the other's output); fp32 runs them in backbone order.  cin: the f16x3 input's channel count when it
        differs from the conv's (4: the padded image)."""
        if self.precision == "f16x3" and len(convs) > 1 and not any(kw.get("merge_max") for kw in kws):
            run_f16x3(self.lib, convs[0], [c.group(**kw) for c, kw in zip(convs, kws)], N, H, W, self._ws, s, cin)
            return
        for c, kw in zip(convs, kws):
            c(self.lib, kw.pop("x"), N, H, W, kw.pop("out"), s, ws=self._ws, **kw)

    def _resnets(self, xs, N, H, W, out, s, out_max):
        """Both ResNet-50s to layer3, layer by layer, of NHWC xs[k] [N, H, W, 3]; the RGB backbone writes out
        [N, H/16, W/16, 1024] and the aux backbone's last conv max-merges into it (dimpnet.py:103).  f16x3: every
        conv reads its input's max words and accumulates its output's (out_max for layer3, shared by the two
        backbones so it bounds the merged map)."""
        lib = self.lib
        K = range(len(self.backbones))
        stems = [bb[0] for bb in self.backbones]
        h, w = stems[0].out_hw(H, W)
        t0_max = [self._slot() for k in K]
        f16 = self.precision == "f16x3"   # f16x3: the images come padded to 4 channels
        H2, W2 = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
        cur = [self._buf(f"ping{k}", N * H2 * W2 * 256) for k in K]
        if f16 and STEM_POOL:   # the max-pool fused into the stem: the full-resolution map is never written
            self._layer(stems, [dict(x=xs[k], out=cur[k], relu=True, x_scale=self.image_scale, y_max=t0_max[k],
                                     pool=True) for k in K], N, H, W, s, cin=4)
        else:
            t0 = [self._buf(f"stem{k}", N * h * w * 64) for k in K]
            self._layer(stems, [dict(x=xs[k], out=t0[k], relu=True, x_scale=self.image_scale, y_max=t0_max[k])
                                for k in K], N, H, W, s, cin=4 if f16 else None)
            for k in K:
                _rc(lib.mmt_maxpool2d_f32(_p(t0[k]), N, h, w, 64, 3, 2, 1, _p(cur[k]), s), "mmt_maxpool2d_f32")
        cur_max = t0_max   # a max-pool never exceeds its input's maximum
        H, W = H2, W2
        nxt_name = "pong"
        nblocks = len(self.backbones[0][1])
        for i in range(nblocks):
            c1s, c2s, c3s, dss, fus = zip(*[bb[1][i] for bb in self.backbones])
            Ho, Wo = c2s[0].out_hw(H, W)
            a = [self._buf(f"a{k}", N * H * W * c1s[0].cout) for k in K]
            a_max = [self._slot() for k in K]
            self._layer(c1s, [dict(x=cur[k], out=a[k], relu=True, x_max=cur_max[k], y_max=a_max[k]) for k in K],
                        N, H, W, s)
            b = [self._buf(f"b{k}", N * Ho * Wo * c2s[0].cout) for k in K]
            b_max = [self._slot() for k in K]
            self._layer(c2s, [dict(x=a[k], out=b[k], relu=True, x_max=a_max[k], y_max=b_max[k]) for k in K],
                        N, H, W, s)
            last = i == nblocks - 1
            fused = fus[0] is not None and DS_FUSE and not last
            if fused:   # conv3 + downsample in one GEMM: relu(conv3(b) + ds(cur) + b3 + b_d)
                o = [self._buf(f"{nxt_name}{k}", N * Ho * Wo * c3s[0].cout) for k in K]
                o_max = [self._slot() for k in K]
                fus[0].run(lib, [fu.group(b[k], o[k], x_max=b_max[k], y_max=o_max[k]) for k, fu in zip(K, fus)],
                           [(cur[k], cur_max[k]) for k in K], N, Ho, Wo, H, W, self._ws, s)
                cur, cur_max, nxt_name = o, o_max, ("ping" if nxt_name == "pong" else "pong")
                H, W = Ho, Wo
                continue
            if dss[0] is not None:
                res = [self._buf(f"res{k}", N * Ho * Wo * dss[0].cout) for k in K]
                # only ever a residual operand: no max words
                self._layer(dss, [dict(x=cur[k], out=res[k], x_max=cur_max[k]) for k in K], N, H, W, s)
            else:
                res = cur
            if last:
                o, o_max = [out] * len(K), [out_max] * len(K)
                for k in K:   # the RGB map first, then the aux map merged into it
                    self._layer([c3s[k]], [dict(x=b[k], out=out, relu=True, resid=res[k], merge_max=k > 0,
                                                x_max=b_max[k], y_max=out_max)], N, Ho, Wo, s)
            else:
                o = [self._buf(f"{nxt_name}{k}", N * Ho * Wo * c3s[0].cout) for k in K]
                o_max = [self._slot() for k in K]
                self._layer(c3s, [dict(x=b[k], out=o[k], relu=True, resid=res[k], x_max=b_max[k], y_max=o_max[k])
                                  for k in K], N, Ho, Wo, s)
            cur, cur_max, nxt_name = o, o_max, ("ping" if nxt_name == "pong" else "pong")
            H, W = Ho, Wo
        return H, W

    def flops(self, H=288, W=288):
        """Algorithmic FLOPs (2 x MACs) of extract_backbone + extract_classification_feat for one [6, H, W] image."""
        total = 0
        for stem, blocks in self.backbones:
            h, w = stem.out_hw(H, W)
            total += 2 * h * w * stem.cout * stem.kh * stem.kw * stem.cin
            h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
            for c1, c2, c3, ds, _ in blocks:
                ho, wo = c2.out_hw(h, w)
                total += 2 * h * w * c1.cout * c1.cin
                total += 2 * ho * wo * c2.cout * 9 * c2.cin
                total += 2 * ho * wo * c3.cout * c3.cin
                if ds is not None:
                    total += 2 * ho * wo * ds.cout * ds.cin
                h, w = ho, wo
        return total + 2 * h * w * self.clf.cout * 9 * self.clf.cin

    def layer_work(self, H=288, W=288):
        """(FLOPs, minimum HBM bytes) of every conv and max-pool of extract_backbone + the clf conv for one
        [6, H, W] image: each layer's input read once, its output written once (and read back by the MAX merge),
        the residual read, fp32 activations, f16x3 weights (hi + lo, read once per launch -- amortised over
        the batch, so not counted per image).  The per-layer roofline of a batch is the sum over layers of
        max(FLOPs / matrix peak, bytes / HBM bandwidth).  (The reference's layers as the yardstick: the fused
        conv3 + downsample of the f16x3 path moves fewer bytes than the two layers it replaces.)"""
        out = []
        for bi, (stem, blocks) in enumerate(self.backbones):
            h, w = stem.out_hw(H, W)
            out.append((2 * h * w * stem.cout * stem.kh * stem.kw * stem.cin, 4 * (H * W * 3 + h * w * stem.cout)))
            h2, w2 = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
            out.append((0, 4 * (h * w * 64 + h2 * w2 * 64)))   # max-pool
            h, w, cin = h2, w2, 64
            for k, (c1, c2, c3, ds, _) in enumerate(blocks):
                ho, wo = c2.out_hw(h, w)
                out.append((2 * h * w * c1.cout * c1.cin, 4 * (h * w * cin + h * w * c1.cout)))
                out.append((2 * ho * wo * c2.cout * 9 * c2.cin, 4 * (h * w * c2.cin + ho * wo * c2.cout)))
                merge = bi > 0 and k == len(blocks) - 1
                out.append((2 * ho * wo * c3.cout * c3.cin,
                            4 * (ho * wo * c3.cin + (3 if merge else 2) * ho * wo * c3.cout)))
                if ds is not None:
                    out.append((2 * ho * wo * ds.cout * ds.cin, 4 * (h * w * cin + ho * wo * ds.cout)))
                h, w, cin = ho, wo, c3.cout
        out.append((2 * h * w * self.clf.cout * 9 * self.clf.cin, 4 * (h * w * self.clf.cin + h * w * self.clf.cout)))
        return out

    def roofline_ms(self, n, peak_tflops, hbm_tbps, H=288, W=288):
        """The per-layer roofline time (ms) of extract_backbone + clf conv over a batch of n images."""
        return sum(max(n * f / (peak_tflops * 1e12), n * b / (hbm_tbps * 1e12)) for f, b in self.layer_work(H, W)) * 1e3

    # ------------------------------------------------------------------ the network's tracker-side entry points
    def extract_backbone(self, im):
        """im: [N, 6, H, W] fp32 CUDA pixel values (0..255) -> merged layer3 NHWC [N, H/16, W/16, 1024]."""
        if not (isinstance(im, torch.Tensor) and im.is_cuda and im.dtype == torch.float32 and im.dim() == 4
                and im.shape[1] == 6):
            raise ValueError("im must be an [N, 6, H, W] float32 CUDA tensor")
        im = im.contiguous()
        N, _, H, W = im.shape
        s = self._stream()
        f16 = self.precision == "f16x3"
        pc = 4 if f16 else 3   # f16x3: pixels padded to 4 channels (one 16-B load per stem tap)
        xa = self._buf("xa", N * H * W * pc)
        xb = self._buf("xb", N * H * W * pc)
        norm = self.lib.mmt_image_normalize4 if f16 else self.lib.mmt_image_normalize
        _rc(norm(_p(im), N, 6, H, W, self._mean, self._std, _p(xa), _p(xb), s), "mmt_image_normalize")
        return self._backbones(xa, xb, N, H, W, s)

    def norm4_buffers(self, N, H, W):
        """f16x3: the two normalised 4-channel NHWC halves [N*H*W*4] that extract_backbone_norm4 reads (a sampler
        that normalises, mmt_dimp_track_sample_norm4, writes them directly)."""
        if self.precision != "f16x3":
            raise ValueError("norm4 buffers: f16x3 only")
        return self._buf("xa", N * H * W * 4), self._buf("xb", N * H * W * 4)

    def max_words(self):
        """f16x3: the device words of every tensor's sharded max|y| (zeroed before each extract_backbone)."""
        return self._max_words

    def extract_backbone_norm4(self, N, H, W, words_cleared=False):
        """extract_backbone on the patches already normalised into norm4_buffers(N, H, W); words_cleared: the
        max words were zeroed by an earlier launch on the stream (the normalising sampler)."""
        xa, xb = self.norm4_buffers(N, H, W)
        return self._backbones(xa, xb, N, H, W, self._stream(), words_cleared)

    def _backbones(self, xa, xb, N, H, W, s, words_cleared=False):
        Hf, Wf = (H + 15) // 16, (W + 15) // 16
        out = torch.empty(N, Hf, Wf, 1024, dtype=torch.float32, device=self.dev)
        if self._max_words is not None:
            if not words_cleared:
                self._max_words.zero_()
            self._nslot = 0
        out_max = self._slot()
        h, w = self._resnets([xa, xb], N, H, W, out, s, out_max)
        assert (h, w) == (Hf, Wf)
        self._layer3_max = (out, out_max)
        return out

    def extract_classification_feat(self, layer3, nhwc=False):
        """layer3 NHWC [N, h, w, 1024] -> clf features [N, 512, h, w] (and the NHWC copy when nhwc=True)."""
        N, h, w, _ = layer3.shape
        s = self._stream()
        t = self._buf("clf", N * h * w * self.out_dim)
        lm = getattr(self, "_layer3_max", None)
        if self.precision == "f16x3" and (lm is None or lm[0] is not layer3):
            raise ValueError("f16x3: extract_classification_feat takes the layer3 map of the last extract_backbone")
        self.clf(self.lib, layer3, N, h, w, t, s, x_max=lm[1] if lm else None, ws=self._ws)
        out = torch.empty(N, self.out_dim, h, w, dtype=torch.float32, device=self.dev)
        out_nhwc = torch.empty(N, h, w, self.out_dim, dtype=torch.float32, device=self.dev) if nhwc else None
        l2ws = self._buf("l2ws", (self.lib.mmt_instance_l2norm_ws_bytes(N, h, w) + 3) // 4)
        _rc(self.lib.mmt_instance_l2norm(_p(t), N, h, w, self.out_dim, self.norm_scale, 1e-5, _p(out_nhwc), _p(out),
                                         _p(l2ws), s), "mmt_instance_l2norm")
        return (out, out_nhwc) if nhwc else out

    def init_filter(self, feat_nhwc, bb):
        """feat_nhwc [N, h, w, 512] (extract_classification_feat(..., nhwc=True)[1]); bb [N, 4] xywh (sample
        coordinates) -> filter [1, 512, fs, fs]."""
        N, h, w, C = feat_nhwc.shape
        s = self._stream()
        f = self._buf("fconv", N * h * w * C)
        # the InstanceL2Norm output: |y| <= norm_scale * sqrt(C h w) (normalization.py:6-21)
        self.fconv(self.lib, feat_nhwc, N, h, w, f, s, x_scale=self.l2_scale(C * h * w), ws=self._ws)
        bb = torch.as_tensor(bb, dtype=torch.float32).reshape(-1, 4).clone()
        bb[:, 2:4] = bb[:, 0:2] + bb[:, 2:4]
        rois = bb.to(self.dev)
        fs = self.filter_size
        pooled = torch.empty(N, C, fs, fs, dtype=torch.float32, device=self.dev)
        _rc(self.lib.mmt_prroi_pool(_p(f), N, h, w, C, _p(rois), 1.0 / self.feat_stride, fs, fs, _p(pooled), s),
            "mmt_prroi_pool")
        return pooled.mean(0, keepdim=True) if N > 1 else pooled

    def classify(self, weights, feat):
        from .dimp import apply_filter
        return apply_filter(feat.reshape(-1, 1, *feat.shape[-3:]), weights)


def sample_patch_device(frame, geom, out_hw):
    """mmt_sample_patch: frame H x W x C uint8 CUDA tensor, geom (df, os_y, os_x, tl_y, tl_x, sz_h, sz_w)
    -> [1, C, out_h, out_w] fp32 CUDA tensor."""
    lib = _lib.load()
    H, W, C = frame.shape
    out = torch.empty(1, C, int(out_hw[0]), int(out_hw[1]), dtype=torch.float32, device=frame.device)
    g = (ctypes.c_int * 7)(*[int(v) for v in geom])
    _rc(lib.mmt_sample_patch(_p(frame), H, W, C, frame.stride(0), g, int(out_hw[0]), int(out_hw[1]), _p(out),
                             ctypes.c_void_p(torch.cuda.current_stream(frame.device).cuda_stream)), "mmt_sample_patch")
    return out


def patch_transform_device(img, tf, out_hw):
    """mmt_patch_transform of a [1, C, E_h, E_w] fp32 CUDA patch with one _lib.MmtPatchTf -> [1, C, oh, ow]."""
    lib = _lib.load()
    _, C, Eh, Ew = img.shape
    img = img.contiguous()
    out = torch.empty(1, C, int(out_hw[0]), int(out_hw[1]), dtype=torch.float32, device=img.device)
    _rc(lib.mmt_patch_transform(_p(img), C, Eh, Ew, ctypes.byref(tf), int(out_hw[0]), int(out_hw[1]), _p(out),
                                ctypes.c_void_p(torch.cuda.current_stream(img.device).cuda_stream)),
        "mmt_patch_transform")
    return out


def conv2d(x_nchw, w, bias=None, stride=1, pad=0, resid=None, relu=False, w4=True, precision="fp32", x_max=None,
           y_max=None, split=False, merge_into=None):
    """Test / tool helper: torch NCHW conv through mmt_conv2d_f32 or (precision "f16x3") mmt_conv2d_f16x3
    (weights nn.Conv2d layout; f16x3 input range: x_max words, else the static scale of max|x|; split: give the
    library a split-K workspace; merge_into: an NHWC map the output is max-merged into (and returned))."""
    lib = _lib.load()
    f16 = precision == "f16x3"
    conv = _Conv(w, bias=bias, stride=stride, pad=pad, dev=x_nchw.device, w4=w4, f16x3=f16)
    N, C, H, W = x_nchw.shape
    Ho, Wo = conv.out_hw(H, W)
    x = x_nchw.permute(0, 2, 3, 1).contiguous()
    out = merge_into if merge_into is not None else torch.empty(N, Ho, Wo, conv.cout, dtype=torch.float32,
                                                                device=x.device)
    r = resid.permute(0, 2, 3, 1).contiguous() if resid is not None else None
    kw = {}
    if f16:
        kw = dict(x_max=x_max, x_scale=0.0 if x_max is not None else range_scale(float(x.abs().max())), y_max=y_max)
        if split:
            kw["ws"] = lambda n: torch.empty((n + 3) // 4, dtype=torch.float32, device=x.device)
    conv(lib, x, N, H, W, out, ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream), relu=relu, resid=r,
         merge_max=merge_into is not None, **kw)
    return out.permute(0, 3, 1, 2)


def prroi_pool(feat_nchw, rois_xyxy, spatial_scale, ph, pw):
    """Test helper: PrRoIPool2D of roi n on image n."""
    lib = _lib.load()
    N, C, H, W = feat_nchw.shape
    f = feat_nchw.permute(0, 2, 3, 1).contiguous()
    out = torch.empty(N, C, ph, pw, dtype=torch.float32, device=f.device)
    r = torch.as_tensor(rois_xyxy, dtype=torch.float32).reshape(N, 4).to(f.device)
    _rc(lib.mmt_prroi_pool(_p(f), N, H, W, C, _p(r), spatial_scale, ph, pw, _p(out),
                           ctypes.c_void_p(torch.cuda.current_stream(f.device).cuda_stream)), "mmt_prroi_pool")
    return out


__all__ = ["DiMPNet", "sample_patch_device", "patch_transform_device", "conv2d", "prroi_pool"]
