"""CPU restatement of the DeT / mfDiMP DiMP-50 classification path (TEST ORACLE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline import this module.  mfDiMP's own
source is absent (RGBT/models/end2end_rgbt_tracking/ is an empty submodule); the in-tree multi-modal
DiMP is DeT's, whose pieces this restates in fp32 torch on the CPU:

* ``preprocess``        pytracking/features/net_wrappers.py:55-79 (each 3-channel half /255, -mean, /std)
* ``resnet_layer3``     ltr/models/backbone/resnet.py (conv1 7x7/2 + BN + ReLU, maxpool 3x3/2, Bottleneck
                        layer1..layer3 with the stride on the 3x3 conv and a 1x1 downsample)
* ``backbone``          ltr/models/tracking/dimpnet.py:88-133 (RGB / aux backbones, merge_type 'max')
* ``clf_features``      ltr/models/target_classifier/features.py:47-66 (final 3x3 conv, no bias) +
                        ltr/models/layers/normalization.py:6-21 (InstanceL2Norm, size_average)
* ``prroi_pool``        ltr/external/PreciseRoIPooling/src/prroi_pooling_gpu_impl.cu:37-212 (forward)
* ``init_filter``       ltr/models/target_classifier/initializer.py:118-170 (FilterInitializerLinear)
* ``sample_patch``      pytracking/features/preprocessing.py:49-125
Pinned by tests/golden/dimpnet_deT.npz (the reference DiMPnet_DeT run on the same seeded weights);
PrRoIPool (a CUDA extension) is pinned only to this restatement.
"""
import math

import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
LAYERS = ((64, 3, 1), (128, 4, 2), (256, 6, 2))


def preprocess(im):
    """im: [N, 6, H, W] pixel values -> normalised (net_wrappers.py:62-72)."""
    mean = torch.tensor(MEAN).view(1, -1, 1, 1)
    std = torch.tensor(STD).view(1, -1, 1, 1)
    halves = []
    for h in (im[:, :3], im[:, 3:]):
        h = h / 255
        h = h - mean
        h = h / std
        halves.append(h)
    return torch.cat(halves, 1)


def _bn(x, sd, pre, eps=1e-5):
    return F.batch_norm(x, sd[pre + ".running_mean"], sd[pre + ".running_var"], sd[pre + ".weight"], sd[pre + ".bias"],
                        False, 0.0, eps)


def _bottleneck(x, sd, pre, stride, down):
    out = F.relu(_bn(F.conv2d(x, sd[pre + ".conv1.weight"]), sd, pre + ".bn1"))
    out = F.relu(_bn(F.conv2d(out, sd[pre + ".conv2.weight"], stride=stride, padding=1), sd, pre + ".bn2"))
    out = _bn(F.conv2d(out, sd[pre + ".conv3.weight"]), sd, pre + ".bn3")
    res = _bn(F.conv2d(x, sd[pre + ".downsample.0.weight"], stride=stride), sd, pre + ".downsample.1") if down else x
    return F.relu(out + res)


def resnet_layer3(x, sd, fe):
    x = F.relu(_bn(F.conv2d(x, sd[fe + ".conv1.weight"], stride=2, padding=3), sd, fe + ".bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, (planes, blocks, stride) in enumerate(LAYERS):
        for b in range(blocks):
            x = _bottleneck(x, sd, f"{fe}.layer{li + 1}.{b}", stride if b == 0 else 1, b == 0)
    return x


def backbone(im_norm, sd):
    """merged layer3 features [N, 1024, H/16, W/16] of a normalised [N, 6, H, W] batch."""
    return torch.max(resnet_layer3(im_norm[:, :3], sd, "feature_extractor"),
                     resnet_layer3(im_norm[:, 3:], sd, "feature_extractor_depth"))


def instance_l2norm(x, scale, eps=1e-5):
    return x * (scale * ((x.shape[1] * x.shape[2] * x.shape[3]) / (
        torch.sum((x * x).view(x.shape[0], 1, 1, -1), dim=3, keepdim=True) + eps)).sqrt())


def clf_features(layer3, sd, out_dim=512, filter_size=4):
    norm_scale = math.sqrt(1.0 / (out_dim * filter_size * filter_size))
    return instance_l2norm(F.conv2d(layer3, sd["classifier.feature_extractor.0.weight"], padding=1), norm_scale)


def _prroi_get(d, h, w):
    if h < 0 or w < 0 or h >= d.shape[-2] or w >= d.shape[-1]:
        return torch.zeros(d.shape[0])
    return d[:, h, w]


def _prroi_cell(d, sh, sw, eh, ew, y0, x0, y1, x1):
    def f(a, b):
        return torch.tensor(a, dtype=torch.float32) - 0.5 * torch.tensor(a, dtype=torch.float32) ** 2 - \
            torch.tensor(b, dtype=torch.float32) + 0.5 * torch.tensor(b, dtype=torch.float32) ** 2
    out = _prroi_get(d, sh, sw) * (f(x1 - sw, x0 - sw) * f(y1 - sh, y0 - sh))
    out = out + _prroi_get(d, sh, ew) * (f(ew - x0, ew - x1) * f(y1 - sh, y0 - sh))
    out = out + _prroi_get(d, eh, sw) * (f(x1 - sw, x0 - sw) * f(eh - y0, eh - y1))
    out = out + _prroi_get(d, eh, ew) * (f(ew - x0, ew - x1) * f(eh - y0, eh - y1))
    return out


def prroi_pool(feat, rois, spatial_scale, ph=4, pw=4):
    """feat [N, C, H, W]; rois [R, 5] = (batch index, x0, y0, x1, y1) -> [R, C, ph, pw]."""
    out = torch.zeros(rois.shape[0], feat.shape[1], ph, pw)
    for r in range(rois.shape[0]):
        d = feat[int(rois[r, 0])]
        sw_, sh_ = float(rois[r, 1]) * spatial_scale, float(rois[r, 2]) * spatial_scale
        ew_, eh_ = float(rois[r, 3]) * spatial_scale, float(rois[r, 4]) * spatial_scale
        bw, bh = max(ew_ - sw_, 0.0) / pw, max(eh_ - sh_, 0.0) / ph
        area = max(0.0, bw * bh)
        if area == 0:
            continue
        for i in range(ph):
            for j in range(pw):
                ws, hs = sw_ + bw * j, sh_ + bh * i
                we, he = ws + bw, hs + bh
                acc = torch.zeros(feat.shape[1])
                for wi in range(math.floor(ws), math.ceil(we)):
                    for hi in range(math.floor(hs), math.ceil(he)):
                        acc = acc + _prroi_cell(d, hi, wi, hi + 1, wi + 1, max(hs, hi), max(ws, wi), min(he, hi + 1.0),
                                                min(we, wi + 1.0))
                out[r, :, i, j] = acc / area
    return out


def init_filter(clf_feat, boxes, sd, filter_size=4, feat_stride=16):
    """FilterInitializerLinear: conv3x3 (+bias) -> PrRoIPool of the xywh boxes -> mean over images."""
    f = F.conv2d(clf_feat, sd["classifier.filter_initializer.filter_conv.weight"],
                 sd["classifier.filter_initializer.filter_conv.bias"], padding=1)
    bb = boxes.reshape(-1, 4).clone()
    bb[:, 2:4] = bb[:, 0:2] + bb[:, 2:4]
    rois = torch.cat([torch.arange(bb.shape[0], dtype=torch.float32).view(-1, 1), bb], 1)
    w = prroi_pool(f, rois, 1.0 / feat_stride, filter_size, filter_size)
    return w.mean(0, keepdim=True) if w.shape[0] > 1 else w


def patch_geometry(im_hw, pos, sample_sz, output_sz):
    """sample_patch's integer geometry (preprocessing.py:69-104, mode 'replicate'):
    (df, os_y, os_x, tl_y, tl_x, sz_h, sz_w) in the df-strided image."""
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
    return [df, int(os_[0]), int(os_[1]), int(tl[0]), int(tl[1]), int(szl[0]), int(szl[1])]


def sample_patch(im, pos, sample_sz, output_sz):
    """The reference's replicate-mode sample_patch on an [1, C, H, W] float image."""
    posl = pos.long().clone()
    resize_factor = torch.min(sample_sz.float() / output_sz.float()).item()
    df = int(max(int(resize_factor - 0.1), 1))
    sz = sample_sz.float() / df
    if df > 1:
        os_ = posl % df
        posl = (posl - os_) // df
        im2 = im[..., os_[0].item()::df, os_[1].item()::df]
    else:
        im2 = im
    szl = torch.max(sz.round(), torch.Tensor([2])).long()
    tl = posl - (szl - 1) // 2
    br = posl + szl // 2 + 1
    im_patch = F.pad(im2, (-tl[1].item(), br[1].item() - im2.shape[3], -tl[0].item(), br[0].item() - im2.shape[2]),
                     'replicate')
    patch_coord = df * torch.cat((tl, br)).view(1, 4)
    if im_patch.shape[-2] == output_sz[0] and im_patch.shape[-1] == output_sz[1]:
        return im_patch.clone(), patch_coord
    return F.interpolate(im_patch, output_sz.long().tolist(), mode='bilinear'), patch_coord


def warp_affine_replicate(img, M, dsize):
    """cv2.warpAffine(img, M, dsize, flags=INTER_LINEAR, borderMode=BORDER_REPLICATE) for a float32 H x W x C
    image (OpenCV imgwarp.cpp, restated: M inverted to dst -> src in double, source coordinates in 1/32-pixel
    fixed point -- AB_BITS 10, INTER_BITS 5, round_delta 16 --, bilinear weights of the 32 x 32 table,
    replicated border).  OpenCV is absent from this image: parity unpinned at this boundary."""
    import numpy as np
    M = [float(v) for v in np.asarray(M, dtype=np.float64).reshape(-1)]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0], M[1], M[3], M[4] = A11, M[1] * -D, M[3] * -D, A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    W, H = dsize
    ys = np.arange(H, dtype=np.float64).reshape(-1, 1)
    xs = np.arange(W, dtype=np.float64).reshape(1, -1)
    X0 = np.rint((M[1] * ys + M[2]) * 1024.0).astype(np.int64) + 16
    Y0 = np.rint((M[4] * ys + M[5]) * 1024.0).astype(np.int64) + 16
    X = (X0 + np.rint(M[0] * xs * 1024.0).astype(np.int64)) >> 5
    Y = (Y0 + np.rint(M[3] * xs * 1024.0).astype(np.int64)) >> 5
    sx, sy = X >> 5, Y >> 5
    ax = ((X & 31).astype(np.float32) * np.float32(1.0 / 32))[..., None]
    ay = ((Y & 31).astype(np.float32) * np.float32(1.0 / 32))[..., None]
    h, w = img.shape[:2]
    x0, x1 = np.clip(sx, 0, w - 1), np.clip(sx + 1, 0, w - 1)
    y0, y1 = np.clip(sy, 0, h - 1), np.clip(sy + 1, 0, h - 1)
    one = np.float32(1.0)
    w00, w01, w10, w11 = (one - ay) * (one - ax), (one - ay) * ax, ay * (one - ax), ay * ax
    out = img[y0, x0] * w00 + img[y0, x1] * w01 + img[y1, x0] * w10 + img[y1, x1] * w11
    return out.astype(np.float32)
