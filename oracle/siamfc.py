"""CPU restatement of the SiamFC tracker (TEST ORACLE) -- parity unpinned.

The reference's RGBE/models/siamfc/ is an empty, un-vendored submodule (only ``python test.py``
is named, RGBE/benchmark.py:42-49; the paper is cited at readme.md:47). Its upstream module and
pinned version are unknown, so this restates the published SiamFC tracker in the form of the
widely used PyTorch implementation (TrackerSiamFC: AlexNetV1 backbone, ``_fast_xcorr`` head with
out_scale 1e-3, 3-scale search, x16 INTER_CUBIC upsampling, cosine window):
* ``crop_and_resize`` -- square window round(size) at round(center - (size-1)/2), constant border
  of the frame's mean colour, cv2 INTER_LINEAR (oracle.crop.cv2_resize_linear_u8);
* ``cv2_resize_cubic_f32`` -- cv::resize INTER_CUBIC on CV_32F (A = -0.75, replicate borders);
* ``alexnet`` / ``xcorr`` -- torch fp32 CPU; ``OracleSiamFC`` -- init / update.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .crop import cv2_resize_linear_u8

CFG = dict(out_scale=0.001, exemplar_sz=127, instance_sz=255, context=0.5, scale_num=3, scale_step=1.0375,
           scale_lr=0.59, scale_penalty=0.9745, window_influence=0.176, response_sz=17, response_up=16,
           total_stride=8)


def crop_and_resize(img, center, size, out_size, border_value):
    size = round(size)
    c0 = np.round(center - (size - 1) / 2)
    corners = np.round(np.concatenate((c0, c0 + size))).astype(int)
    pads = np.concatenate((-corners[:2], corners[2:] - np.array(img.shape[:2])))
    npad = max(0, int(pads.max()))
    if npad > 0:
        bv = np.clip(np.rint(np.asarray(border_value, dtype=np.float64)), 0, 255).astype(np.uint8)
        padded = np.empty((img.shape[0] + 2 * npad, img.shape[1] + 2 * npad, img.shape[2]), dtype=np.uint8)
        padded[...] = bv
        padded[npad:npad + img.shape[0], npad:npad + img.shape[1]] = img
        img = padded
    corners = (corners + npad).astype(int)
    patch = img[corners[0]:corners[2], corners[1]:corners[3]]
    return cv2_resize_linear_u8(patch, out_size, out_size)


def _cubic_coeffs(x):
    A = np.float32(-0.75)
    x = np.float32(x)
    one = np.float32(1.0)
    x1 = x + one
    omx = one - x
    c0 = ((A * x1 - np.float32(5.0) * A) * x1 + np.float32(8.0) * A) * x1 - np.float32(4.0) * A
    c1 = ((A + np.float32(2.0)) * x - (A + np.float32(3.0))) * x * x + one
    c2 = ((A + np.float32(2.0)) * omx - (A + np.float32(3.0))) * omx * omx + one
    c3 = one - c0 - c1 - c2
    return np.array([c0, c1, c2, c3], dtype=np.float32)


def cv2_resize_cubic_f32(src, out):
    """cv2.resize(src, (out, out), interpolation=INTER_CUBIC) for a square float32 map."""
    S = src.shape[0]
    scale = 1.0 / (float(out) / float(S))
    idx, coef = [], []
    for d in range(out):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        idx.append([min(max(s + k - 1, 0), S - 1) for k in range(4)])
        coef.append(_cubic_coeffs(f))
    idx = np.array(idx)
    coef = np.array(coef, dtype=np.float32)
    src = src.astype(np.float32)
    # horizontal: h[r, ox] = sum_k src[r, idx[ox,k]] * coef[ox,k]  (left-to-right float32 adds)
    h = src[:, idx[:, 0]] * coef[None, :, 0]
    for k in range(1, 4):
        h = h + src[:, idx[:, k]] * coef[None, :, k]
    v = h[idx[:, 0], :] * coef[:, 0, None]
    for k in range(1, 4):
        v = v + h[idx[:, k], :] * coef[:, k, None]
    return v.astype(np.float32)


def alexnet(sd, x):
    """AlexNetV1 (BN eps 1e-6, eval) on an N x 3 x H x W float tensor."""
    def bn(y, p):
        return F.batch_norm(y, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                            False, 0.0, 1e-6)

    def conv(y, p, stride=1, groups=1):
        return F.conv2d(y, sd[p + ".weight"], sd[p + ".bias"], stride=stride, groups=groups)

    b = "backbone."
    x = F.max_pool2d(F.relu(bn(conv(x, b + "conv1.0", 2), b + "conv1.1")), 3, 2)
    x = F.max_pool2d(F.relu(bn(conv(x, b + "conv2.0", 1, 2), b + "conv2.1")), 3, 2)
    x = F.relu(bn(conv(x, b + "conv3.0"), b + "conv3.1"))
    x = F.relu(bn(conv(x, b + "conv4.0", 1, 2), b + "conv4.1"))
    return conv(x, b + "conv5.0", 1, 2)


def xcorr(z, x, out_scale=0.001):
    """_fast_xcorr: F.conv2d(x.view(-1, nz*c, h, w), z, groups=nz) * out_scale."""
    nz = z.size(0)
    nx, c, h, w = x.size()
    out = F.conv2d(x.view(-1, nz * c, h, w), z, groups=nz)
    return out.view(nx, -1, out.size(-2), out.size(-1)) * out_scale


def response_select(responses, cfg=CFG):
    """TrackerSiamFC.update post-correlation: -> (scale_id, (row, col), windowed value, response map)."""
    n = cfg["scale_num"]
    up = cfg["response_up"] * cfg["response_sz"]
    responses = np.stack([cv2_resize_cubic_f32(u, up) for u in responses])
    responses[:n // 2] *= cfg["scale_penalty"]
    responses[n // 2 + 1:] *= cfg["scale_penalty"]
    scale_id = int(np.argmax(np.amax(responses, axis=(1, 2))))
    response = responses[scale_id]
    response -= response.min()
    response /= response.sum() + 1e-16
    hann = np.outer(np.hanning(up), np.hanning(up))
    hann /= hann.sum()
    response = (1 - cfg["window_influence"]) * response + cfg["window_influence"] * hann
    loc = np.unravel_index(response.argmax(), response.shape)
    return scale_id, (int(loc[0]), int(loc[1])), float(response[loc]), response


class OracleSiamFC:
    def __init__(self, state_dict, cfg=CFG):
        self.sd = {k: v.float() for k, v in state_dict.items()}
        self.cfg = dict(cfg)

    def init(self, img, box):
        c = self.cfg
        img = img[..., :3]
        box = np.array([box[1] - 1 + (box[3] - 1) / 2, box[0] - 1 + (box[2] - 1) / 2, box[3], box[2]],
                       dtype=np.float32)
        self.center, self.target_sz = box[:2], box[2:]
        self.upscale_sz = c["response_up"] * c["response_sz"]
        n = c["scale_num"]
        self.scale_factors = c["scale_step"] ** np.linspace(-(n // 2), n // 2, n)
        context = c["context"] * np.sum(self.target_sz)
        self.z_sz = np.sqrt(np.prod(self.target_sz + context))
        self.x_sz = self.z_sz * c["instance_sz"] / c["exemplar_sz"]
        self.avg_color = np.mean(img, axis=(0, 1))
        z = crop_and_resize(img, self.center, self.z_sz, c["exemplar_sz"], self.avg_color)
        zt = torch.from_numpy(z).permute(2, 0, 1).unsqueeze(0).float()
        self.kernel = alexnet(self.sd, zt)
        self.last_z = z

    def update(self, img):
        c = self.cfg
        img = img[..., :3]
        x = np.stack([crop_and_resize(img, self.center, self.x_sz * f, c["instance_sz"], self.avg_color)
                      for f in self.scale_factors])
        self.last_x = x
        xt = torch.from_numpy(x).permute(0, 3, 1, 2).float()
        responses = xcorr(self.kernel, alexnet(self.sd, xt), c["out_scale"]).squeeze(1).numpy()
        self.last_responses = responses
        scale_id, loc, val, _ = response_select(responses, c)
        disp_in_response = np.array(loc) - (self.upscale_sz - 1) / 2
        disp_in_instance = disp_in_response * c["total_stride"] / c["response_up"]
        disp_in_image = disp_in_instance * self.x_sz * self.scale_factors[scale_id] / c["instance_sz"]
        self.center = self.center + disp_in_image
        scale = (1 - c["scale_lr"]) * 1.0 + c["scale_lr"] * self.scale_factors[scale_id]
        self.target_sz = self.target_sz * scale
        self.z_sz = self.z_sz * scale
        self.x_sz = self.x_sz * scale
        return np.array([self.center[1] + 1 - (self.target_sz[1] - 1) / 2,
                         self.center[0] + 1 - (self.target_sz[0] - 1) / 2,
                         self.target_sz[1], self.target_sz[0]])
