"""CPU restatement of the search/template crop (TEST ORACLE).

* ``sample_target`` — ``ViPT/lib/train/data/processing_utils.py:14-81``
  (square crop, Python ``round`` corners, zero ``copyMakeBorder`` pad, resize).
* ``cv2_resize_linear_u8`` — OpenCV ``cv::resize(..., INTER_LINEAR)`` on
  CV_8U, restated from OpenCV 4.x ``imgproc/src/resize.cpp`` (the image pins
  ``opencv-python`` unversioned, ``install_vipt.sh:28``; OpenCV is absent
  here, so this restatement is *parity unpinned at the cv2 boundary*):

  - coefficients: ``fx = (float)((dx+0.5)*scale - 0.5)``, ``sx = floor(fx)``,
    ``fx -= sx``; x-borders clamp ``(sx, fx)`` to ``(0, 0)`` / ``(w-1, 0)``;
    y-borders clamp the row index only; ``alpha = cvRound((1-fx)*2048)``,
    ``cvRound(fx*2048)`` (INTER_RESIZE_COEF_BITS = 11);
  - horizontal pass: ``D = S[sx]*a0 + S[sx+1]*a1`` (int32);
  - vertical pass, SIMD body (``VResizeLinearVec_32s8u``, used for the whole
    row because every width here is a multiple of 32 bytes):
    ``u8((((D0>>4)*b0 >> 16) + ((D1>>4)*b1 >> 16) + 2) >> 2)``;
  - exact 2x down-scale is rerouted to INTER_AREA's fast path
    (``resize()``: ``is_area_fast && iscale == 2``): ``(a+b+c+d+2)>>2``.
* ``preprocess`` — ``PreprocessorMM.process`` (``ViPT/lib/test/tracker/data_utils.py:20-24``).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _coeffs(dsize: int, ssize: int, clamp_frac: bool):
    inv = float(dsize) / float(ssize)
    scale = 1.0 / inv
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp_frac:
        lo = s < 0
        f[lo] = 0.0
        s[lo] = 0
        hi = s >= ssize - 1
        f[hi] = 0.0
        s[hi] = ssize - 1
    one = np.float32(1.0)
    a0 = np.rint((one - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, a0, a1


def cv2_resize_linear_u8(src: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """``cv2.resize(src, (out_w, out_h))`` for an H x W x C uint8 image (see module doc)."""
    h, w = src.shape[:2]
    squeeze = src.ndim == 2
    if squeeze:
        src = src[..., None]
    scale_x = 1.0 / (float(out_w) / float(w))
    scale_y = 1.0 / (float(out_h) / float(h))
    if (abs(scale_x - 2.0) < np.finfo(np.float64).eps and abs(scale_y - 2.0) < np.finfo(np.float64).eps):
        s = src.astype(np.int32)
        o = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
        o = o[:out_h, :out_w].astype(np.uint8)
        return o[..., 0] if squeeze else o
    sx, a0, a1 = _coeffs(out_w, w, True)
    sy, b0, b1 = _coeffs(out_h, h, False)
    sx1 = np.minimum(sx + 1, w - 1)
    s = src.astype(np.int64)
    # horizontal pass on every source row
    D = s[:, sx, :] * a0[None, :, None] + s[:, sx1, :] * a1[None, :, None]
    r0 = np.clip(sy, 0, h - 1)
    r1 = np.clip(sy + 1, 0, h - 1)
    t0 = D[r0] >> 4
    t1 = D[r1] >> 4
    v = ((t0 * b0[:, None, None]) >> 16) + ((t1 * b1[:, None, None]) >> 16)
    o = np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)
    return o[..., 0] if squeeze else o


def crop_geometry(target_bb, search_area_factor: float, output_sz: int):
    """processing_utils.py:28-41, 69 — returns (x1, y1, crop_sz, resize_factor)."""
    x, y, w, h = [float(v) for v in target_bb]
    crop_sz = math.ceil(math.sqrt(w * h) * search_area_factor)
    if crop_sz < 1:
        raise Exception('Too small bounding box.')
    x1 = round(x + 0.5 * w - crop_sz * 0.5)
    y1 = round(y + 0.5 * h - crop_sz * 0.5)
    return x1, y1, crop_sz, output_sz / crop_sz


def sample_target(im: np.ndarray, target_bb, search_area_factor: float, output_sz: int):
    """processing_utils.py:14-81 (image path; the att_mask is not used by ViPT)."""
    x1, y1, crop_sz, resize_factor = crop_geometry(target_bb, search_area_factor, output_sz)
    x2 = x1 + crop_sz
    y2 = y1 + crop_sz
    x1_pad = max(0, -x1)
    x2_pad = max(x2 - im.shape[1] + 1, 0)
    y1_pad = max(0, -y1)
    y2_pad = max(y2 - im.shape[0] + 1, 0)
    im_crop = im[y1 + y1_pad:y2 - y2_pad, x1 + x1_pad:x2 - x2_pad, :]
    padded = np.zeros((im_crop.shape[0] + y1_pad + y2_pad, im_crop.shape[1] + x1_pad + x2_pad, im.shape[2]),
                      dtype=im.dtype)
    padded[y1_pad:y1_pad + im_crop.shape[0], x1_pad:x1_pad + im_crop.shape[1]] = im_crop
    return cv2_resize_linear_u8(padded, output_sz, output_sz), resize_factor


MEAN6 = [0.485, 0.456, 0.406, 0.485, 0.456, 0.406]
STD6 = [0.229, 0.224, 0.225, 0.229, 0.224, 0.225]


def preprocess(patch: np.ndarray) -> torch.Tensor:
    """``PreprocessorMM.process`` / ``Preprocessor.process`` on the CPU (data_utils.py:9-24)."""
    C = patch.shape[2]
    mean = torch.tensor(MEAN6[:C]).view((1, C, 1, 1))
    std = torch.tensor(STD6[:C]).view((1, C, 1, 1))
    t = torch.tensor(patch).float().permute((2, 0, 1)).unsqueeze(dim=0)
    return ((t / 255.0) - mean) / std
