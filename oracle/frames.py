"""CPU restatement of the RGB-D frame assembly (TEST ORACLE; parity unpinned at the OpenCV boundary).

get_rgbd_frame(color, depth, dtype='rgbcolormap', depth_clip) -- ViPT/lib/train/dataset/depth_utils.py:7-58:
* depth clip (:20-22): max_depth = min(np.median(dp) * 3, 10000); dp[dp > max_depth] = max_depth
  (assignment into uint16 truncates);
* cv2.normalize(dp, None, 0, 255, NORM_MINMAX) (:47): scale = 255 / (max - min) (0 if equal),
  shift = -min * scale in double; OpenCV's convertTo computes dp * (float)scale + (float)shift in
  float and saturate_casts (round half to even) to uint16; np.asarray(.., uint8) keeps the low byte;
* cv2.applyColorMap(.., COLORMAP_JET) (:49): the published piecewise-linear JET table (BGR);
* cv2.merge((rgb, colormap)) (:50).
OpenCV is absent here, so its exact JET table and convertTo rounding are restated, not pinned.
"""
import numpy as np


def jet_bgr():
    x = np.arange(256) / 255.0
    r = np.clip(np.minimum(4 * x - 1.5, -4 * x + 4.5), 0, 1)
    g = np.clip(np.minimum(4 * x - 0.5, -4 * x + 3.5), 0, 1)
    b = np.clip(np.minimum(4 * x + 0.5, -4 * x + 2.5), 0, 1)
    return np.rint(np.stack([b, g, r], axis=1) * 255).astype(np.uint8)


def normalize_minmax_u8(dp):
    lo, hi = float(dp.min()), float(dp.max())
    scale = 255.0 / (hi - lo) if (hi - lo) > np.finfo(np.float64).eps else 0.0
    shift = 0.0 - lo * scale
    f = dp.astype(np.float32) * np.float32(scale) + np.float32(shift)
    v = np.clip(np.rint(f), 0, 65535).astype(np.int64)
    return (v & 0xFF).astype(np.uint8)


def rgbd_frame(rgb, dp, depth_clip=True, lut_bgr=None):
    dp = dp.copy()
    if depth_clip:
        max_depth = min(np.median(dp) * 3, 10000)
        dp[dp > max_depth] = max_depth
    d8 = normalize_minmax_u8(dp)
    lut = jet_bgr() if lut_bgr is None else np.asarray(lut_bgr, np.uint8).reshape(256, 3)
    return np.concatenate([rgb, lut[d8]], axis=2)
