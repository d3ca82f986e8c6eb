"""Multi-modal frame assembly (ViPT/lib/train/dataset/depth_utils.py:7-132) without OpenCV.

H x W x 6 uint8 frames: RGB, then the aux modality as 'rgbrgb' (aux image BGR->RGB), 'rgbcolormap'
(MINMAX-normalised depth through the JET colormap), 'rgb3x' ... .  Images are read with PIL
(cv2.imread returns BGR; the reference converts to RGB first, so the result is the same order).
The JET colormap and NORM_MINMAX follow OpenCV's published definitions (parity unpinned: OpenCV is
absent from the image)."""
import numpy as np


def _imread(path, unchanged=False):
    """cv2.imread(path) (IMREAD_COLOR: always 3 channels) + BGR2RGB for colour reads; cv2.imread(path, -1)
    (IMREAD_UNCHANGED: 16-bit depth and grayscale stay single-channel, palette images expand to colour)
    for the aux modality (depth_utils.py:79-85)."""
    from PIL import Image
    im = Image.open(path)
    if not unchanged:
        return np.asarray(im.convert('RGB'))
    if im.mode == 'P':
        im = im.convert('RGB')
    a = np.asarray(im)
    if a.ndim == 3 and a.shape[2] == 4:
        a = a[..., :3]
    return a


def normalize_minmax_u8(dp: np.ndarray) -> np.ndarray:
    """cv2.normalize(dp, None, 0, 255, NORM_MINMAX) followed by the uint8 cast of np.asarray: scale and
    shift in double, applied as OpenCV's convertTo does (float multiply-add, round half to even,
    saturate to the source type), then the low byte (the GPU path, mmt_rgbd_assemble, is identical)."""
    lo, hi = float(dp.min()), float(dp.max())
    scale = 255.0 / (hi - lo) if (hi - lo) > np.finfo(np.float64).eps else 0.0
    shift = 0.0 - lo * scale
    f = dp.astype(np.float32) * np.float32(scale) + np.float32(shift)
    top = 255 if dp.dtype == np.uint8 else 65535
    v = np.clip(np.rint(f), 0, top).astype(np.int64)
    return (v & 0xFF).astype(np.uint8)


def _jet_lut():
    # OpenCV COLORMAP_JET, as BGR output per value 0..255 (piecewise-linear r,g,b from 4 control points)
    x = np.arange(256) / 255.0
    r = np.clip(np.minimum(4 * x - 1.5, -4 * x + 4.5), 0, 1)
    g = np.clip(np.minimum(4 * x - 0.5, -4 * x + 3.5), 0, 1)
    b = np.clip(np.minimum(4 * x + 0.5, -4 * x + 2.5), 0, 1)
    return np.rint(np.stack([b, g, r], axis=1) * 255).astype(np.uint8)   # BGR like cv2


JET_BGR = _jet_lut()


def apply_colormap_jet(dp_u8: np.ndarray) -> np.ndarray:
    return JET_BGR[dp_u8]


def get_x_frame(color_path, depth_path, dtype='rgbcolormap', depth_clip=False):
    rgb = _imread(color_path) if color_path else None
    dp = _imread(depth_path, unchanged=True) if depth_path else None
    if dp is not None and depth_clip:
        max_depth = min(np.median(dp) * 3, 10000)
        dp = dp.copy()
        dp[dp > max_depth] = max_depth
    if dtype == 'color':
        return rgb
    if dtype == 'raw_x':
        return dp
    if dtype == 'rgbrgb':            # aux image read as RGB already (cv2: BGR then cvtColor BGR2RGB)
        return np.concatenate([rgb, dp if dp.ndim == 3 else np.repeat(dp[..., None], 3, 2)], axis=2)
    d8 = normalize_minmax_u8(dp if dp.ndim == 2 else dp[..., 0])
    if dtype == 'colormap':
        return apply_colormap_jet(d8)
    if dtype in ('3x', '3xD'):
        return np.stack([d8] * 3, axis=2)
    if dtype in ('normalized_x', 'normalized_depth'):
        return d8
    if dtype == 'rgbcolormap':
        return np.concatenate([rgb, apply_colormap_jet(d8)], axis=2)
    if dtype in ('rgb3x', 'rgb3d'):
        return np.concatenate([rgb, np.stack([d8] * 3, axis=2)], axis=2)
    print('No such dtype !!! ')
    return None


def get_rgbd_frame(color_path, depth_path, dtype='rgbcolormap', depth_clip=False):
    return get_x_frame(color_path, depth_path, dtype=dtype, depth_clip=depth_clip)


def get_rgbd_frame_device(color_path, depth_path, depth_clip=True, device=None):
    """get_rgbd_frame(color, depth, 'rgbcolormap', depth_clip) with the clip / NORM_MINMAX / JET / merge
    done on the GPU (mmtrack_amd.frames.assemble_rgbd): returns the H x W x 6 frame as a CUDA tensor,
    which the tracker reads in place.  Only the decoded RGB (3 B/pixel) and depth (2 B/pixel) cross PCIe."""
    from mmtrack_amd.frames import assemble_rgbd
    rgb = _imread(color_path)
    dp = _imread(depth_path, unchanged=True)
    if dp.ndim == 3:
        dp = dp[..., 0]
    return assemble_rgbd(rgb, dp.astype(np.uint16, copy=False), depth_clip=depth_clip, device=device)



def get_x_frame_device(color_path, aux_path, dtype='rgbrgb', device=None):
    """get_x_frame(color, aux, dtype='rgbrgb') with the merge done on the GPU (mmtrack_amd.frames.merge_rgbx):
    returns the H x W x 6 frame as a CUDA tensor the tracker reads in place (the RGB-T / RGB-E workspace
    path, test_rgbt_mgpus.py:106).  Other dtypes are host-assembled (get_x_frame)."""
    if dtype != 'rgbrgb':
        return get_x_frame(color_path, aux_path, dtype=dtype)
    from mmtrack_amd.frames import merge_rgbx
    return merge_rgbx(_imread(color_path), _imread(aux_path, unchanged=True), device=device)
