"""Multi-modal frame assembly on the GPU (mmt_rgbd_assemble, mmt_rgbx_merge).

``assemble_rgbd`` is get_rgbd_frame(color, depth, dtype='rgbcolormap', depth_clip=...) of
ViPT/lib/train/dataset/depth_utils.py:7-58 (median-based depth clip, cv2 NORM_MINMAX, JET colormap,
merge) producing the H x W x 6 uint8 frame directly in HBM, where the tracker reads it.
``merge_rgbx`` is get_x_frame(color, aux, dtype='rgbrgb') (depth_utils.py:71-132, the RGB-T / RGB-E
workspaces' call, test_rgbt_mgpus.py:106): the two decoded RGB images merged into the HBM frame.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_WS = {}


def _dev(x, dtype, dev):
    if isinstance(x, torch.Tensor):
        t = x.to(dev) if not x.is_cuda else x
    else:
        t = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    if t.dtype != dtype:
        raise ValueError(f"expected {dtype}, got {t.dtype}")
    return t.contiguous()


def assemble_rgbd(rgb, depth, depth_clip: bool = True, lut_bgr=None, out=None, device=None):
    """rgb: H x W x 3 uint8, depth: H x W uint16 (numpy or CUDA tensors) -> CUDA H x W x 6 uint8."""
    lib = _lib.load()
    if not torch.cuda.is_available():
        raise RuntimeError("assemble_rgbd needs an MI355X (HIP device); there is no CPU path")
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    r = _dev(rgb, torch.uint8, dev)
    if isinstance(depth, np.ndarray):   # uint16 depth travels as its int16 bit pattern
        d = _dev(np.ascontiguousarray(depth.astype(np.uint16, copy=False)).view(np.int16), torch.int16, dev)
    else:
        d = depth.view(torch.int16) if depth.dtype == getattr(torch, "uint16", None) else depth
        d = _dev(d, torch.int16, dev)
    if r.dim() != 3 or r.shape[2] != 3 or d.dim() != 2 or tuple(d.shape) != tuple(r.shape[:2]):
        raise ValueError("rgb must be H x W x 3 and depth H x W")
    H, W = d.shape
    if out is None:
        out = torch.empty(H, W, 6, dtype=torch.uint8, device=dev)
    nbytes = lib.mmt_rgbd_workspace_bytes()
    ws = _WS.get(dev)
    if ws is None:
        ws = _WS[dev] = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    lut = None
    if lut_bgr is not None:
        lut = _dev(np.asarray(lut_bgr, dtype=np.uint8).reshape(256, 3), torch.uint8, dev)
    rc = lib.mmt_rgbd_assemble(r.data_ptr(), r.stride(0), d.data_ptr(), d.stride(0), H, W, int(bool(depth_clip)),
                               lut.data_ptr() if lut is not None else None, out.data_ptr(), out.stride(0),
                               ws.data_ptr(), nbytes, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    if rc == -1:
        raise ValueError("mmt_rgbd_assemble: invalid argument")
    if rc != 0:
        raise RuntimeError(f"mmt_rgbd_assemble failed ({rc})")
    return out


def merge_rgbx(rgb, aux, out=None, device=None):
    """rgb: H x W x 3 uint8, aux: H x W x 3 (or H x W, replicated) uint8 -> CUDA H x W x 6 uint8 frame."""
    lib = _lib.load()
    if not torch.cuda.is_available():
        raise RuntimeError("merge_rgbx needs an MI355X (HIP device); there is no CPU path")
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    r, a = _dev(rgb, torch.uint8, dev), _dev(aux, torch.uint8, dev)
    if r.dim() != 3 or r.shape[2] != 3:
        raise ValueError("rgb must be H x W x 3")
    ach = 1 if a.dim() == 2 else a.shape[2]
    if a.dim() not in (2, 3) or ach not in (1, 3) or tuple(a.shape[:2]) != tuple(r.shape[:2]):
        raise ValueError("aux must be H x W x 3 or H x W with rgb's H x W")
    H, W = r.shape[:2]
    if out is None:
        out = torch.empty(H, W, 6, dtype=torch.uint8, device=dev)
    rc = lib.mmt_rgbx_merge(r.data_ptr(), r.stride(0), a.data_ptr(), a.stride(0), ach, H, W, out.data_ptr(),
                            out.stride(0), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    if rc == -1:
        raise ValueError("mmt_rgbx_merge: invalid argument")
    if rc != 0:
        raise RuntimeError(f"mmt_rgbx_merge failed ({rc})")
    return out
