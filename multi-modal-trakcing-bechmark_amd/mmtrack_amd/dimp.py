"""DiMP / mfDiMP target-classifier inner loop on the HIP path (mmt_dimp_* in include/mmtrack.h).

Mirrors the reference's operator interface (RGBD/models/DeT/ltr/models/layers/filter.py:5-148 and
ltr/models/target_classifier/optimizer.py:15-170): ``apply_filter``, ``apply_feat_transpose`` and
``DiMPSteepestDescentGN`` with the same argument meaning, on device-resident fp32 tensors.
No CPU fallback: a missing libmmtrack.so raises ImportError and CPU tensors raise ValueError.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib


def _check(t, name, dims):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32):
        raise ValueError(f"{name} must be a float32 CUDA tensor")
    if t.dim() != dims:
        raise ValueError(f"{name} must have {dims} dims, got {tuple(t.shape)}")
    return t.contiguous()


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _rc(rc, what):
    if rc == -1:
        raise ValueError(f"{what}: invalid argument")
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


def apply_filter(feat, filter):
    """feat [I, S, C, H, W], filter [S, C, fh, fw] -> scores [I, S, H', W'] (filter.py:5-54, padding fh//2)."""
    lib = _lib.load()
    feat, filt = _check(feat, "feat", 5), _check(filter, "filter", 4)
    I, S, C, H, W = feat.shape
    fh, fw = filt.shape[-2:]
    if filt.shape[0] != S or filt.shape[1] != C:
        raise ValueError("filter shape does not match feat")
    out = torch.empty(I, S, H + 2 * (fh // 2) - fh + 1, W + 2 * (fw // 2) - fw + 1, device=feat.device)
    _rc(lib.mmt_dimp_apply_filter(feat.data_ptr(), filt.data_ptr(), out.data_ptr(), I, S, C, H, W, fh, fw,
                                  _stream(feat.device)), "mmt_dimp_apply_filter")
    return out


def apply_feat_transpose(feat, input, filter_ksz, training=True):
    """Gradient of sum(input * apply_filter(feat, w)) w.r.t. w -> [S, C, fh, fw] (filter.py:57-148)."""
    lib = _lib.load()
    feat, r = _check(feat, "feat", 5), _check(input, "input", 4)
    I, S, C, H, W = feat.shape
    fh, fw = (filter_ksz, filter_ksz) if isinstance(filter_ksz, int) else tuple(filter_ksz)
    if tuple(r.shape) != (I, S, H + 2 * (fh // 2) - fh + 1, W + 2 * (fw // 2) - fw + 1):
        raise ValueError("input shape does not match feat / filter size")
    out = torch.empty(S, C, fh, fw, device=feat.device)
    _rc(lib.mmt_dimp_feat_transpose(feat.data_ptr(), r.data_ptr(), out.data_ptr(), I, S, C, H, W, fh, fw,
                                    _stream(feat.device)), "mmt_dimp_feat_transpose")
    return out


class DiMPSteepestDescentGN:
    """optimizer.py:15-170 with score_act='relu', act_param=None, mask_act='sigmoid' (DiMP/mfDiMP setting).

    Learnt state comes from the reference module's state_dict (``log_step_length``, ``filter_reg``,
    ``label_map_predictor.weight``, ``target_mask_predictor.0.weight``, ``spatial_weight_predictor.weight``).
    """

    def __init__(self, state_dict, num_iter=1, feat_stride=16, min_filter_reg=1e-3, alpha_eps=0.0,
                 num_dist_bins=10, bin_displacement=0.5, detach_length=float("inf")):
        if num_dist_bins > 128:
            raise ValueError("num_dist_bins must be <= 128")
        self.num_iter = num_iter
        p = _lib.MmtDimpParams()
        p.feat_stride = feat_stride
        p.log_step_length = float(state_dict["log_step_length"].reshape(-1)[0])
        p.filter_reg = float(state_dict["filter_reg"].reshape(-1)[0])
        p.min_filter_reg = min_filter_reg
        p.alpha_eps = alpha_eps
        p.bin_displacement = bin_displacement
        p.num_dist_bins = num_dist_bins
        for field, key in (("label_w", "label_map_predictor.weight"), ("mask_w", "target_mask_predictor.0.weight"),
                           ("spatial_w", "spatial_weight_predictor.weight")):
            v = torch.as_tensor(state_dict[key]).detach().float().reshape(-1).cpu()
            if v.numel() != num_dist_bins:
                raise ValueError(f"{key} has {v.numel()} bins, expected {num_dist_bins}")
            arr = getattr(p, field)
            for k in range(num_dist_bins):
                arr[k] = float(v[k])
        self.params = p
        self._ws = None

    def _workspace(self, dev, nbytes):
        if self._ws is None or self._ws.numel() < nbytes or self._ws.device != dev:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        return self._ws

    def __call__(self, weights, feat, bb, sample_weight=None, num_iter=None, compute_losses=True):
        """Returns (weights, weight_iterates, losses) like optimizer.py:85-170 (losses as a tensor list)."""
        lib = _lib.load()
        num_iter = self.num_iter if num_iter is None else num_iter
        feat = _check(feat, "feat", 5)
        w = _check(weights, "weights", 4).clone()
        I, S, C, H, W = feat.shape
        fh, fw = w.shape[-2:]
        bbh = torch.as_tensor(bb, dtype=torch.float32).detach().cpu().contiguous().reshape(I, S, 4)
        swh = None
        if sample_weight is not None:
            swh = torch.as_tensor(sample_weight, dtype=torch.float32).detach().cpu().contiguous().reshape(I, S)
        nbytes = lib.mmt_dimp_workspace_bytes(I, S, C, H, W, fh, fw, num_iter)
        if nbytes == 0:
            raise ValueError("unsupported DiMP problem shape")
        ws = self._workspace(feat.device, nbytes)
        iterates = [weights]
        losses = []
        # one call per iteration keeps every iterate (the reference returns them all)
        for it in range(num_iter):
            lbuf = (ctypes.c_float * 2)()
            _rc(lib.mmt_dimp_optimize(feat.data_ptr(), I, S, C, H, W, w.data_ptr(), fh, fw, bbh.data_ptr(),
                                      swh.data_ptr() if swh is not None else None, ctypes.byref(self.params), 1,
                                      ws.data_ptr(), nbytes, lbuf if compute_losses else None, _stream(feat.device)),
                "mmt_dimp_optimize")
            if compute_losses:
                losses.append(torch.tensor(lbuf[0]))
                if it == num_iter - 1:
                    losses.append(torch.tensor(lbuf[1]))
            iterates.append(w.clone())
        if num_iter == 0 and compute_losses:
            lbuf = (ctypes.c_float * 1)()
            _rc(lib.mmt_dimp_optimize(feat.data_ptr(), I, S, C, H, W, w.data_ptr(), fh, fw, bbh.data_ptr(),
                                      swh.data_ptr() if swh is not None else None, ctypes.byref(self.params), 0,
                                      ws.data_ptr(), nbytes, lbuf, _stream(feat.device)), "mmt_dimp_optimize")
            losses.append(torch.tensor(lbuf[0]))
        return w, iterates, losses

    def optimize_dev(self, weights, feat, bb_ptr, sw_ptr, num_iter, bb_strides=(-1, -1), sw_strides=(-1, -1)):
        """num_iter steps in place on ``weights`` (a contiguous [S, C, fh, fw] CUDA tensor) over ``feat``
        [I, S, C, H, W] -- any strides on the first two dims, e.g. a DimpPool's memory[a:b, :I].transpose(0, 1)
        -- with the boxes and sample weights at device addresses (the device tracker state), strides in floats
        as (sample, sequence), -1: contiguous [I][S] (0 is a real stride: a broadcast operand); no host staging, no synchronisation (mmt_dimp_optimize_strided)."""
        lib = _lib.load()
        if not (isinstance(feat, torch.Tensor) and feat.is_cuda and feat.dtype == torch.float32 and feat.dim() == 5):
            raise ValueError("feat must be a 5-dim float32 CUDA tensor")
        I, S, C, H, W = feat.shape
        if feat.stride()[2:] != (H * W, W, 1):
            raise ValueError("feat must be contiguous over [C, H, W]")
        if not (weights.is_contiguous() and tuple(weights.shape[:2]) == (S, C)):
            raise ValueError("weights must be a contiguous [S, C, fh, fw] tensor")
        fh, fw = weights.shape[-2:]
        nbytes = lib.mmt_dimp_workspace_bytes(I, S, C, H, W, fh, fw, num_iter)
        if nbytes == 0:
            raise ValueError("unsupported DiMP problem shape")
        ws = self._workspace(feat.device, nbytes)
        _rc(lib.mmt_dimp_optimize_strided(feat.data_ptr(), feat.stride(0), feat.stride(1), I, S, C, H, W,
                                          weights.data_ptr(), fh, fw, ctypes.c_void_p(bb_ptr), bb_strides[0],
                                          bb_strides[1], ctypes.c_void_p(sw_ptr) if sw_ptr else None, sw_strides[0],
                                          sw_strides[1], ctypes.byref(self.params), num_iter, ws.data_ptr(), nbytes,
                                          _stream(feat.device)), "mmt_dimp_optimize_strided")
        return weights

    def optimize(self, weights, feat, bb, sample_weight=None, num_iter=None):
        """All iterations in one call (no per-iterate copies, no host sync): the tracker-side use."""
        lib = _lib.load()
        num_iter = self.num_iter if num_iter is None else num_iter
        feat = _check(feat, "feat", 5)
        w = _check(weights, "weights", 4).clone()
        I, S, C, H, W = feat.shape
        fh, fw = w.shape[-2:]
        bbh = torch.as_tensor(bb, dtype=torch.float32).detach().cpu().contiguous().reshape(I, S, 4)
        swh = None
        if sample_weight is not None:
            swh = torch.as_tensor(sample_weight, dtype=torch.float32).detach().cpu().contiguous().reshape(I, S)
        nbytes = lib.mmt_dimp_workspace_bytes(I, S, C, H, W, fh, fw, num_iter)
        if nbytes == 0:
            raise ValueError("unsupported DiMP problem shape")
        ws = self._workspace(feat.device, nbytes)
        _rc(lib.mmt_dimp_optimize(feat.data_ptr(), I, S, C, H, W, w.data_ptr(), fh, fw, bbh.data_ptr(),
                                  swh.data_ptr() if swh is not None else None, ctypes.byref(self.params), num_iter,
                                  ws.data_ptr(), nbytes, None, _stream(feat.device)), "mmt_dimp_optimize")
        return w
