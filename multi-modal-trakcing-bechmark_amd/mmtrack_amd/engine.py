"""Python handle on the MI355X tracking engine (C ABI of include/mmtrack.h).

``Engine`` owns one device engine: the ViPT / OSTrack weights in HBM (bf16 GEMM operands, BN
folded into the head convs), ``max_batch`` sequence slots, and the per-frame launch sequence.
It is what the reference-shaped tracker classes (``lib/test/tracker/vipt.py`` etc.) wrap.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np

from . import _lib as L


class TrackerError(Exception):
    pass


@dataclass
class EngineConfig:
    model: str = "vipt"               # "vipt" | "ostrack"
    prompt_type: str = "vipt_deep"    # cfg.TRAIN.PROMPT.TYPE
    in_chans: int = 6
    template_size: int = 128
    search_size: int = 256
    template_factor: float = 2.0
    search_factor: float = 4.0
    ce_loc: List[int] = field(default_factory=lambda: [3, 6, 9])
    ce_keep_ratio: List[float] = field(default_factory=lambda: [0.7, 0.7, 0.7])
    ce_template_range: str = "CTR_POINT"
    head_channels: int = 256
    max_batch: int = 1
    use_graphs: bool = True
    debug_outputs: bool = False
    precision: str = "fp32"           # "fp32": parity mode, f16x3 split products (common.h); "bf16": plain bf16

    @classmethod
    def from_cfg(cls, cfg, **kw):
        """From a reference-layout cfg (lib/config/vipt/config.py + experiments yaml)."""
        backbone = cfg.MODEL.BACKBONE.TYPE
        model = "ostrack" if "prompt" not in backbone else "vipt"
        return cls(model=model, prompt_type=cfg.TRAIN.PROMPT.TYPE if model == "vipt" else "none",
                   in_chans=6 if model == "vipt" else 3, template_size=cfg.TEST.TEMPLATE_SIZE,
                   search_size=cfg.TEST.SEARCH_SIZE, template_factor=cfg.TEST.TEMPLATE_FACTOR,
                   search_factor=cfg.TEST.SEARCH_FACTOR, ce_loc=list(cfg.MODEL.BACKBONE.CE_LOC),
                   ce_keep_ratio=list(cfg.MODEL.BACKBONE.CE_KEEP_RATIO),
                   ce_template_range=cfg.MODEL.BACKBONE.CE_TEMPLATE_RANGE,
                   head_channels=cfg.MODEL.HEAD.NUM_CHANNELS, **kw)

    def ctr_point_index(self) -> int:
        """generate_mask_cond CTR_POINT (ViPT/lib/utils/ce_utils.py:22-35)."""
        tf = self.template_size // 16
        idx = {8: 3, 12: 5, 7: 3, 14: 6}.get(tf)
        if idx is None:
            raise NotImplementedError
        return idx * tf + idx

    def to_c(self) -> L.MmtConfig:
        c = L.MmtConfig()
        c.model = L.MMT_MODEL_VIPT if self.model == "vipt" else L.MMT_MODEL_OSTRACK
        c.prompt_type = {"vipt_deep": L.MMT_PROMPT_DEEP, "vipt_shaw": L.MMT_PROMPT_SHAW}.get(self.prompt_type,
                                                                                        L.MMT_PROMPT_NONE)
        c.in_chans = self.in_chans
        c.template_size = self.template_size
        c.search_size = self.search_size
        c.template_factor = self.template_factor
        c.search_factor = self.search_factor
        if self.ce_loc and self.ce_template_range != "CTR_POINT":
            raise NotImplementedError("only CE_TEMPLATE_RANGE = CTR_POINT is supported")
        c.n_ce = len(self.ce_loc)
        for i, (loc, r) in enumerate(zip(self.ce_loc, self.ce_keep_ratio)):
            c.ce_loc[i] = int(loc)
            c.ce_keep_ratio[i] = float(r)
        c.ce_template_index = self.ctr_point_index() if self.ce_loc else -1
        c.head_channels = self.head_channels
        c.max_batch = self.max_batch
        c.use_graphs = int(self.use_graphs)
        c.debug_outputs = int(self.debug_outputs)
        if self.precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' or 'fp32', got {self.precision!r}")
        c.precision = 0 if self.precision == "bf16" else 1
        return c


def hann_window(feat_sz: int) -> np.ndarray:
    """hann2d(feat_sz) computed with torch exactly as ViPT/lib/test/utils/hann.py:6-16 does."""
    import torch
    h = 0.5 * (1 - torch.cos((2 * math.pi / (feat_sz + 1)) * torch.arange(1, feat_sz + 1).float()))
    return (h.reshape(1, 1, -1, 1) * h.reshape(1, 1, 1, -1)).numpy()


def _frame_arg(frame):
    """(pointer, H, W, C, row_stride, is_device) of a numpy H x W x C uint8 array or a device tensor."""
    if isinstance(frame, np.ndarray):
        if frame.dtype != np.uint8 or frame.ndim != 3:
            raise ValueError("frame must be an H x W x C uint8 array")
        if not (frame.flags.c_contiguous or (frame.strides[2] == 1 and frame.strides[1] == frame.shape[2])):
            frame = np.ascontiguousarray(frame)
        return frame, frame.ctypes.data, frame.shape[0], frame.shape[1], frame.shape[2], frame.strides[0], 0
    # torch tensor on the GPU
    if frame.dtype.__str__() != "torch.uint8" or frame.dim() != 3 or frame.stride(2) != 1:
        raise ValueError("device frame must be an H x W x C uint8 tensor with unit channel stride")
    return frame, frame.data_ptr(), frame.shape[0], frame.shape[1], frame.shape[2], frame.stride(0), int(
        frame.is_cuda)


class Engine:
    def __init__(self, cfg: EngineConfig, state_dict=None, device: int = 0):
        self.lib = L.load()
        self.cfg = cfg
        self.device = device
        h = ctypes.c_void_p()
        c = cfg.to_c()
        rc = self.lib.mmt_create(ctypes.byref(c), device, ctypes.byref(h))
        if rc != L.MMT_OK:
            raise TrackerError(f"mmt_create failed ({rc}) for {cfg}")
        self.h = h
        self._pending = {}
        self.feat_sz = cfg.search_size // 16
        if state_dict is not None:
            self.load_state_dict(state_dict)

    # -- weights (load_state_dict(strict=True) semantics)
    def expected_keys(self) -> List[str]:
        return [self.lib.mmt_expected_key(self.h, i).decode() for i in range(self.lib.mmt_num_expected_keys(self.h))]

    def _check(self, rc):
        if rc == L.MMT_OK:
            return
        msg = self.lib.mmt_last_error(self.h).decode()
        if rc == L.MMT_E_BOX:
            raise Exception(msg)            # processing_utils.py:34-35 raises a bare Exception
        if rc == L.MMT_E_WEIGHTS:
            raise RuntimeError("Error(s) in loading state_dict: " + msg)
        if rc == L.MMT_E_ARG:
            raise ValueError(msg)
        raise TrackerError(f"{msg} (code {rc})")

    def load_state_dict(self, sd, window=None):
        import torch
        for k, v in sd.items():
            t = v.detach().to("cpu", torch.float32).contiguous().numpy() if hasattr(v, "detach") else \
                np.ascontiguousarray(v, dtype=np.float32)
            shape = (ctypes.c_int64 * max(t.ndim, 1))(*t.shape)
            self._check(self.lib.mmt_set_tensor(self.h, k.encode(), t.ctypes.data, shape, t.ndim))
        w = hann_window(self.feat_sz) if window is None else np.ascontiguousarray(window, dtype=np.float32)
        shape = (ctypes.c_int64 * 4)(*w.shape)
        self._check(self.lib.mmt_set_tensor(self.h, b"output_window", w.ctypes.data, shape, 4))
        self._check(self.lib.mmt_finalize(self.h))

    # -- tracking
    def _order_device_frames(self, dev):
        """Device frames are read in place on the engine stream: order it after torch's current stream
        (where the caller produced the frame, e.g. frames.assemble_rgbd / merge_rgbx)."""
        if dev:
            import torch
            s = torch.cuda.current_stream(self.device).cuda_stream
            if s != getattr(self, "_frame_stream", None):
                self._check(self.lib.mmt_set_frame_stream(self.h, ctypes.c_void_p(s)))
                self._frame_stream = s

    def initialize(self, slot: int, image, box: Sequence[float]):
        keep, ptr, H, W, C, stride, dev = _frame_arg(image)
        self._order_device_frames(dev)
        b = (ctypes.c_double * 4)(*[float(v) for v in box])
        self._check(self.lib.mmt_initialize(self.h, slot, ptr, H, W, C, stride, dev, b))

    def track(self, slot: int, image):
        keep, ptr, H, W, C, stride, dev = _frame_arg(image)
        self._order_device_frames(dev)
        out = (ctypes.c_double * 4)()
        sc = ctypes.c_float()
        self._check(self.lib.mmt_track(self.h, slot, ptr, H, W, C, stride, dev, out, ctypes.byref(sc)))
        return [out[0], out[1], out[2], out[3]], float(sc.value)

    def track_batch(self, first_slot: int, frames) -> tuple:
        n = len(frames)
        args = [_frame_arg(f) for f in frames]
        ptrs = (ctypes.c_void_p * n)(*[a[1] for a in args])
        Hs = (ctypes.c_int * n)(*[a[2] for a in args])
        Ws = (ctypes.c_int * n)(*[a[3] for a in args])
        strides = (ctypes.c_int64 * n)(*[a[5] for a in args])
        C = args[0][4]
        dev = args[0][6]
        self._order_device_frames(dev)
        out = (ctypes.c_double * (4 * n))()
        sc = (ctypes.c_float * n)()
        self._check(self.lib.mmt_track_batch(self.h, first_slot, n, ptrs, Hs, Ws, C, strides, dev, out, sc))
        return np.array(out[:], dtype=np.float64).reshape(n, 4), np.array(sc[:], dtype=np.float32)

    # -- pipelined frames: the tracker state lives on the device, so frame t+1 of every sequence can be
    # submitted before frame t's boxes are fetched (include/mmtrack.h, mmt_track_batch_submit)
    def track_batch_submit(self, first_slot: int, frames) -> int:
        n = len(frames)
        args = [_frame_arg(f) for f in frames]
        ptrs = (ctypes.c_void_p * n)(*[a[1] for a in args])
        Hs = (ctypes.c_int * n)(*[a[2] for a in args])
        Ws = (ctypes.c_int * n)(*[a[3] for a in args])
        strides = (ctypes.c_int64 * n)(*[a[5] for a in args])
        ticket = ctypes.c_int64()
        self._order_device_frames(args[0][6])
        self._check(self.lib.mmt_track_batch_submit(self.h, first_slot, n, ptrs, Hs, Ws, args[0][4], strides,
                                                    args[0][6], ctypes.byref(ticket)))
        self._pending[ticket.value] = (n, args)   # keep host frames alive until their copy has run
        return ticket.value

    def track_batch_fetch(self, ticket: int) -> tuple:
        if ticket not in self._pending:
            raise ValueError("unknown or already fetched ticket")
        n, _ = self._pending.pop(ticket)
        out = (ctypes.c_double * (4 * n))()
        sc = (ctypes.c_float * n)()
        self._check(self.lib.mmt_track_batch_fetch(self.h, ticket, out, sc))
        return np.array(out[:], dtype=np.float64).reshape(n, 4), np.array(sc[:], dtype=np.float32)

    def state(self, slot: int):
        out = (ctypes.c_double * 4)()
        self._check(self.lib.mmt_get_state(self.h, slot, out))
        return list(out)

    def set_state(self, slot: int, box):
        b = (ctypes.c_double * 4)(*[float(v) for v in box])
        self._check(self.lib.mmt_set_state(self.h, slot, b))

    # -- parity read-back
    def debug(self, what: str, bi: int = 0) -> np.ndarray:
        S, C, fs = self.cfg.search_size, self.cfg.in_chans, self.feat_sz
        L_ = (self.cfg.template_size // 16) ** 2 + fs * fs
        nce = max(len(self.cfg.ce_loc), 1)
        spec = {"crop": (np.uint8, (S, S, C)), "maps": (np.float32, (5, fs, fs)), "feat": (np.float32, (L_, 768)),
                "removed": (np.int32, (fs * fs,)), "result": (np.float32, (8,)),
                "ce_keys": (np.float32, (nce, fs * fs))}[what]
        out = np.empty(spec[1], dtype=spec[0])
        self._check(self.lib.mmt_debug_fetch(self.h, what.encode(), bi, out.ctypes.data, out.nbytes))
        return out

    def force_ce(self, slot: int, keys=None):
        """Teacher-forced CE (parity diagnosis): keys [n_ce][Lx] by slot id, e.g. the reference's own CE
        scores; None turns forcing off."""
        if keys is None:
            self._check(self.lib.mmt_debug_force_ce(self.h, slot, None, 0))
            return
        k = np.ascontiguousarray(keys, dtype=np.float32)
        self._check(self.lib.mmt_debug_force_ce(self.h, slot, k.ctypes.data, k.size))

    # -- kernel timing probe (bench roofline)
    def timing_enable(self, cls: str | None):
        self._check(self.lib.mmt_timing_enable(self.h, (cls or "").encode()))

    def timing_read(self):
        n = ctypes.c_int()
        ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.mmt_timing_read(self.h, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(fl),
                                             ctypes.byref(by)))
        return {"launches": n.value, "total_ms": ms.value, "flops": fl.value, "bytes": by.value}

    def close(self):
        if getattr(self, "h", None):
            self.lib.mmt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def xcorr(z, x, scale: float = 1.0, bias: float = 0.0, stream=None):
    """SiamFC / DiMP cross-correlation on device tensors (fp32 NCHW): out [B,1,Ho,Wo]."""
    import torch
    lib = L.load()
    B, C, hz, wz = z.shape
    _, _, hx, wx = x.shape
    out = torch.empty((B, 1, hx - hz + 1, wx - wz + 1), device=x.device, dtype=torch.float32)
    s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
    rc = lib.mmt_xcorr(z.data_ptr(), x.data_ptr(), out.data_ptr(), B, C, hz, wz, hx, wx, scale, bias, s)
    if rc != L.MMT_OK:
        raise ValueError(f"mmt_xcorr failed ({rc})")
    return out
