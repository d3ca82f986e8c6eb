"""SiamFC tracker on the MI355X path (RGBE/models/siamfc; the reference's folder is an empty
submodule, so this follows the published SiamFC tracker -- see oracle/siamfc.py for the restated
algorithm and DESIGN.md §8). Per frame, on the GPU:

  mmt_siamfc_crop (3-scale instance pyramid from the HBM-resident frame, cv2 INTER_LINEAR, mean-colour
  border, NHWC) -> AlexNetV1 backbone (HIP fp32-MFMA implicit-GEMM convs + max-pools, BN folded) ->
  mmt_xcorr_nhwc (HIP correlation, out_scale 1e-3) -> mmt_siamfc_response (x16 INTER_CUBIC, scale penalty, normalise, cosine window,
  argmax) -> 4 floats to the host for the box update (float64, as the reference).

GOT-10k-style tracker interface: ``init(img, box)``, ``update(img) -> box``, ``track(frames, box)``.
No CPU path: frames go to the device and every op raises without the HIP library.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib

MMT_CONV_RELU, MMT_CONV_W4 = 1, 4   # include/mmtrack.h

CFG = dict(out_scale=0.001, exemplar_sz=127, instance_sz=255, context=0.5, scale_num=3, scale_step=1.0375,
           scale_lr=0.59, scale_penalty=0.9745, window_influence=0.176, response_sz=17, response_up=16,
           total_stride=8)


def _rc(rc, what):
    if rc == -1:
        raise ValueError(f"{what}: invalid argument")
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


class AlexNetV1:
    """conv1 11/2 + BN + ReLU + pool3/2, conv2 5 g2 + BN + ReLU + pool, conv3 3, conv4 3 g2, conv5 3 g2 (BN eps 1e-6
    folded into the conv weights at load), on the HIP fp32-MFMA implicit-GEMM conv (``mmt_conv2d_f32_ld``: NHWC, a
    group = channel offsets into pitched rows) and ``mmt_maxpool2d_f32``.  Input: NHWC [n][H][W][3] float (what
    ``mmt_siamfc_crop_nhwc`` writes); output NHWC [n][Ho][Wo][256].  conv1's 96 output channels are zero-padded
    to 128 (the conv kernel's 64-channel tiles; the padded channels are ReLU(0) = 0 and never read by conv2)."""
    LAYERS = [("conv1", 2, 1, True, True), ("conv2", 1, 2, True, True), ("conv3", 1, 1, True, False),
              ("conv4", 1, 2, True, False), ("conv5", 1, 2, False, False)]

    def __init__(self, state_dict, device):
        self.lib = _lib.load()
        self.device = device
        self.layers = []
        cin_pitch = 3
        for li, (name, stride, groups, bn, pool) in enumerate(self.LAYERS):
            w = state_dict[f"backbone.{name}.0.weight"].double()
            b = state_dict[f"backbone.{name}.0.bias"].double()
            if bn:
                p = f"backbone.{name}.1."
                s = state_dict[p + "weight"].double() / torch.sqrt(state_dict[p + "running_var"].double() + 1e-6)
                b = (b - state_dict[p + "running_mean"].double()) * s + state_dict[p + "bias"].double()
                w = w * s.view(-1, 1, 1, 1)
            cout, cin_g, kh, kw = w.shape
            cout_g = cout // groups
            w = w.permute(0, 2, 3, 1).float()          # [Cout][kh][kw][Cin_g]
            flags = MMT_CONV_RELU if bn else 0
            if li == 0:                               # the 3-channel stem: one tap (3 values + 0) per load
                w = F.pad(w, (0, 1))
                flags |= MMT_CONV_W4
            pad_out = -cout_g % 64                    # 64-channel output tiles
            ldy = groups * (cout_g + pad_out)
            gw, gb = [], []
            for g in range(groups):
                wg = w[g * cout_g:(g + 1) * cout_g]
                bg = b[g * cout_g:(g + 1) * cout_g].float()
                if pad_out:
                    wg = torch.cat([wg, wg.new_zeros((pad_out,) + tuple(wg.shape[1:]))])
                    bg = torch.cat([bg, bg.new_zeros(pad_out)])
                gw.append(wg.contiguous().to(device))
                gb.append(bg.contiguous().to(device))
            self.layers.append(dict(w=gw, b=gb, stride=stride, groups=groups, cin_g=cin_g, ldx=cin_pitch,
                                    cout_g=cout_g + pad_out, ldy=ldy, kh=kh, kw=kw, flags=flags, pool=pool))
            cin_pitch = ldy
        self.out_channels = self.layers[-1]["ldy"]
        self._bufs = {}

    def _buffers(self, n, H, W):
        key = (n, H, W)
        if key not in self._bufs:
            bufs = []
            for L in self.layers:
                H = (H - L["kh"]) // L["stride"] + 1
                W = (W - L["kw"]) // L["stride"] + 1
                y = torch.empty(n, H, W, L["ldy"], device=self.device)
                p = None
                if L["pool"]:
                    H, W = (H - 3) // 2 + 1, (W - 3) // 2 + 1
                    p = torch.empty(n, H, W, L["ldy"], device=self.device)
                bufs.append((y, p))
            self._bufs[key] = bufs
        return self._bufs[key]

    def __call__(self, x, stream):
        """x: NHWC [n][H][W][3] float on the device -> NHWC features (a buffer reused by the next call of the
        same shape)."""
        n, H, W, _ = x.shape
        cur = x
        for L, (y, p) in zip(self.layers, self._buffers(n, H, W)):
            for g in range(L["groups"]):
                xo = cur.data_ptr() + 4 * g * L["cin_g"]
                yo = y.data_ptr() + 4 * g * L["cout_g"]
                _rc(self.lib.mmt_conv2d_f32_ld(xo, n, H, W, L["cin_g"], L["ldx"], L["w"][g].data_ptr(),
                                               L["b"][g].data_ptr(), L["cout_g"], L["kh"], L["kw"], L["stride"], 0,
                                               None, yo, L["ldy"], L["flags"], stream), "mmt_conv2d_f32_ld")
            H, W = y.shape[1], y.shape[2]
            cur = y
            if p is not None:
                _rc(self.lib.mmt_maxpool2d_f32(y.data_ptr(), n, H, W, L["ldy"], 3, 2, 0, p.data_ptr(), stream),
                    "mmt_maxpool2d_f32")
                H, W = p.shape[1], p.shape[2]
                cur = p
        return cur


class TrackerSiamFC:
    name = "SiamFC"
    is_deterministic = True

    def __init__(self, net_path=None, state_dict=None, device=None, **kwargs):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("TrackerSiamFC needs an MI355X (HIP device); there is no CPU path")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.cfg = dict(CFG, **kwargs)
        if state_dict is None:
            state_dict = torch.load(net_path, map_location="cpu", weights_only=True)
        state_dict = {k[len("module."):] if k.startswith("module.") else k: v for k, v in state_dict.items()}
        self.backbone = AlexNetV1(state_dict, self.device)
        c = self.cfg
        self.upscale_sz = c["response_up"] * c["response_sz"]
        h = np.hanning(self.upscale_sz)
        self.hann1d = torch.from_numpy(h).to(self.device)
        self.hann_sum = float(np.outer(h, h).sum())
        n = c["scale_num"]
        self.scale_factors = c["scale_step"] ** np.linspace(-(n // 2), n // 2, n)
        self.scratch = torch.empty(n * self.upscale_sz ** 2, device=self.device)
        self.result = torch.empty(4, device=self.device)
        self.xbuf = torch.empty(n, c["instance_sz"], c["instance_sz"], 3, device=self.device)
        self.zbuf = torch.empty(1, c["exemplar_sz"], c["exemplar_sz"], 3, device=self.device)
        self.resp = torch.empty(n, 1, c["response_sz"], c["response_sz"], device=self.device)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _frame(self, img):
        if isinstance(img, torch.Tensor):
            t = img if img.is_cuda else img.to(self.device)
        else:
            t = torch.from_numpy(np.ascontiguousarray(img)).to(self.device, non_blocking=False)
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] < 3:
            raise ValueError("frame must be H x W x C uint8 with C >= 3")
        return t.contiguous()

    def _crop(self, frame, sizes, out_sz, out):
        n = len(sizes)
        y0, x0, side = [], [], []
        for s in sizes:
            s = round(s)
            c0 = np.round(self.center - (s - 1) / 2)
            y0.append(int(np.round(c0[0])))
            x0.append(int(np.round(c0[1])))
            side.append(int(s))
        H, W, C = frame.shape
        arr = lambda v: (ctypes.c_int * len(v))(*v)
        nhwc = out.shape[-1] == 3 and out.shape[1] == out_sz
        fn = self.lib.mmt_siamfc_crop_nhwc if nhwc else self.lib.mmt_siamfc_crop
        _rc(fn(frame.data_ptr(), H, W, C, frame.stride(0), n, arr(y0), arr(x0), arr(side), arr(self.pad), out_sz,
               out.data_ptr(), self._stream()), "mmt_siamfc_crop")
        return out

    def _xcorr(self, z, x):
        """z: the exemplar's NHWC features [1][hz][wz][C] (shared by every scale), x: [n][hx][wx][C]"""
        n, hx, wx, C = x.shape
        hz, wz = z.shape[1:3]
        _rc(self.lib.mmt_xcorr_nhwc(z.data_ptr(), 0, x.data_ptr(), self.resp.data_ptr(), n, C, hz, wz, hx, wx,
                                    ctypes.c_float(self.cfg["out_scale"]), ctypes.c_float(0.0), self._stream()),
            "mmt_xcorr_nhwc")
        return self.resp

    @torch.no_grad()
    def init(self, img, box):
        c = self.cfg
        box = np.array([box[1] - 1 + (box[3] - 1) / 2, box[0] - 1 + (box[2] - 1) / 2, box[3], box[2]],
                       dtype=np.float32)
        self.center, self.target_sz = box[:2], box[2:]
        context = c["context"] * np.sum(self.target_sz)
        self.z_sz = np.sqrt(np.prod(self.target_sz + context))
        self.x_sz = self.z_sz * c["instance_sz"] / c["exemplar_sz"]
        frame = self._frame(img)
        avg = frame[..., :3].double().mean(dim=(0, 1)).cpu().numpy()
        self.avg_color = avg
        self.pad = [int(v) for v in np.clip(np.rint(avg), 0, 255)]
        z = self._crop(frame, [self.z_sz], c["exemplar_sz"], self.zbuf)
        self.kernel = self.backbone(z, self._stream()).clone()   # kept across frames (the buffer is reused)

    @torch.no_grad()
    def update(self, img):
        c = self.cfg
        frame = self._frame(img)
        x = self._crop(frame, [self.x_sz * f for f in self.scale_factors], c["instance_sz"], self.xbuf)
        resp = self._xcorr(self.kernel, self.backbone(x, self._stream()))
        _rc(self.lib.mmt_siamfc_response(resp.data_ptr(), c["scale_num"], c["response_sz"], self.upscale_sz,
                                         ctypes.c_float(c["scale_penalty"]), c["window_influence"],
                                         self.hann1d.data_ptr(), self.hann_sum, self.scratch.data_ptr(),
                                         self.result.data_ptr(), self._stream()), "mmt_siamfc_response")
        sid, ly, lx, _ = self.result.tolist()
        scale_id = int(sid)
        disp_in_response = np.array([ly, lx]) - (self.upscale_sz - 1) / 2
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

    def track(self, frames, box):
        """Whole sequence: frames is a sequence of H x W x C uint8 images; returns (boxes, times)."""
        n = len(frames)
        boxes = np.zeros((n, 4))
        boxes[0] = box
        times = np.zeros(n)
        for f, img in enumerate(frames):
            begin = time.time()
            if f == 0:
                self.init(img, box)
            else:
                boxes[f, :] = self.update(img)
            times[f] = time.time() - begin
        return boxes, times
