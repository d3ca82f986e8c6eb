"""Where the HIP DiMP tracker's per-frame search patch departs from a bilinear resample of the frame at the
sample coordinates it reports (GPU diagnostic, not a test): the tracker_dimp.npz sequence, frames 1-6; per frame
the max |HIP patch - numpy restatement| and its location, for the coordinates in the device state."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "multi-modal-trakcing-bechmark_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmtrack_amd import _lib, synth  # noqa: E402
from mmtrack_amd.dimp_tracker import DiMP, parameters  # noqa: E402
from mmtrack_amd.dimpnet import DiMPNet  # noqa: E402


def emulate(img, y0c, x0c, h, w, oh=288, ow=288):
    H, W, C = img.shape
    f32 = np.float32

    def axis(sz, o, n):
        s = f32(sz) / f32(o)
        f = np.maximum(s * (np.arange(o, dtype=f32) + f32(0.5)) - f32(0.5), f32(0))
        i0 = f.astype(np.int64)
        i1 = i0 + (i0 < sz - 1)
        l1 = (f - i0).astype(f32)
        return i0, i1, f32(1) - l1, l1
    ry0, ry1, ly0, ly1 = axis(h, oh, H)
    rx0, rx1, lx0, lx1 = axis(w, ow, W)
    cy = lambda r: np.clip(y0c + r, 0, H - 1)
    cx = lambda q: np.clip(x0c + q, 0, W - 1)
    im = img.astype(f32)
    a = im[cy(ry0)[:, None], cx(rx0)[None, :]]
    b = im[cy(ry0)[:, None], cx(rx1)[None, :]]
    c = im[cy(ry1)[:, None], cx(rx0)[None, :]]
    d = im[cy(ry1)[:, None], cx(rx1)[None, :]]
    t0 = b * lx1[None, :, None] + a * lx0[None, :, None]
    t1 = d * lx1[None, :, None] + c * lx0[None, :, None]
    return (t1 * ly1[:, None, None] + t0 * ly0[:, None, None]).transpose(2, 0, 1)


gd = np.load(os.path.join(REPO, "tests", "golden", "tracker_dimp.npz"))
seed, n, H, W, C, tseed = [int(v) for v in gd["meta"]]
frames, _ = synth.make_frames(seed, n, H, W, C, box=tuple(gd["init_box"]))
g = np.load(os.path.join(REPO, "tests", "golden", "dimp_stages.npz"))
net = DiMPNet(synth.make_dimp_state_dict(0), precision="f16x3")
tr = DiMP(parameters(), net=net)
caps = []
eb = net.extract_backbone
net.extract_backbone = lambda p: (caps.append(p.detach().cpu().numpy()), eb(p))[1]
torch.manual_seed(tseed)
tr.initialize(frames[0], {"init_bbox": list(gd["init_box"])})
for t in range(1, 7):
    tr.track(frames[t])
    pool = tr.pool
    st = _lib.MmtDimpState.from_buffer_copy(bytes(pool.states[tr.slot * pool.sbytes:(tr.slot + 1) * pool.sbytes]
                                                  .cpu().numpy()))
    co = [float(v) for v in st.coords]
    hp = caps[t][0]
    em = emulate(frames[t], int(co[0]), int(co[1]), int(co[2] - co[0]), int(co[3] - co[1]))
    d = np.abs(hp - em)
    k = np.unravel_index(d.argmax(), d.shape)
    rs = g[f"f{t}_patch_sub"][0]
    dr = np.abs(hp[:, ::8, ::8] - rs)
    kr = np.unravel_index(dr.argmax(), dr.shape)
    # the same patch from the neighbouring frames (a stale frame would match one of them)
    others = {u: float(np.abs(hp - emulate(frames[u], int(co[0]), int(co[1]), int(co[2] - co[0]),
                                           int(co[3] - co[1]))).max()) for u in (t - 1, t + 1) if 0 <= u < n}
    print(f"frame {t} coords {co} | HIP vs restatement max {d.max():.4g} at {k} | HIP vs reference (every 8th) "
          f"{dr.max():.4g} at {kr} | vs restatement of frames {others} | ref coords {g[f'f{t}_coords'].tolist()}",
          flush=True)
